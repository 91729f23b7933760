"""Server settings: CLI flag > ``SELKIES_<NAME>`` env > legacy env > default.

Same surface as the reference (``src/selkies/settings.py:36-222``): 56 settings,
kebab-case CLI flags, ``SELKIES_*`` variables, optional legacy variable names,
``true|locked`` booleans, comma lists where the first item is the default and
the list narrows what clients may choose, ``min-max`` ranges (a single number
locks the value), unknown CLI flags ignored (containers pass legacy flags), and
manual-resolution auto-lock. The resolved values feed the ``server_settings``
message the browser client builds its UI from (see :meth:`Settings.client_payload`).

Implementation is ours: every definition is a typed :class:`Spec` object that
parses its own raw string; values are stored as ``Resolved`` tuples that match
the shapes the server code expects (bool -> (value, locked), range -> (lo, hi)).
"""
from __future__ import annotations

import argparse
import logging
import os
from dataclasses import dataclass, field
from typing import Any, Optional, Sequence

log = logging.getLogger("settings")


@dataclass
class Spec:
    name: str
    kind: str                      # bool | enum | list | range | int | str
    default: Any
    help: str = ""
    allowed: Optional[list] = None  # enum / list choices (narrowed by overrides)
    default_value: Optional[int] = None  # range: value used when not locked
    legacy_env: Optional[str] = None

    @property
    def flag(self) -> str:
        return "--" + self.name.replace("_", "-")

    @property
    def env(self) -> str:
        return "SELKIES_" + self.name.upper()

    # -- parsing -----------------------------------------------------------
    def parse(self, raw: Any, overridden: bool):
        if self.kind == "bool":
            text = str(raw).strip().lower()
            base, _, suffix = text.partition("|")
            return (base in ("true", "1", "yes", "on"), suffix == "locked")
        if self.kind in ("enum", "list"):
            master = list(self.allowed or [])
            if overridden:
                items = [x.strip() for x in str(raw).split(",") if x.strip()]
                valid = [x for x in items if x in master]
                if not valid:
                    log.warning("invalid value %r for %s, keeping the default", raw, self.name)
                    valid = [x.strip() for x in str(self.default).split(",") if x.strip() in master]
                self.allowed = valid
            else:
                valid = [x.strip() for x in str(self.default).split(",") if x.strip()]
            if self.kind == "enum":
                return valid[0] if valid else self.default
            return valid
        if self.kind == "int":
            return int(str(raw).strip())
        if self.kind == "str":
            return str(raw)
        if self.kind == "range":
            text = str(raw).strip()
            if "-" in text[1:]:
                lo, hi = text.split("-", 1)
                return (int(lo), int(hi))
            v = int(text)
            return (v, v)
        raise ValueError(f"unknown setting kind {self.kind}")

    def initial(self, value):
        """Value a new session starts with (range: locked value or default_value)."""
        if self.kind == "range":
            lo, hi = value
            return lo if lo == hi else self.default_value
        if self.kind == "bool":
            return value[0]
        return value


def _b(name, default, help_, **kw):
    return Spec(name, "bool", default, help_, **kw)


def _r(name, rng, dv, help_):
    return Spec(name, "range", rng, help_, default_value=dv)


UI_FLAGS = ["video_settings", "screen_settings", "audio_settings", "stats", "clipboard", "files", "apps",
            "sharing", "gamepads", "fullscreen", "gaming_mode", "trackpad", "keyboard_button", "soft_buttons"]


def build_specs() -> list[Spec]:
    specs = [
        _b("audio_enabled", True, "Enable server-to-client audio streaming."),
        _b("microphone_enabled", True, "Enable client-to-server microphone forwarding."),
        _b("gamepad_enabled", True, "Enable gamepad support."),
        _b("clipboard_enabled", True, "Enable clipboard synchronization."),
        _b("command_enabled", True, "Enable parsing of command websocket messages."),
        Spec("file_transfers", "list", "upload,download", "Allowed file transfer directions.",
             allowed=["upload", "download"]),
        Spec("encoder", "enum", "x264enc", "The default video encoder (x265enc: HEVC Main full-frame, "
             "svtav1enc: AV1 Main full-frame; both MI355X-only extensions of the reference's list).",
             allowed=["x264enc", "x264enc-striped", "jpeg", "x265enc", "svtav1enc"]),
        _r("framerate", "8-120", 60, "Allowed framerate range or a fixed value."),
        _r("h264_crf", "5-50", 25, "Allowed H.264 CRF range or a fixed value."),
        _r("h264_bitrate", "0-500000", 0, "H.264 bitrate in kbit/s: 0 = CRF (complexity-adaptive QP around "
           "h264_crf), > 0 = CBR with a 1.5-frame VBV (extension; the reference has CRF only)."),
        _r("jpeg_quality", "1-100", 40, "Allowed JPEG quality range or a fixed value."),
        _b("h264_fullcolor", False, "H.264 full colour range."),
        _b("h264_streaming_mode", False, "H.264 streaming mode (encode every frame)."),
        Spec("h264_aq_strength", "int", 0, "H.264 MB-level adaptive QP strength in 1/16 (16 = x264 aq-strength "
             "1.0; 0 = constant QP like the ultrafast preset)."),
        _b("h264_subpel", True, "H.264 quarter-pel motion refinement (adaptive per stripe)."),
        _b("h264_intra4x4", False, "H.264 Intra4x4 (I_NxN) macroblocks in keyframes: fewer bits on text, "
           "~3x the keyframe encode time."),
        _b("use_cpu", False, "Force the CPU reference encoder instead of the MI355X pipeline."),
        _b("use_paint_over_quality", True, "High-quality paint-over for static regions."),
        _r("paint_over_jpeg_quality", "1-100", 90, "JPEG paint-over quality range or value."),
        _r("h264_paintover_crf", "5-50", 18, "H.264 paint-over CRF range or value."),
        _r("h264_paintover_burst_frames", "1-30", 5, "H.264 paint-over burst frames range or value."),
        _b("second_screen", True, "Enable a second display."),
        Spec("audio_bitrate", "enum", "320000", "The default audio bitrate.",
             allowed=["64000", "128000", "265000", "320000"]),
        _b("is_manual_resolution_mode", False, "Lock the resolution to manual width/height."),
        Spec("manual_width", "int", 0, "Fixed width (forces manual resolution mode)."),
        Spec("manual_height", "int", 0, "Fixed height (forces manual resolution mode)."),
        Spec("scaling_dpi", "enum", "96", "Default DPI for UI scaling.",
             allowed=["96", "120", "144", "168", "192", "216", "240", "264", "288"]),
        _b("enable_binary_clipboard", False, "Allow binary clipboard content (images)."),
        _b("use_browser_cursors", False, "Use browser CSS cursors instead of canvas rendering."),
        _b("use_css_scaling", False, "Client-side CSS scaling instead of HiDPI."),
        Spec("ui_title", "str", "Selkies", "Title in the sidebar."),
        _b("ui_show_logo", True, "Show the logo in the sidebar."),
        _b("ui_show_core_buttons", True, "Show core component buttons."),
        _b("ui_show_sidebar", True, "Show the main sidebar UI."),
        Spec("ui_dashboard", "enum", "selkies", "Dashboard layout (selkies: left sidebar, zinc: right side menu, "
             "wish: top menu bar; the three reference dashboards).", allowed=["selkies", "zinc", "wish"]),
    ]
    specs += [_b(f"ui_sidebar_show_{f}", True, f"Show the {f.replace('_', ' ')} section in the sidebar.")
              for f in UI_FLAGS]
    specs += [
        Spec("port", "int", 8082, "Port of the data websocket server.", legacy_env="CUSTOM_WS_PORT"),
        Spec("dri_node", "str", "", "Render node (kept for compatibility; HIP device selection uses --gpu-id).",
             legacy_env="DRI_NODE"),
        Spec("audio_device_name", "str", "output.monitor", "PulseAudio source for audio capture."),
        Spec("watermark_path", "str", "", "Absolute path of a watermark PNG.", legacy_env="WATERMARK_PNG"),
        Spec("watermark_location", "int", -1, "Watermark location enum (0-6).", legacy_env="WATERMARK_LOCATION"),
        _b("debug", False, "Enable debug logging."),
        _b("enable_sharing", True, "Master toggle for sharing features."),
        _b("enable_collab", True, "Collaborative (read-write) sharing link."),
        _b("enable_shared", True, "View-only sharing links."),
        _b("enable_player2", True, "Gamepad player 2 link."),
        _b("enable_player3", True, "Gamepad player 3 link."),
        _b("enable_player4", True, "Gamepad player 4 link."),
    ]
    return specs


# Settings that are only meaningful to the server and never sent to clients.
SERVER_ONLY = ("port", "dri_node", "debug", "audio_device_name", "watermark_path", "h264_aq_strength", "h264_subpel",
               "h264_intra4x4")


class Settings:
    """Resolved settings; attribute access by setting name."""

    def __init__(self, argv: Optional[Sequence[str]] = None, env: Optional[dict] = None):
        self.specs = build_specs()
        self.by_name = {s.name: s for s in self.specs}
        env = os.environ if env is None else env
        parser = argparse.ArgumentParser(description="Selkies MI355X streaming server", add_help=False)
        for s in self.specs:
            via = f"{s.env}" + (f" or {s.legacy_env}" if s.legacy_env else "")
            parser.add_argument(s.flag, dest=s.name, type=str, default=None, help=f"{s.help} (env {via})")
        args, self.unknown_args = parser.parse_known_args(argv if argv is not None else [])
        self.overridden: dict[str, bool] = {}
        self.values: dict[str, Any] = {}
        for s in self.specs:
            raw = getattr(args, s.name)
            if raw is None:
                raw = env.get(s.env)
            if raw is None and s.legacy_env:
                raw = env.get(s.legacy_env)
            overridden = raw is not None
            self.overridden[s.name] = overridden
            try:
                value = s.parse(raw if overridden else s.default, overridden)
            except (TypeError, ValueError) as e:
                log.error("cannot parse %s=%r (%s); using the default", s.name, raw, e)
                value = s.parse(s.default, False)
            self.values[s.name] = value
        # a manual width/height (or the flag) locks manual resolution mode
        if (self.overridden["manual_width"] or self.overridden["manual_height"]
                or self.values["is_manual_resolution_mode"][0]):
            self.values["is_manual_resolution_mode"] = (True, True)
            if self.values["manual_width"] <= 0:
                self.values["manual_width"] = 1024
            if self.values["manual_height"] <= 0:
                self.values["manual_height"] = 768

    def __getattr__(self, name):
        values = self.__dict__.get("values")
        if values is not None and name in values:
            return values[name]
        raise AttributeError(name)

    def initial(self, name):
        return self.by_name[name].initial(self.values[name])

    def client_payload(self) -> dict:
        """The ``server_settings`` message (wire format of the reference client)."""
        out = {}
        for s in self.specs:
            if s.name in SERVER_ONLY:
                continue
            v = self.values[s.name]
            if s.kind == "bool":
                entry = {"value": v[0], "locked": v[1]}
            else:
                entry = {"value": v}
            if s.kind == "range":
                entry["min"], entry["max"] = v
                if s.default_value is not None:
                    entry["default"] = s.default_value
            elif s.kind in ("enum", "list") and s.allowed is not None:
                entry["allowed"] = list(s.allowed)
            out[s.name] = entry
        return {"type": "server_settings", "settings": out}

    def sanitize(self, name: str, client_value):
        """Clamp/validate a value a client asked for against the server limits."""
        s = self.by_name.get(name)
        if s is None:
            return None
        server = self.values[name]
        if client_value is None:
            return s.initial(server)
        try:
            if s.kind == "range":
                lo, hi = server
                return max(lo, min(int(client_value), hi))
            if s.kind == "enum":
                allowed = s.allowed or []
                if str(client_value) in allowed:
                    return client_value
                return allowed[0] if allowed else s.default
            if s.kind == "bool":
                val, locked = server
                want = str(client_value).lower() in ("true", "1")
                return val if locked else want
        except (TypeError, ValueError):
            return s.default_value if s.default_value is not None else s.default
        return client_value

    def as_dict(self) -> dict:
        return dict(self.values)


def configure_logging(settings: Settings):
    level = logging.DEBUG if settings.debug[0] else logging.INFO
    logging.getLogger().setLevel(level)
    for noisy in ("aiohttp.access", "websockets"):
        logging.getLogger(noisy).setLevel(logging.WARNING)
