"""Legacy WebRTC streaming mode: signalling + one WebRTC peer per browser.

Reference: legacy/webrtc.py (main, ~45 ``SELKIES_*`` flags with a JSON overlay
file, RTC-config sources, the signalling retry loop, app-ready wait, metrics,
start/stop hooks) and legacy/gstwebrtc_app.py (webrtcbin pipeline, the "input"
data channel, the server→client JSON messages). SURVEY C19/C20/C23/C25.

MI355X path: the GStreamer element chain (ximagesrc → convert → encoder →
rtph264pay → webrtcbin) is replaced by the native capture session (X11 SHM →
HIP convert/damage/H.264 in full-frame mode, csrc/runtime/capture.cpp) feeding
:class:`~selkies_gstreamer_amd.webrtc.peer.PeerConnection`, whose per-frame
RTP packetisation + SRTP is C++ (csrc/rtc). Bitrate requests (``vb``, REMB) set
the encoder's CBR target at runtime (``ScreenCapture.set_rate``: the native K10
controller, csrc/codec/ratecontrol.h, runs the VBV loop); PLI/FIR and new sessions
force an IDR.

    python -m selkies_gstreamer_amd.legacy.webrtc_app --port 8080 --web_root selkies_gstreamer_amd/web
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import subprocess
import sys
import time
from typing import Optional

from selkies_gstreamer_amd.server import display as display_mod
from selkies_gstreamer_amd.server import stats as stats_mod
from selkies_gstreamer_amd.server.turn import parse_rtc_config, rtc_config, legacy_rtc_config
from selkies_gstreamer_amd.webrtc.turn_client import parse_turn_url
from selkies_gstreamer_amd.webrtc.peer import PeerConnection

from .signalling import SignallingServer
from .signalling_client import SignallingClient, SignallingError

log = logging.getLogger("webrtc_app")

WEB_ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "web")

# (flag, env, default, help) — names and defaults follow legacy/webrtc.py:330-521
FLAGS = [
    ("json_config", "SELKIES_JSON_CONFIG", "/tmp/selkies_config.json", "JSON overlay of argument values (writable)"),
    ("addr", "SELKIES_ADDR", "0.0.0.0", "signalling / web server host"),
    ("port", "SELKIES_PORT", "8080", "signalling / web server port"),
    ("web_root", "SELKIES_WEB_ROOT", WEB_ROOT, "directory with the web client"),
    ("enable_https", "SELKIES_ENABLE_HTTPS", "false", "serve HTTPS"),
    ("https_cert", "SELKIES_HTTPS_CERT", "/etc/ssl/certs/ssl-cert-snakeoil.pem", "TLS certificate"),
    ("https_key", "SELKIES_HTTPS_KEY", "/etc/ssl/private/ssl-cert-snakeoil.key", "TLS private key"),
    ("enable_basic_auth", "SELKIES_ENABLE_BASIC_AUTH", "true", "basic authentication"),
    ("basic_auth_user", "SELKIES_BASIC_AUTH_USER", os.environ.get("USER", ""), "basic auth user"),
    ("basic_auth_password", "SELKIES_BASIC_AUTH_PASSWORD", "mypasswd", "basic auth password"),
    ("rtc_config_json", "SELKIES_RTC_CONFIG_JSON", "/tmp/rtc.json", "RTC config JSON file (overrides STUN/TURN)"),
    ("turn_rest_uri", "SELKIES_TURN_REST_URI", "", "TURN REST API URI"),
    ("turn_rest_username", "SELKIES_TURN_REST_USERNAME", "selkies", "TURN REST user"),
    ("turn_rest_username_auth_header", "SELKIES_TURN_REST_USERNAME_AUTH_HEADER", "x-auth-user", "user header"),
    ("turn_rest_protocol_header", "SELKIES_TURN_REST_PROTOCOL_HEADER", "x-turn-protocol", "protocol header"),
    ("turn_rest_tls_header", "SELKIES_TURN_REST_TLS_HEADER", "x-turn-tls", "TLS header"),
    ("turn_host", "SELKIES_TURN_HOST", "staticauth.openrelay.metered.ca", "TURN host"),
    ("turn_port", "SELKIES_TURN_PORT", "443", "TURN port"),
    ("turn_protocol", "SELKIES_TURN_PROTOCOL", "udp", "TURN protocol (udp/tcp)"),
    ("turn_tls", "SELKIES_TURN_TLS", "false", "TURN over (D)TLS"),
    ("turn_shared_secret", "SELKIES_TURN_SHARED_SECRET", "openrelayprojectsecret", "TURN HMAC secret"),
    ("turn_username", "SELKIES_TURN_USERNAME", "", "long-term TURN user"),
    ("turn_password", "SELKIES_TURN_PASSWORD", "", "long-term TURN password"),
    ("stun_host", "SELKIES_STUN_HOST", "stun.l.google.com", "STUN host"),
    ("stun_port", "SELKIES_STUN_PORT", "19302", "STUN port"),
    ("ice_transport_policy", "SELKIES_ICE_TRANSPORT_POLICY", "all",
     "all: host/srflx/relay candidates; relay: only the TURN relay candidate (server behind a UDP-blocking NAT)"),
    ("enable_cloudflare_turn", "SELKIES_ENABLE_CLOUDFLARE_TURN", "false", "Cloudflare TURN (needs network)"),
    ("cloudflare_turn_token_id", "SELKIES_CLOUDFLARE_TURN_TOKEN_ID", "", "Cloudflare token id"),
    ("cloudflare_turn_api_token", "SELKIES_CLOUDFLARE_TURN_API_TOKEN", "", "Cloudflare API token"),
    ("app_wait_ready", "SELKIES_APP_WAIT_READY", "false", "wait for --app_ready_file before streaming"),
    ("app_ready_file", "SELKIES_APP_READY_FILE", "/tmp/selkies-appready", "app-ready marker file"),
    ("uinput_mouse_socket", "SELKIES_UINPUT_MOUSE_SOCKET", "", "uinput mouse socket path"),
    ("js_socket_path", "SELKIES_JS_SOCKET_PATH", "/tmp", "joystick interposer socket directory"),
    ("encoder", "SELKIES_ENCODER", "x264enc",
     "video encoder (H.264 names map to the HIP H.264 encoder, x265enc/nvh265enc/vah265enc to HIP HEVC, "
     "av1enc/svtav1enc/rav1enc/nvav1enc/vaav1enc to HIP AV1)"),
    ("gpu_id", "SELKIES_GPU_ID", "0", "GPU ordinal"),
    ("framerate", "SELKIES_FRAMERATE", "60", "frames per second"),
    ("video_bitrate", "SELKIES_VIDEO_BITRATE", "8000", "video bitrate (kbit/s)"),
    ("keyframe_distance", "SELKIES_KEYFRAME_DISTANCE", "-1", "seconds between keyframes (-1: infinite)"),
    ("congestion_control", "SELKIES_CONGESTION_CONTROL", "false", "follow REMB bandwidth estimates"),
    ("video_packetloss_percent", "SELKIES_VIDEO_PACKETLOSS_PERCENT", "0",
     "expected video packet loss (percent): > 0 adds RED + ULPFEC with that much redundancy (NACK still active)"),
    ("audio_bitrate", "SELKIES_AUDIO_BITRATE", "128000", "audio bitrate (bit/s)"),
    ("audio_channels", "SELKIES_AUDIO_CHANNELS", "2", "audio channels"),
    ("audio_packetloss_percent", "SELKIES_AUDIO_PACKETLOSS_PERCENT", "0", "audio FEC (Opus in-band)"),
    ("enable_clipboard", "SELKIES_ENABLE_CLIPBOARD", "true", "clipboard: true/false/in/out"),
    ("enable_resize", "SELKIES_ENABLE_RESIZE", "false", "resize the desktop to the browser window"),
    ("enable_cursors", "SELKIES_ENABLE_CURSORS", "true", "send remote cursors"),
    ("debug_cursors", "SELKIES_DEBUG_CURSORS", "false", "cursor debug logging"),
    ("cursor_size", "SELKIES_CURSOR_SIZE", os.environ.get("XCURSOR_SIZE", "-1"), "cursor size"),
    ("enable_webrtc_statistics", "SELKIES_ENABLE_WEBRTC_STATISTICS", "false", "dump client stats as CSV"),
    ("webrtc_statistics_dir", "SELKIES_WEBRTC_STATISTICS_DIR", "/tmp", "CSV directory"),
    ("enable_metrics_http", "SELKIES_ENABLE_METRICS_HTTP", "false", "Prometheus metrics server"),
    ("metrics_http_port", "SELKIES_METRICS_HTTP_PORT", "8000", "Prometheus metrics port"),
    ("start_after_connect", "SELKIES_START_AFTER_CONNECT", "", "command after the first client connects"),
    ("start_after_disconnect", "SELKIES_START_AFTER_DISCONNECT", "", "command after the last client leaves"),
    ("capture_source", "SELKIES_CAPTURE_SOURCE", "auto", "auto / x11 / synthetic (headless nodes, tests)"),
    ("use_cpu", "SELKIES_USE_CPU", "false", "CPU reference encoder instead of the HIP one"),
    ("initial_resolution", "SELKIES_INITIAL_RESOLUTION", "1920x1080", "capture size until the client resizes"),
    ("video_pipeline", "SELKIES_VIDEO_PIPELINE", "",
     "GStreamer launch string (ximagesrc ! ... ! x264enc ... ! rtph264pay); mapped onto the HIP engine"),
]
# values the client may change at runtime and that persist in the JSON overlay
PERSISTED = ("framerate", "video_bitrate", "audio_bitrate", "enable_resize", "encoder")


def _truthy(v) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def parse_args(argv=None, env=None) -> argparse.Namespace:
    env = os.environ if env is None else env
    ap = argparse.ArgumentParser(description="selkies legacy WebRTC mode (MI355X encoder)")
    for name, var, default, helptext in FLAGS:
        ap.add_argument(f"--{name}", default=env.get(var, default), help=helptext)
    ap.add_argument("--debug", action="store_true", help="debug logging")
    args = ap.parse_args(argv)
    overlay = load_overlay(args.json_config)
    explicit = {a.split("=")[0].lstrip("-") for a in (argv or []) if a.startswith("--")}
    for k, v in overlay.items():
        if k in PERSISTED and k not in explicit and not env.get(f"SELKIES_{k.upper()}"):
            setattr(args, k, str(v))
    if args.video_pipeline:
        from .pipeline import apply_to_args, parse_pipeline
        apply_to_args(parse_pipeline(args.video_pipeline), args)
    return args


def load_overlay(path: str) -> dict:
    try:
        with open(path) as f:
            d = json.load(f)
        return d if isinstance(d, dict) else {}
    except (OSError, ValueError):
        return {}


def save_overlay(path: str, args: argparse.Namespace) -> None:
    d = load_overlay(path)
    d.update({k: getattr(args, k) for k in PERSISTED})
    try:
        with open(path, "w") as f:
            json.dump(d, f, indent=1)
    except OSError as e:
        log.debug("cannot write %s: %s", path, e)


def ice_servers_from_rtc(cfg: dict) -> tuple:
    """(stun (host, port) | None, turn (host, port, user, password) | None) for the
    server's own ICE agent from an RTCConfiguration dict: the first STUN server and the
    first UDP TURN server (webrtcbin's stun-server / turn-server, gstwebrtc_app.py:149-197)."""
    try:
        stun_urls, turn_urls, _ = parse_rtc_config(cfg)
    except ValueError:
        return None, None
    stun_srv = None
    for u in stun_urls:
        host, _, port = u.split(":", 1)[1].partition(":")
        stun_srv = (host, int(port or 3478))
        break
    turn_srv = None
    for u in turn_urls:
        turn_srv = parse_turn_url(u)
        if turn_srv:
            break
    return stun_srv, turn_srv


def build_rtc_config(args) -> dict:
    """RTC configuration for the browser (and the server's own STUN lookup)."""
    if args.rtc_config_json and os.path.exists(args.rtc_config_json):
        try:
            with open(args.rtc_config_json) as f:
                stun, turn, cfg = parse_rtc_config(f.read())
            return cfg
        except (OSError, ValueError) as e:
            log.warning("bad RTC config %s: %s", args.rtc_config_json, e)
    if args.turn_username and args.turn_password:
        return legacy_rtc_config(args.turn_host, args.turn_port, args.turn_username, args.turn_password,
                                 args.turn_protocol, _truthy(args.turn_tls), args.stun_host, args.stun_port)
    if args.turn_shared_secret and args.turn_host:
        return rtc_config(args.turn_host, args.turn_port, args.turn_shared_secret, args.turn_rest_username,
                          args.turn_protocol, _truthy(args.turn_tls), args.stun_host, args.stun_port)
    return {"iceServers": [{"urls": [f"stun:{args.stun_host}:{args.stun_port}"]}]}


class StreamSession:
    """One browser peer. media="video" (the reference's uid 0 -> 1 call): capture ->
    H.264 / H.265 / AV1 -> RTP, data-channel input and telemetry; media="audio" (uid 2 ->
    3, webrtc.py:554-557, 581, 720-722): the Opus pipeline alone on its own connection;
    media="both": one connection carrying everything."""

    def __init__(self, args, send_sdp, send_ice, input_factory=None, addresses=None, media: str = "both",
                 peers: Optional[dict] = None):
        self.args = args
        self.media = media
        self.peers = peers if peers is not None else {}   # media -> live session (ab, on the video peer)
        from selkies_gstreamer_amd.legacy.pipeline import AV1_ENCODERS, H265_ENCODERS
        self.hevc = str(getattr(args, "encoder", "")) in H265_ENCODERS
        self.av1 = str(getattr(args, "encoder", "")) in AV1_ENCODERS
        self.send_sdp, self.send_ice = send_sdp, send_ice
        self.fps = int(args.framerate)
        self.target_bps = max(100_000, int(args.video_bitrate) * 1000)   # CBR target of the encoder
        stun_srv, turn_srv = ice_servers_from_rtc(build_rtc_config(args))
        self.pc = PeerConnection(addresses=addresses, video=media != "audio", audio=media != "video",
                                 data=media != "audio",
                                 video_codec="H265" if self.hevc else ("AV1" if self.av1 else "H264"),
                                 stun_server=stun_srv,
                                 turn_server=turn_srv,
                                 fec_percentage=int(float(getattr(args, "video_packetloss_percent", 0) or 0)),
                                 relay_only=str(getattr(args, "ice_transport_policy", "all")) == "relay")
        self.channel = None
        self.capture = None
        self.audio = None
        self._input_factory = input_factory
        self.input = None
        self.loop: Optional[asyncio.AbstractEventLoop] = None
        self.frames_sent = 0
        self.bytes_sent = 0
        self.client_fps = 0
        self.client_latency = 0
        self.ping_sent: Optional[float] = None
        self.latency_ms: Optional[float] = None
        self._tasks: list = []
        self._t0 = time.monotonic()
        self._audio_ts = 0
        self.closed = asyncio.Event()
        self.width, self.height = (int(v) for v in args.initial_resolution.lower().split("x"))

    # -- negotiation ------------------------------------------------------------------------
    async def start(self) -> None:
        self.loop = asyncio.get_running_loop()
        if self._input_factory is not None:
            self.input = await self._input_factory(self)
        self.pc.on_keyframe_request = self._keyframe
        self.pc.on_bitrate = self._on_remb
        self.pc.on_state = self._on_state
        offer = await self.pc.create_offer()
        await self.send_sdp("offer", offer)
        self.peers[self.media] = self
        if self.media == "audio":
            return
        self.channel = self.pc.create_data_channel("input")
        self.channel.on_message = lambda m: asyncio.ensure_future(self.on_message(m)) if isinstance(m, str) else None
        self.channel.on_open = self._on_channel_open

    async def on_remote_sdp(self, kind: str, text: str) -> None:
        await self.pc.set_remote_description(text, kind)
        self._tasks.append(asyncio.ensure_future(self._connect()))

    def on_remote_ice(self, candidate: Optional[str]) -> None:
        if self.pc.ice is not None:
            self.pc.add_ice_candidate(candidate)

    async def _connect(self) -> None:
        try:
            await self.pc.connect(30)
        except Exception as e:
            log.error("WebRTC connection failed: %s", e)
            await self.stop()
            return
        await self._start_media()

    def _on_state(self, st: str) -> None:
        log.info("peer connection %s", st)
        if st in ("failed", "closed") and self.loop:
            self.loop.call_soon(lambda: asyncio.ensure_future(self.stop()))

    # -- media --------------------------------------------------------------------------------
    async def _start_media(self) -> None:
        if self.media == "audio":
            self._tasks.append(asyncio.ensure_future(self._start_audio()))
            return
        import pixelflux
        src = {"x11": 0, "synthetic": 2}.get(self.args.capture_source, -1)
        w, h = self.width, self.height
        s = pixelflux.default_settings(w, h, target_fps=float(self.fps), h264_fullframe=1,
                                       output_mode=pixelflux.OUTPUT_MODE_HEVC if self.hevc else
                                       (pixelflux.OUTPUT_MODE_AV1 if self.av1 else pixelflux.OUTPUT_MODE_H264),
                                       # K10 in the encoder: CBR with a 1.5-frame VBV (gstwebrtc_app.py:101-105),
                                       # starting from the reference's default CRF / paint-over CRF
                                       h264_crf=25, h264_paintover_crf=18,
                                       h264_rc_mode=2, h264_bitrate_kbps=max(1, self.target_bps // 1000),
                                       use_cpu=1 if _truthy(self.args.use_cpu) else 0, source=src,
                                       # x264enc speed-preset=ultrafast (gstwebrtc_app.py:637) on
                                       # the CPU: diamond search, integer-pel vectors
                                       h264_me_full=-1 if _truthy(self.args.use_cpu) else 0,
                                       h264_subpel=-1 if _truthy(self.args.use_cpu) else 0,
                                       device=int(self.args.gpu_id), stripe_height=64,
                                       capture_cursor=0 if _truthy(self.args.enable_cursors) else 1)
        self.capture = pixelflux.ScreenCapture()
        loop = self.loop

        def on_stripe(res_ptr, user):
            r = res_ptr.contents
            data = bytes(r.data[:r.size])
            loop.call_soon_threadsafe(self._on_packet, data)

        self._stripe_cb = pixelflux.StripeCallback(on_stripe)
        await loop.run_in_executor(None, self.capture.start_capture, s, self._stripe_cb)
        self._tasks.append(asyncio.ensure_future(self._telemetry_loop()))
        if self.media == "both":
            self._tasks.append(asyncio.ensure_future(self._start_audio()))
        kd = int(self.args.keyframe_distance)
        if kd > 0:
            self._tasks.append(asyncio.ensure_future(self._keyframe_loop(kd)))

    def _on_packet(self, data: bytes) -> None:
        if len(data) < 10 or data[0] != 0x04:
            return
        key = data[1] == 1
        ts = int((time.monotonic() - self._t0) * 90000)
        self.pc.send_video(data[10:], ts)
        self.frames_sent += 1
        self.bytes_sent += len(data) - 10

    def _apply_rate(self) -> None:
        """Current target (vb, / REMB) -> the encoder's CBR budget from its next frame."""
        if self.capture is not None:
            self.capture.set_rate("cbr", max(1, self.target_bps // 1000))

    async def _start_audio(self) -> None:
        from selkies_gstreamer_amd.server.audio import AudioPipeline

        async def send(pkt: bytes):
            self.pc.send_audio(pkt[2:], self._audio_ts)
            self._audio_ts = (self._audio_ts + 960) & 0xFFFFFFFF
        self.audio = AudioPipeline(send, os.environ.get("SELKIES_AUDIO_DEVICE_NAME", "output.monitor"),
                                   int(self.args.audio_channels))
        if not await self.audio.start(int(self.args.audio_bitrate)):
            self.audio = None

    async def restart_audio(self) -> None:
        """New Opus bitrate: the running audio pipeline is rebuilt at args.audio_bitrate."""
        if self.audio is not None:
            aud, self.audio = self.audio, None
            await aud.stop()
            await self._start_audio()

    def _keyframe(self) -> None:
        if self.capture is not None:
            self.capture.request_keyframe()

    async def _keyframe_loop(self, seconds: int) -> None:
        while True:
            await asyncio.sleep(seconds)
            self._keyframe()

    def _on_remb(self, bps: int) -> None:
        if _truthy(self.args.congestion_control):
            self.target_bps = max(100_000, min(bps, int(self.args.video_bitrate) * 1000))
            self._apply_rate()

    # -- data channel ------------------------------------------------------------------------------
    def send_message(self, msg_type: str, data) -> None:
        """{"type": ..., "data": ...} like gstwebrtc_app.__send_data_channel_message (1481-1496)."""
        if self.channel is None or self.channel.ready_state != "open":
            return
        self.channel.send(json.dumps({"type": msg_type, "data": data}))

    def _on_channel_open(self) -> None:
        self.send_message("system", {"action": f"framerate,{self.fps}"})
        self.send_message("system", {"action": f"video_bitrate,{int(self.args.video_bitrate)}"})
        self.send_message("system", {"action": f"audio_bitrate,{int(self.args.audio_bitrate)}"})
        self.send_message("system", {"action": f"encoder,{self.args.encoder}"})
        self.send_message("system", {"action": f"resize,{str(_truthy(self.args.enable_resize)).lower()}"})
        self.send_message("system", {"action": f"resolution,{self.width}x{self.height}"})

    async def on_message(self, msg: str) -> None:
        toks = msg.split(",")
        t = toks[0]
        try:
            if t == "vb":
                kbps = int(toks[1])
                self.args.video_bitrate = str(kbps)
                self.target_bps = max(100_000, kbps * 1000)
                self._apply_rate()
                self.send_message("pipeline", {"status": f"Video bitrate set to: {kbps}"})
                save_overlay(self.args.json_config, self.args)
            elif t == "ab":
                self.args.audio_bitrate = str(int(toks[1]))
                aud = self.peers.get("audio", self) if self.media == "video" else self
                await aud.restart_audio()   # the Opus encoder takes the new rate (audio peer's pipeline)
                self.send_message("pipeline", {"status": f"Audio bitrate set to: {int(toks[1])}"})
                save_overlay(self.args.json_config, self.args)
            elif t == "_arg_fps":
                self.fps = int(toks[1])
                self.args.framerate = str(self.fps)
                save_overlay(self.args.json_config, self.args)
                self.send_message("system", {"action": f"framerate,{self.fps}"})
            elif t == "r":
                await self._resize(toks[1])
            elif t == "s":
                dpi = int(96 * float(toks[1]))
                await display_mod.set_dpi(dpi)
            elif t == "pong":
                if self.ping_sent is not None:
                    self.latency_ms = (time.time() - self.ping_sent) * 1000.0 / 2
                    self.send_message("latency_measurement", {"latency_ms": round(self.latency_ms, 1)})
            elif t == "_f":
                self.client_fps = int(toks[1])
            elif t == "_l":
                self.client_latency = int(toks[1])
            elif t in ("_stats_video", "_stats_audio"):
                self._dump_stats(t, ",".join(toks[1:]))
            elif self.input is not None:
                await self.input.on_message(msg)
        except (ValueError, IndexError) as e:
            log.warning("bad data channel message %r: %s", msg[:80], e)

    async def _resize(self, res: str) -> None:
        if not _truthy(self.args.enable_resize):
            return
        w, h = (int(v) for v in res.lower().split("x"))
        w, h = display_mod.fit_resolution(w - w % 2, h - h % 2)
        xr = display_mod.XrandrDisplay()
        if xr.available:
            await xr.apply({"primary": {"x": 0, "y": 0, "w": w, "h": h}}, w, h)
        self.width, self.height = w, h
        if self.capture is not None:   # restart capture at the new size, new IDR
            cap, self.capture = self.capture, None
            await self.loop.run_in_executor(None, cap.stop_capture)
            cap.close()
            await self._start_media_size_only()
        self.send_message("system", {"action": f"resolution,{w}x{h}"})

    async def _start_media_size_only(self) -> None:
        for t in self._tasks:
            t.cancel()
        self._tasks.clear()
        await self._start_media()

    def _dump_stats(self, kind: str, payload: str) -> None:
        if not _truthy(self.args.enable_webrtc_statistics):
            return
        from selkies_gstreamer_amd.server.metrics import Metrics
        name = "video" if kind == "_stats_video" else "audio"
        path = os.path.join(self.args.webrtc_statistics_dir, f"selkies-stats-{name}-{int(self._t0)}.csv")
        Metrics(csv_path=path).set_webrtc_stats(kind, payload)

    async def _telemetry_loop(self) -> None:
        n = 0
        while True:
            await asyncio.sleep(1.0)
            n += 1
            st = stats_mod.system_stats()
            self.send_message("system_stats", {"cpu_percent": st.get("cpu_percent"),
                                               "mem_total": st.get("mem_total"), "mem_used": st.get("mem_used")})
            g = stats_mod.gpu_stats(int(self.args.gpu_id))
            if g:
                self.send_message("gpu_stats", {"load": g.get("load"), "memory_total": g.get("memory_total"),
                                                "memory_used": g.get("memory_used")})
            if n % 5 == 0:
                self.ping_sent = time.time()
                self.send_message("ping", {"start_time": round(self.ping_sent, 3)})

    async def stop(self) -> None:
        if self.closed.is_set():
            return
        self.closed.set()
        if self.peers.get(self.media) is self:
            del self.peers[self.media]
        for t in self._tasks:
            t.cancel()
        if self.audio is not None:
            await self.audio.stop()
        if self.input is not None:
            await self.input.close()
        if self.capture is not None:
            cap, self.capture = self.capture, None
            await asyncio.get_running_loop().run_in_executor(None, cap.stop_capture)
            cap.close()
        await self.pc.close()


def _run_hook(cmd: str) -> None:
    if cmd:
        try:
            subprocess.Popen(cmd, shell=True)
        except OSError as e:
            log.warning("hook %r failed: %s", cmd, e)


async def serve(args, input_factory=None, addresses=None, stop: Optional[asyncio.Event] = None) -> None:
    """Signalling server + the streaming peers calling the browser in loops: video and input
    (uid 0 -> 1) and audio (uid 2 -> 3)."""
    if _truthy(args.app_wait_ready):
        while not os.path.exists(args.app_ready_file):
            await asyncio.sleep(0.2)
    rtc = build_rtc_config(args)
    server = SignallingServer(addr=args.addr, port=int(args.port), web_root=args.web_root,
                              enable_basic_auth=_truthy(args.enable_basic_auth) and bool(args.basic_auth_password),
                              basic_auth_user=args.basic_auth_user, basic_auth_password=args.basic_auth_password,
                              turn_shared_secret=args.turn_shared_secret, turn_host=args.turn_host,
                              turn_port=args.turn_port, turn_protocol=args.turn_protocol,
                              turn_tls=_truthy(args.turn_tls), stun_host=args.stun_host, stun_port=args.stun_port,
                              rtc_config_json=args.rtc_config_json if os.path.exists(args.rtc_config_json) else None,
                              https_cert=args.https_cert if _truthy(args.enable_https) else None,
                              https_key=args.https_key if _truthy(args.enable_https) else None)
    port = await server.start()
    args.port = str(port)
    log.info("signalling + web on %s:%d (rtc config: %d ice servers)", args.addr, port,
             len(rtc.get("iceServers", [])))
    if _truthy(args.enable_metrics_http):
        await _start_metrics(int(args.metrics_http_port))
    stop = stop or asyncio.Event()
    scheme = "wss" if _truthy(args.enable_https) else "ws"
    auth = (args.basic_auth_user, args.basic_auth_password) if (_truthy(args.enable_basic_auth) and
                                                               args.basic_auth_password) else None
    url = f"{scheme}://127.0.0.1:{port}/ws"
    peers: dict = {}

    async def loop(my_id, peer_id, media):
        while not stop.is_set():
            await _one_session(url, args, auth, input_factory, addresses, stop, my_id, peer_id, media, peers)
    try:
        # two calls like the reference: video + input (0 -> 1) and audio (2 -> 3)
        await asyncio.gather(loop(0, 1, "video"), loop(2, 3, "audio"))
    finally:
        await server.stop()


async def _one_session(url, args, auth, input_factory, addresses, stop, my_id=0, peer_id=1, media="both",
                       peers=None) -> None:
    sig = SignallingClient(url, my_id, basic_auth=auth, ssl=False)
    await sig.connect()
    session: dict = {}
    done = asyncio.Event()

    async def send_sdp(kind, text):
        await sig.send_sdp(kind, text)

    async def send_ice(idx, cand):
        await sig.send_ice(idx, cand)

    async def start_session():
        s = StreamSession(args, send_sdp, send_ice, input_factory if media != "audio" else None, addresses,
                          media=media, peers=peers)
        session["s"] = s
        if media != "audio":
            _run_hook(args.start_after_connect)
        await s.start()
        await s.closed.wait()
        done.set()

    def on_error(e):
        if "not found" in str(e) or "busy" in str(e):
            async def retry():
                await asyncio.sleep(1.0)
                if not done.is_set() and "s" not in session:
                    await sig.setup_call(peer_id)
            asyncio.ensure_future(retry())
        else:
            log.error("signalling: %s", e)

    sig.on_connect = lambda: asyncio.ensure_future(sig.setup_call(peer_id))
    sig.on_session = lambda meta: asyncio.ensure_future(start_session())
    sig.on_sdp = lambda kind, text: asyncio.ensure_future(session["s"].on_remote_sdp(kind, text)) \
        if "s" in session else None
    sig.on_ice = lambda idx, cand: session["s"].on_remote_ice(cand) if "s" in session else None
    sig.on_error = on_error
    sig.on_disconnect = done.set
    reader = asyncio.ensure_future(sig.start())
    stopper = asyncio.ensure_future(stop.wait())
    await asyncio.wait([asyncio.ensure_future(done.wait()), stopper], return_when=asyncio.FIRST_COMPLETED)
    stopper.cancel()
    if "s" in session:
        await session["s"].stop()
        if media != "audio":
            _run_hook(args.start_after_disconnect)
    reader.cancel()
    await sig.stop()


async def _start_metrics(port: int) -> None:
    from aiohttp import web
    from selkies_gstreamer_amd.server.metrics import Metrics
    m = Metrics()
    app = web.Application()
    app.router.add_get("/metrics", m.handler)
    runner = web.AppRunner(app)
    await runner.setup()
    await web.TCPSite(runner, "0.0.0.0", port).start()


async def default_input_factory(session: StreamSession):
    """X11 (XTest) injection, optional uinput mouse, gamepads over the js interposer sockets,
    clipboard and cursor updates on the data channel (webrtc_input.py / gstwebrtc_app.py)."""
    import base64
    import threading
    from selkies_gstreamer_amd.server.gamepad import GamepadHub
    from selkies_gstreamer_amd.server.input import (Clipboard, CursorWatcher, InputHandler, Injector,
                                                    UinputMouse, X11Injector)
    args = session.args
    disp = os.environ.get("DISPLAY")
    inj = X11Injector(disp) if disp else Injector()
    if args.uinput_mouse_socket:
        inj = UinputMouse(args.uinput_mouse_socket, inj)
    hub = GamepadHub(args.js_socket_path)
    await hub.start()

    async def send_clipboard(data: bytes, mime: str):
        session.send_message("clipboard", {"content": base64.b64encode(data).decode()})
    handler = InputHandler(inj, gamepads=hub, clipboard=Clipboard(), enable_clipboard=args.enable_clipboard,
                           send_clipboard=send_clipboard,
                           on_client_fps=lambda f: setattr(session, "client_fps", f))
    handler.start_clipboard_monitor()
    if disp and _truthy(args.enable_cursors):
        watcher = CursorWatcher(lambda msg: session.loop.call_soon_threadsafe(session.send_message, "cursor", msg),
                                disp)
        if watcher.available:
            threading.Thread(target=watcher.run, name="cursor-watch", daemon=True).start()
            orig = handler.close

            async def close():
                watcher.stop()
                await orig()
            handler.close = close
    return handler


def main(argv=None) -> int:
    args = parse_args(argv)
    logging.basicConfig(level=logging.DEBUG if args.debug else logging.INFO)
    try:
        asyncio.run(serve(args, default_input_factory))
    except (KeyboardInterrupt, SignallingError):
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
