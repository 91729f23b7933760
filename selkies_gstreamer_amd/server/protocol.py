"""Wire protocol of the data websocket (shared with the browser client).

Server -> client binary frames (first byte = type, reference selkies-core.js:2890-3010):
  ``0x01 0x00 + opus``            audio packet
  ``0x03 0x00 + fid16 + y16 + JPEG`` JPEG stripe (server adds the 2-byte prefix)
  ``0x04 key fid16 y16 w16 h16 + AnnexB`` H.264 stripe (emitted as-is by the encoder)
Server -> client text: ``MODE websockets``, ``server_settings`` JSON,
  ``system_stats``/``gpu_stats``/``network_stats`` JSON, ``stream_resolution``,
  ``DISPLAY_CONFIG_UPDATE,{json}``, ``PIPELINE_RESETTING <id>``, ``VIDEO_STARTED``,
  ``VIDEO_STOPPED``, ``AUDIO_STARTED``, ``AUDIO_STOPPED``, ``KILL <reason>``,
  ``cursor,{json}``, ``clipboard,<b64>`` / ``clipboard_binary,<mime>,<b64>`` /
  ``clipboard_start,<mime>,<size>`` + ``clipboard_data,<b64>`` + ``clipboard_finish``.
Client -> server: ``SETTINGS,{json}``, ``CLIENT_FRAME_ACK <fid>``, ``START_VIDEO``,
  ``STOP_VIDEO``, ``START_AUDIO``, ``STOP_AUDIO``, ``r,WxH,<display>``, ``s,<dpi>``,
  ``SET_NATIVE_CURSOR_RENDERING,<0|1>``, ``cmd,<shell>``, ``FILE_UPLOAD_START:<path>:<size>``,
  ``FILE_UPLOAD_END:<path>``, ``FILE_UPLOAD_ERROR:<path>:<msg>``, binary
  ``0x01+chunk`` (upload data) / ``0x02+pcm`` (microphone s16le mono 24 kHz), and the
  input vocabulary handled by :mod:`.input` (``kd``, ``ku``, ``m``, ``js`` ...).

Everything here is pure (no sockets, no clocks of its own) so it is unit-tested
directly; cf. reference selkies.py:1260-1310 (payload parsing), 1165-1236
(backpressure), 1843-1916 (upload path checks).
"""
from __future__ import annotations

import base64
import json
import os
from collections import OrderedDict, deque
from dataclasses import dataclass, field
from typing import Optional

MAX_FRAME_ID = 65535
SUSPICIOUS_GAP = MAX_FRAME_ID // 2
ALLOWED_DESYNC_MS = 2000
LATENCY_THRESHOLD_MS = 50
CHECK_INTERVAL_S = 0.5
STALL_TIMEOUT_S = 4.0
RTT_SAMPLES = 20
SENT_HISTORY = 1000
CLIPBOARD_CHUNK = 750 * 1024

AUDIO_PREFIX = b"\x01\x00"
JPEG_PREFIX = b"\x03\x00"
H264_TYPE = 0x04

MIC_SAMPLE_RATE = 24000
MIC_BUFFER_MAX = MIC_SAMPLE_RATE * 2 * 2  # 2 s of s16 mono


# --------------------------------------------------------------------------- SETTINGS
_INT_KEYS = ("framerate", "h264_crf", "manual_width", "manual_height", "audio_bitrate", "initialClientWidth",
             "initialClientHeight", "jpeg_quality", "paint_over_jpeg_quality", "h264_paintover_crf",
             "h264_paintover_burst_frames", "scaling_dpi", "h264_bitrate")
_BOOL_KEYS = ("h264_fullcolor", "h264_streaming_mode", "is_manual_resolution_mode", "use_cpu",
              "use_paint_over_quality", "enable_binary_clipboard")
_STR_KEYS = ("encoder", "displayId", "displayPosition")


def parse_settings_payload(payload: str) -> dict:
    """Parses the JSON of a ``SETTINGS,`` message into typed values (missing -> None)."""
    raw = json.loads(payload)
    if not isinstance(raw, dict):
        raise ValueError("SETTINGS payload must be a JSON object")
    out: dict = {}
    for k in _INT_KEYS:
        v = raw.get(k)
        out[k] = int(v) if v is not None else None
    for k in _BOOL_KEYS:
        v = raw.get(k)
        out[k] = (str(v).lower() == "true") if v is not None else None
    for k in _STR_KEYS:
        v = raw.get(k)
        out[k] = str(v) if v is not None else None
    return out


def settings_message(payload: dict) -> str:
    return "SETTINGS," + json.dumps(payload)


# --------------------------------------------------------------------------- frames
def frame_desync(server_id: int, client_id: int) -> int:
    """Frames the client is behind, modulo the 16-bit frame counter."""
    if server_id >= client_id:
        return server_id - client_id
    return (MAX_FRAME_ID - client_id) + server_id + 1


def parse_frame_ack(msg: str) -> int:
    parts = msg.split(" ")
    if len(parts) < 2:
        raise ValueError("ACK message has too few parts")
    return int(parts[-1])


@dataclass
class DisplayFlow:
    """Per-display send/ACK bookkeeping and the frame-based backpressure gate."""
    acknowledged: int = -1
    last_sent: int = 0
    sent_at: "OrderedDict[int, float]" = field(default_factory=OrderedDict)
    rtt: deque = field(default_factory=lambda: deque(maxlen=RTT_SAMPLES))
    smoothed_rtt_ms: float = 0.0
    last_ack_time: float = 0.0
    client_fps: float = 0.0
    enabled: bool = True     # True = frames may be sent

    def reset(self, now: float):
        self.acknowledged, self.last_sent = -1, 0
        self.sent_at.clear()
        self.rtt.clear()
        self.smoothed_rtt_ms = 0.0
        self.last_ack_time = now
        self.enabled = True

    def on_sent(self, frame_id: int, now: float):
        if not self.enabled:
            return
        self.sent_at[frame_id] = now
        self.last_sent = frame_id
        if len(self.sent_at) > SENT_HISTORY:
            self.sent_at.popitem(last=False)

    def on_ack(self, frame_id: int, now: float):
        self.acknowledged = frame_id
        self.last_ack_time = now
        t = self.sent_at.pop(frame_id, None)
        if t is not None:
            ms = (now - t) * 1000.0
            if ms >= 0:
                self.rtt.append(ms)
                self.smoothed_rtt_ms = sum(self.rtt) / len(self.rtt)

    def evaluate(self, now: float, capturing: bool, framerate: float,
                 allowed_desync_ms: float = ALLOWED_DESYNC_MS,
                 latency_threshold_ms: float = LATENCY_THRESHOLD_MS,
                 stall_timeout_s: float = STALL_TIMEOUT_S) -> bool:
        """One backpressure decision (run every CHECK_INTERVAL_S); returns ``enabled``.

        Frames stop when the client is more than ``allowed_desync_ms`` worth of
        frames behind (RTT-compensated above the latency threshold) or has not
        ACKed for ``stall_timeout_s``; a suspicious gap (counter wrap/reset) or no
        ACK yet always lifts backpressure.
        """
        if not capturing or self.acknowledged == -1:
            self.enabled = True
            if self.acknowledged == -1:
                self.last_ack_time = now
            return True
        fps = self.client_fps if self.client_fps > 0 else framerate
        s, c = self.last_sent, self.acknowledged
        if abs(s - c) > SUSPICIOUS_GAP:
            self.enabled = True
            self.last_ack_time = now
            return True
        if s == 0:
            return self.enabled
        desync = frame_desync(s, c)
        allowed = allowed_desync_ms / 1000.0 * fps
        adjust = self.smoothed_rtt_ms / 1000.0 * fps if self.smoothed_rtt_ms > latency_threshold_ms else 0.0
        if now - self.last_ack_time > stall_timeout_s:
            self.enabled = False
        else:
            self.enabled = (desync - adjust) <= allowed
        return self.enabled


# --------------------------------------------------------------------------- uploads
def sanitize_upload_path(upload_dir: str, rel_path: str) -> Optional[str]:
    """Resolves a client-supplied relative upload path inside ``upload_dir``.

    Leading separators are stripped (paths are always relative to the upload
    directory). Returns None for empty paths, ``..`` components, NUL bytes, an
    existing symlink target, or anything whose parent resolves (symlinks
    included) outside the upload directory.
    """
    if not rel_path:
        return None
    cleaned = rel_path.replace("\\", "/").lstrip("/")
    comps = [c for c in cleaned.split("/") if c not in ("", ".")]
    if not comps or any(c == ".." for c in comps) or any("\x00" in c for c in comps):
        return None
    root = os.path.realpath(upload_dir)
    target = os.path.join(root, *comps)
    parent = os.path.realpath(os.path.dirname(target))
    if parent != root and not parent.startswith(root + os.sep):
        return None
    if os.path.islink(target):
        return None
    return target


def parse_upload_start(msg: str):
    """``FILE_UPLOAD_START:<rel_path>:<size>`` -> (rel_path, size)."""
    body = msg[len("FILE_UPLOAD_START:"):]
    rel, _, size = body.rpartition(":")
    if not rel:
        raise ValueError("malformed FILE_UPLOAD_START")
    return rel, int(size)


# --------------------------------------------------------------------------- clipboard
def clipboard_messages(data: bytes, mime_type: str = "text/plain", chunk: int = CLIPBOARD_CHUNK) -> list[str]:
    """Server -> client clipboard messages (single or multipart)."""
    binary = mime_type != "text/plain"
    if len(data) < chunk:
        b64 = base64.b64encode(data).decode("ascii")
        return [f"clipboard_binary,{mime_type},{b64}" if binary else f"clipboard,{b64}"]
    out = [f"clipboard_start,{mime_type},{len(data)}"]
    for off in range(0, len(data), chunk):
        out.append("clipboard_data," + base64.b64encode(data[off:off + chunk]).decode("ascii"))
    out.append("clipboard_finish")
    return out


class ClipboardAssembler:
    """Client -> server multipart clipboard (``cws``/``cbs`` + ``cwd``/``cbd`` + ``cwe``/``cbe``)."""

    def __init__(self):
        self.buf: Optional[bytearray] = None
        self.mime = "text/plain"
        self.total = 0

    def start(self, mime: str, total: int):
        self.buf, self.mime, self.total = bytearray(), mime, int(total)

    def data(self, b64: str) -> bool:
        if self.buf is None:
            return False
        try:
            self.buf += base64.b64decode(b64)
            return True
        except (ValueError, TypeError):
            self.buf = None
            return False

    def end(self):
        """Returns (mime, bytes) when the size matches, else None."""
        buf, self.buf = self.buf, None
        if buf is None or len(buf) != self.total:
            return None
        return self.mime, bytes(buf)


# --------------------------------------------------------------------------- misc
def even_dims(w: int, h: int) -> tuple[int, int]:
    return w - (w % 2), h - (h % 2)


def parse_resolution(text: str) -> tuple[int, int]:
    w, h = text.lower().split("x")
    w, h = int(w), int(h)
    if w <= 0 or h <= 0:
        raise ValueError("non-positive resolution")
    return w, h


def stream_resolution_message(w: int, h: int) -> str:
    return json.dumps({"type": "stream_resolution", "width": w, "height": h})


def display_config_message(displays: list[str]) -> str:
    return "DISPLAY_CONFIG_UPDATE," + json.dumps({"type": "display_config_update", "displays": displays})
