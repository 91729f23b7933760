"""pixelflux-compatible screen capture API backed by the MI355X encoder.

The reference server drives an external ``pixelflux`` module (selkies.py:64-75,
2846-2964): it fills a ``CaptureSettings`` structure, wraps a Python function in
``StripeCallback`` and calls ``ScreenCapture().start_capture(settings, cb)``; the
callback receives a ``StripeEncodeResult`` pointer per encoded stripe
(``.data[:.size]``, ``.frame_id``, ``.stripe_y_start``). This module keeps that
contract so the server code and existing integrations work unchanged, while the
capture/encode loop itself runs in ``libselkies_native.so`` (csrc/runtime/capture.cpp):
X11 MIT-SHM grab -> HIP colour convert / damage / H.264 or JPEG stripe encode on
gfx950 -> callback from the native thread.

Extensions over the reference: ``device`` (HIP ordinal), ``stripe_height``,
``source`` (-1 auto, 0 X11 only, 1/2/3 synthetic motion/desktop/noise) and
``display``. Without an X server the synthetic desktop keeps the pipeline
testable.
"""
from __future__ import annotations

import ctypes
import threading

from selkies_gstreamer_amd.ops import native as _native

CaptureSettings = _native.SkCaptureSettings
ENCODE_MS_BUCKETS = (0.25, 0.5, 1, 2, 4, 8, 16, 33, float("inf"))   # csrc/runtime/capture.cpp kHistLe
StripeEncodeResult = _native.SkStripeResult
StripeCallback = _native.SK_STRIPE_CB
# Extension: one call per encoded frame, (results pointer, count, user), so a
# consumer pays one Python call per frame instead of one per stripe.
FrameCallback = _native.SK_FRAME_CB

OUTPUT_MODE_JPEG = 0
OUTPUT_MODE_H264 = 1
OUTPUT_MODE_HEVC = 2   # extension: H.265 full-frame pictures
OUTPUT_MODE_AV1 = 3    # extension: AV1 temporal units (OBUs), full frame
SOURCE_POOL = 4        # extension: caller-owned frame pool (settings.pool / pool_frames)


def default_settings(width: int = 1920, height: int = 1080, **kw) -> CaptureSettings:
    """CaptureSettings with the server defaults (selkies.py:2925-2962)."""
    s = CaptureSettings()
    s.capture_width, s.capture_height = width, height
    s.capture_x = s.capture_y = 0
    s.target_fps = 60.0
    s.capture_cursor = 0
    s.output_mode = OUTPUT_MODE_H264
    s.jpeg_quality, s.paint_over_jpeg_quality, s.use_paint_over_quality = 40, 90, 1
    s.paint_over_trigger_frames, s.damage_block_threshold, s.damage_block_duration = 15, 10, 20
    s.h264_crf, s.h264_paintover_crf, s.h264_paintover_burst_frames = 25, 18, 5
    s.h264_rc_mode, s.h264_bitrate_kbps = 1, 0   # K10: CRF around h264_crf (x264 crf semantics)
    s.h264_fullcolor = s.h264_streaming_mode = s.h264_fullframe = 0
    s.use_cpu = 0
    s.vaapi_render_node_index = -1
    s.watermark_path = None
    s.watermark_location_enum = -1
    s.device = 0
    s.stripe_height = 64
    s.source = -1
    s.display = None
    s.step_mode = 0
    s.pool = None
    s.pool_frames = s.pool_stride = s.pool_phase = 0
    for k, v in kw.items():
        if isinstance(v, str):
            v = v.encode()
        setattr(s, k, v)
    return s


class ScreenCapture:
    """One capture + encode session (one per display / per GPU)."""

    def __init__(self):
        self._lib = _native.lib()
        self._h = self._lib.sk_capture_create()
        self._cb = None
        self._settings = None
        self._lock = threading.Lock()

    def set_watermark(self, path: str, location: int) -> bool:
        """Loads a PNG (alpha respected) to composite at `location` (0-6, see csrc/runtime/capture.cpp)."""
        try:
            import numpy as np
            from PIL import Image
            im = np.asarray(Image.open(path).convert("RGBA"), dtype=np.uint16)
        except (OSError, ImportError, ValueError):
            return False
        a = im[..., 3:4]
        bgra = np.concatenate([(im[..., 2::-1] * a + 127) // 255, a], axis=2).astype(np.uint8)
        bgra = np.ascontiguousarray(bgra)
        self._wm = bgra
        self._lib.sk_capture_set_watermark(self._h, bgra.ctypes.data, bgra.shape[1], bgra.shape[0], int(location))
        return True

    def start_capture(self, settings: CaptureSettings, callback) -> None:
        if not isinstance(callback, StripeCallback):
            callback = StripeCallback(callback)
        if settings.watermark_path and settings.watermark_location_enum >= 0:
            self.set_watermark(settings.watermark_path.decode(), settings.watermark_location_enum)
        with self._lock:
            self._cb = callback  # keep the thunk alive while the native thread runs
            self._settings = settings
            rc = self._lib.sk_capture_start(self._h, ctypes.byref(settings), callback, None)
            if rc != 0:
                self._cb = None
                raise RuntimeError(f"start_capture failed: {self._lib.sk_last_error().decode()}")

    def start_frame_capture(self, settings: CaptureSettings, callback) -> None:
        """Like start_capture, but ``callback(results, n, user)`` runs once per frame."""
        if not isinstance(callback, FrameCallback):
            callback = FrameCallback(callback)
        if settings.watermark_path and settings.watermark_location_enum >= 0:
            self.set_watermark(settings.watermark_path.decode(), settings.watermark_location_enum)
        with self._lock:
            self._cb = callback
            self._settings = settings
            rc = self._lib.sk_capture_start_frames(self._h, ctypes.byref(settings), callback, None)
            if rc != 0:
                self._cb = None
                raise RuntimeError(f"start_capture failed: {self._lib.sk_last_error().decode()}")

    def run(self, frames: int) -> None:
        """Step mode (settings.step_mode = 1): grant `frames` more frames (non-blocking)."""
        self._lib.sk_capture_run(self._h, int(frames))

    def wait(self, timeout_ms: int = -1) -> int:
        """Blocks until every granted frame is delivered: 0, 1 on timeout, -1 if stopped."""
        return int(self._lib.sk_capture_wait(self._h, int(timeout_ms)))

    def latencies(self, reset: bool = False, cap: int = 8192) -> list:
        """Capture-to-packets latency (ms) of the most recent frames, oldest first."""
        arr = (ctypes.c_float * cap)()
        n = self._lib.sk_capture_latencies(self._h, arr, cap, int(reset))
        return list(arr[:n])

    def stop_capture(self) -> None:
        with self._lock:
            if self._h:
                self._lib.sk_capture_stop(self._h)
            self._cb = None

    def request_keyframe(self) -> None:
        if self._h:
            self._lib.sk_capture_request_keyframe(self._h)

    def set_qp(self, qp: int, paint_qp: int = 0) -> None:
        """H.264 rate control from the next frame on (the WebRTC mode's bitrate controller)."""
        if self._h:
            self._lib.sk_capture_set_qp(self._h, int(qp), int(paint_qp))

    def set_rate(self, mode: str = "crf", kbps: int = 0) -> None:
        """K10 rate control from the next frame: 'cqp', 'crf' (around h264_crf) or
        'cbr' at `kbps` with a 1.5-frame VBV (csrc/codec/ratecontrol.h)."""
        if self._h:
            self._lib.sk_capture_set_rate(self._h, {"cqp": 0, "crf": 1, "cbr": 2}[mode], int(kbps))

    def move_to(self, device: int, timeout_ms: int = 10000) -> str:
        """Moves the running session's encoder to GPU `device` between two frames
        (csrc/runtime/capture.cpp CaptureSession::move_to). Returns "continued" when the
        inter-frame state was carried GPU-to-GPU (the stream goes on with P frames) or
        "keyframe" when the new encoder had to start a fresh stream; raises when the
        session stays where it is."""
        rc = self._lib.sk_capture_move(self._h, int(device), int(timeout_ms)) if self._h else -1
        if rc < 0:
            raise RuntimeError(f"move_to({device}) failed: {self._lib.sk_last_error().decode()}")
        return "continued" if rc == 0 else "keyframe"

    @property
    def device(self) -> int:
        """GPU the session encodes on (-1: CPU reference encoder or not running)."""
        return int(self._lib.sk_capture_device(self._h)) if self._h else -1

    def stats(self) -> dict:
        arr = (ctypes.c_double * 18)()
        self._lib.sk_capture_stats(self._h, arr, 18)
        return {"frames": int(arr[0]), "encode_ms_mean": arr[1], "bytes": int(arr[2]),
                "packets": int(arr[3]), "source": {1.0: "x11", 0.0: "synthetic"}.get(arr[4], "none"),
                "encode_ms_last": arr[5],
                # per-frame encode time histogram (native, bucket upper bounds in ms; last = +Inf)
                "encode_ms_buckets": list(ENCODE_MS_BUCKETS), "encode_ms_counts": [int(x) for x in arr[6:15]],
                "frames_in_flight": int(arr[15]),
                # damage-driven upload: fraction of captured rows that crossed PCIe
                "upload_fraction": arr[16],
                # last live move (move_to): ms the capture thread spent between two frames on it
                "move_stall_ms": arr[17]}

    def close(self) -> None:
        self.stop_capture()
        if self._h:
            self._lib.sk_capture_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
