"""ctypes binding of ``libselkies_native.so`` (C ABI in csrc/runtime/sk_api.h).

The library is built in-tree by ``selkies_gstreamer_amd.ops.build`` (also called
from ``__graft_entry__.build()``). On a GPU box the HIP backend is mandatory for
GPU-marked paths: `require_gpu()` raises instead of silently falling back.
"""
from __future__ import annotations

import collections
import ctypes
import os
import threading
from dataclasses import dataclass
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ["SK_NATIVE_LIB"]) if os.environ.get("SK_NATIVE_LIB") else \
    Path(__file__).resolve().parents[1] / "_lib" / "libselkies_native.so"
_lib = None
_lock = threading.Lock()


class SkH264Config(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("stripe_height", ctypes.c_int32),
        ("fullframe", ctypes.c_int32), ("full_range", ctypes.c_int32),
        ("qp", ctypes.c_int32), ("paint_qp", ctypes.c_int32), ("use_paint_over", ctypes.c_int32),
        ("paint_over_trigger", ctypes.c_int32), ("paint_over_burst", ctypes.c_int32),
        ("streaming_mode", ctypes.c_int32), ("damage_threshold", ctypes.c_int32),
        ("damage_duration", ctypes.c_int32), ("me_range", ctypes.c_int32), ("me_iters", ctypes.c_int32),
        ("scenecut", ctypes.c_int32), ("fps", ctypes.c_float), ("device", ctypes.c_int32),
        ("backend", ctypes.c_int32), ("deblock", ctypes.c_int32), ("me_full", ctypes.c_int32),
        ("shared_copy", ctypes.c_int32), ("src_width", ctypes.c_int32), ("src_height", ctypes.c_int32),
        ("num_refs", ctypes.c_int32), ("codec", ctypes.c_int32), ("aq_strength", ctypes.c_int32),
        ("subpel", ctypes.c_int32), ("intra4x4", ctypes.c_int32),
        ("tile_cols_log2", ctypes.c_int32), ("tile_rows_log2", ctypes.c_int32),
        ("rc_mode", ctypes.c_int32), ("bitrate_kbps", ctypes.c_int32),
    ]


class SkJpegConfig(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "width", "height", "stripe_height", "quality", "paint_quality", "use_paint_over",
        "paint_over_trigger", "device", "backend")]


class SkCaptureSettings(ctypes.Structure):
    """Mirror of ``sk_capture_settings`` (pixelflux CaptureSettings + extensions)."""
    _fields_ = [
        ("capture_width", ctypes.c_int32), ("capture_height", ctypes.c_int32),
        ("capture_x", ctypes.c_int32), ("capture_y", ctypes.c_int32),
        ("target_fps", ctypes.c_double),
        ("capture_cursor", ctypes.c_int32), ("debug_logging", ctypes.c_int32), ("output_mode", ctypes.c_int32),
        ("jpeg_quality", ctypes.c_int32), ("paint_over_jpeg_quality", ctypes.c_int32),
        ("use_paint_over_quality", ctypes.c_int32),
        ("paint_over_trigger_frames", ctypes.c_int32), ("damage_block_threshold", ctypes.c_int32),
        ("damage_block_duration", ctypes.c_int32),
        ("h264_crf", ctypes.c_int32), ("h264_paintover_crf", ctypes.c_int32),
        ("h264_paintover_burst_frames", ctypes.c_int32),
        ("h264_fullcolor", ctypes.c_int32), ("h264_streaming_mode", ctypes.c_int32),
        ("h264_fullframe", ctypes.c_int32),
        ("use_cpu", ctypes.c_int32), ("vaapi_render_node_index", ctypes.c_int32),
        ("watermark_path", ctypes.c_char_p), ("watermark_location_enum", ctypes.c_int32),
        ("device", ctypes.c_int32), ("stripe_height", ctypes.c_int32), ("source", ctypes.c_int32),
        ("display", ctypes.c_char_p),
        ("output_width", ctypes.c_int32), ("output_height", ctypes.c_int32),
        ("step_mode", ctypes.c_int32), ("pool", ctypes.c_void_p),
        ("pool_frames", ctypes.c_int32), ("pool_stride", ctypes.c_int32), ("pool_phase", ctypes.c_int32),
        ("h264_aq_strength", ctypes.c_int32), ("h264_subpel", ctypes.c_int32), ("h264_intra4x4", ctypes.c_int32),
        ("h264_rc_mode", ctypes.c_int32), ("h264_bitrate_kbps", ctypes.c_int32),
        ("h264_me_full", ctypes.c_int32),
    ]


class SkStripeResult(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("stripe_y_start", ctypes.c_int32), ("stripe_height", ctypes.c_int32),
                ("size", ctypes.c_int32), ("data", ctypes.POINTER(ctypes.c_ubyte)), ("frame_id", ctypes.c_int32),
                ("grab_ns", ctypes.c_int64)]


SK_STRIPE_CB = ctypes.CFUNCTYPE(None, ctypes.POINTER(SkStripeResult), ctypes.c_void_p)
SK_FRAME_CB = ctypes.CFUNCTYPE(None, ctypes.POINTER(SkStripeResult), ctypes.c_int32, ctypes.c_void_p)


class SkPacket(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("size", ctypes.c_int32), ("y", ctypes.c_int32),
                ("w", ctypes.c_int32), ("h", ctypes.c_int32), ("key", ctypes.c_int32)]


def lib():
    """Loads (building first if needed and possible) the native library."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not LIB_PATH.exists() and os.environ.get("SK_NO_AUTOBUILD") != "1":
            from .build import build
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        L.sk_version.restype = ctypes.c_char_p
        L.sk_last_error.restype = ctypes.c_char_p
        L.sk_hip_device_count.restype = ctypes.c_int
        L.sk_h264_create.restype = ctypes.c_void_p
        L.sk_h264_create.argtypes = [ctypes.POINTER(SkH264Config)]
        L.sk_h264_destroy.argtypes = [ctypes.c_void_p]
        L.sk_h264_request_keyframe.argtypes = [ctypes.c_void_p]
        L.sk_h264_set_qp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.sk_h264_set_rate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.sk_h264_wait_stream.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.sk_h264_rc_stats.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.sk_h264_set_overlay_image.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                                ctypes.c_int]
        L.sk_h264_set_overlay_pos.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 6
        L.sk_h264_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        L.sk_h264_encode.restype = ctypes.c_int
        L.sk_h264_encode_yuv.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32,
                                         ctypes.c_int32, ctypes.c_int32]
        L.sk_h264_submit.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        L.sk_h264_finish.argtypes = [ctypes.c_void_p]
        L.sk_h264_upload.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
        L.sk_h264_launch.argtypes = [ctypes.c_void_p]
        L.sk_h264_set_upload_rows.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        L.sk_upload_ranges.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
        L.sk_h264_state_bytes.argtypes = [ctypes.c_void_p]
        L.sk_h264_state_bytes.restype = ctypes.c_int64
        L.sk_h264_export_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        L.sk_h264_import_state.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32]
        L.sk_h264_get_packet.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(SkPacket)]
        L.sk_h264_debug_buffer.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int64]
        L.sk_h264_debug_buffer.restype = ctypes.c_int64
        L.sk_h264_stage_times.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int32]
        L.sk_h264_stage_times.restype = ctypes.c_int
        L.sk_host_alloc.restype = ctypes.c_void_p
        L.sk_host_alloc.argtypes = [ctypes.c_int64]
        L.sk_host_free.argtypes = [ctypes.c_void_p]
        L.sk_jpeg_create.restype = ctypes.c_void_p
        L.sk_jpeg_create.argtypes = [ctypes.POINTER(SkJpegConfig)]
        L.sk_capture_create.restype = ctypes.c_void_p
        L.sk_capture_destroy.argtypes = [ctypes.c_void_p]
        L.sk_capture_start.argtypes = [ctypes.c_void_p, ctypes.POINTER(SkCaptureSettings), SK_STRIPE_CB,
                                       ctypes.c_void_p]
        L.sk_capture_start.restype = ctypes.c_int
        L.sk_capture_start_frames.argtypes = [ctypes.c_void_p, ctypes.POINTER(SkCaptureSettings), SK_FRAME_CB,
                                              ctypes.c_void_p]
        L.sk_capture_start_frames.restype = ctypes.c_int
        L.sk_capture_run.argtypes = [ctypes.c_void_p, ctypes.c_int64]
        L.sk_capture_wait.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.sk_capture_wait.restype = ctypes.c_int
        L.sk_capture_latencies.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.c_int, ctypes.c_int]
        L.sk_capture_latencies.restype = ctypes.c_int
        L.sk_capture_stop.argtypes = [ctypes.c_void_p]
        L.sk_capture_request_keyframe.argtypes = [ctypes.c_void_p]
        L.sk_capture_set_qp.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.sk_capture_set_rate.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.sk_capture_move.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.sk_capture_move.restype = ctypes.c_int
        L.sk_capture_device.argtypes = [ctypes.c_void_p]
        L.sk_capture_device.restype = ctypes.c_int
        L.sk_capture_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.sk_capture_set_watermark.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int]
        _lib = L
        return L


def hip_device_count() -> int:
    return int(lib().sk_hip_device_count())


def convert_bgrx(bgrx: np.ndarray, fmt: str = "i420", backend: str = "cpu", device: int = 0,
                 full_range: bool = False):
    """BGRx (H, W, 4) -> 4:2:0 planes with the encoders' K1 arithmetic (hipconvert's
    converter): ``fmt`` "i420" -> (y, u, v), "nv12" -> (y, uv)."""
    L = lib()
    for name, res, args in (("sk_convert_create", ctypes.c_void_p, [ctypes.c_int] * 5),
                            ("sk_convert_run_ex", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                                                 ctypes.c_int32, ctypes.c_int32] +
                             [ctypes.c_void_p, ctypes.c_int32] * 3 + [ctypes.c_int32]),
                            ("sk_convert_destroy", None, [ctypes.c_void_p])):
        getattr(L, name).restype = res
        getattr(L, name).argtypes = args
    H, W = bgrx.shape[:2]
    bgrx = np.ascontiguousarray(bgrx)
    cw, ch = (W + 1) // 2, (H + 1) // 2
    y = np.zeros((H, W), np.uint8)
    nv12 = fmt.lower() == "nv12"
    u = np.zeros((ch, 2 * cw if nv12 else cw), np.uint8)
    v = np.zeros((ch, cw), np.uint8)
    c = L.sk_convert_create(W, H, int(full_range), 1 if backend == "hip" else 0, device)
    if not c:
        raise RuntimeError(L.sk_last_error().decode())
    try:
        if L.sk_convert_run_ex(c, bgrx.ctypes.data, bgrx.strides[0], 0, 2 if nv12 else 1, y.ctypes.data, W,
                               u.ctypes.data, u.strides[0], v.ctypes.data, cw, 0) < 0:
            raise RuntimeError(L.sk_last_error().decode())
    finally:
        L.sk_convert_destroy(c)
    return (y, u) if nv12 else (y, u, v)


class DevicePlane:
    """A 2-D uint8 plane copied into HIP device memory of `device` (libselkies_native's
    sk_dev_* allocator, no torch): pass it to :meth:`H264Encoder.encode_yuv` for device
    input. Freed on close / GC."""

    def __init__(self, array: np.ndarray, device: int = 0):
        L = lib()
        L.sk_dev_alloc.restype = ctypes.c_void_p
        L.sk_dev_alloc.argtypes = [ctypes.c_int32, ctypes.c_int64]
        L.sk_dev_free.argtypes = [ctypes.c_int32, ctypes.c_void_p]
        L.sk_dev_copy.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32]
        a = np.ascontiguousarray(array, np.uint8)
        if a.ndim != 2:
            raise ValueError("planes are 2-D")
        self.device, self.shape, self.stride = device, a.shape, a.strides[0]
        self.dev_ptr = L.sk_dev_alloc(device, max(1, a.nbytes))
        if not self.dev_ptr:
            raise MemoryError(L.sk_last_error().decode())
        if a.nbytes and L.sk_dev_copy(device, self.dev_ptr, a.ctypes.data, a.nbytes, 0) != 0:
            raise RuntimeError(L.sk_last_error().decode())

    def close(self):
        if getattr(self, "dev_ptr", None):
            lib().sk_dev_free(self.device, self.dev_ptr)
            self.dev_ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def upload_ranges(pairs, rows: int):
    """Row ranges a damage-driven upload copies for ``pairs`` [(y0, y1), ...] of a
    ``rows``-row frame (the HIP backend's band union, clamped; bad pairs drop out)."""
    a = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(-1, 2))
    cap = max(1, (int(rows) + 15) // 16)
    out = np.zeros((cap, 2), np.int32)
    n = lib().sk_upload_ranges(a.ctypes.data if a.size else None, a.shape[0], int(rows), out.ctypes.data, cap)
    return [tuple(int(v) for v in r) for r in out[:n]]


def require_gpu():
    if hip_device_count() < 1:
        raise RuntimeError("no HIP device visible to libselkies_native (gfx950 backend required)")


class PinnedBuffer:
    """Page-locked host buffer exposed as a numpy array (frees on close/GC)."""

    def __init__(self, shape, dtype=np.uint8):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        n = int(np.prod(self.shape)) * self.dtype.itemsize
        self._ptr = lib().sk_host_alloc(n)
        if not self._ptr:
            raise MemoryError("sk_host_alloc failed")
        buf = (ctypes.c_uint8 * n).from_address(self._ptr)
        self.array = np.frombuffer(buf, dtype=self.dtype).reshape(self.shape)

    def close(self):
        if self._ptr:
            self.array = None
            lib().sk_host_free(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _buffer_ptr(buf, nbytes: int):
    """(on_device, address) of a numpy array or a torch tensor of at least nbytes."""
    if hasattr(buf, "data_ptr"):
        if buf.numel() * buf.element_size() < nbytes or not buf.is_contiguous():
            raise ValueError("state tensor too small or not contiguous")
        return (1 if buf.is_cuda else 0), buf.data_ptr()
    a = np.asarray(buf)
    if a.nbytes < nbytes or not a.flags["C_CONTIGUOUS"]:
        raise ValueError("state buffer too small or not contiguous")
    return 0, a.ctypes.data


@dataclass
class Packet:
    data: bytes
    y: int
    w: int
    h: int
    key: bool


MB_INFO_DTYPE = np.dtype([
    ("mvx", "<i2"), ("mvy", "<i2"), ("mvdx", "<i2"), ("mvdy", "<i2"), ("type", "u1"), ("i16_mode", "u1"),
    ("chroma_mode", "u1"), ("cbp", "u1"), ("qp", "u1"), ("nnz", "u1", (24,)), ("ref", "u1"), ("pad", "u1", (2,)),
    ("i4lo", "<u4"), ("i4hi", "<u4"),
])
ME_DTYPE = np.dtype([("mvx", "<i2"), ("mvy", "<i2"), ("sad", "<i4"), ("intra_est", "<i4"), ("ref", "<i2"),
                     ("fx", "i1"), ("fy", "i1")])
TASK_DTYPE = np.dtype([(n, "<i4") for n in (
    "action", "qp", "first_row", "num_rows", "pic_row0", "pic_rows", "frame_num", "idr_pic_id",
    "allow_scenecut", "idr_on_intra", "final_action", "num_refs")])


RC_MODES = {"cqp": 0, "crf": 1, "cbr": 2}
RC_FIELDS = ("mode", "base_qp", "qp_min", "qp_max", "budget", "vbv_size", "fullness", "frames", "last_qp_p",
             "last_qp_i", "last_bits_p", "last_bits_i", "last_cplx_p", "last_cplx_i", "cplx_ema", "cur_qp",
             "cur_intra", "cur_cplx", "max_p_bits", "seq", "cur_valid", "pixels", "cur_idr", "redos", "qp_floor", "floor_age", "last_mbs_p", "last_mbs_i", "cur_mbs", "vbv_ms", "last_qpf_p", "last_qpf_i", "cur_qpf",
             "cur_redo", "redo_qpf", "redo_bits", "codec", "lam_boost")


def deblock_mode(deblock) -> int:
    """SkH264Config.deblock of a Python value: True -> 1 (on), False -> -1 (off), "auto" -> 2."""
    if isinstance(deblock, str):
        if deblock != "auto":
            raise ValueError("deblock must be True, False or 'auto'")
        return 2
    return 1 if deblock else -1


class H264Encoder:
    """Stripe H.264 encoder session (CPU reference backend or HIP backend)."""

    def __init__(self, width: int, height: int, *, stripe_height: int = 64, fullframe: bool = False,
                 full_range: bool = False, qp: int = 25, paint_qp: int = 18, use_paint_over: bool = True,
                 paint_over_trigger: int = 15, paint_over_burst: int = 5, streaming_mode: bool = False,
                 damage_threshold: int = 10, damage_duration: int = 20, me_range: int = 64,
                 me_iters: int = 24, scenecut: bool = True, fps: float = 60.0, device: int = 0,
                 backend: str = "cpu", deblock="auto", me_full: bool = True, shared_copy: bool = False,
                 src_width: int = 0, src_height: int = 0, num_refs: int = 1, codec: str = "h264",
                 aq_strength: float = 0.0, subpel: bool = True, intra4x4: bool = False,
                 tile_cols_log2: int = -1, tile_rows_log2: int = -1, rate_control: str = "cqp",
                 bitrate_kbps: int = 0):
        """aq_strength: MB-level adaptive QP (h264_mb.h aq_offset), 1.0 = x264 aq-mode 1
        strength; 0 = constant QP per slice (x264 ultrafast behaviour). deblock: True / False,
        or "auto" (the slices coded at QP >= 34, h264_encoder.h slice_deblock)."""
        L = lib()
        if backend not in ("cpu", "hip"):
            raise ValueError("backend must be 'cpu' or 'hip'")
        if backend == "hip":
            require_gpu()
        self.cfg = SkH264Config(width, height, stripe_height, int(fullframe), int(full_range), qp, paint_qp,
                                int(use_paint_over), paint_over_trigger, paint_over_burst, int(streaming_mode),
                                damage_threshold, damage_duration, me_range, me_iters, int(scenecut), fps,
                                device, 1 if backend == "hip" else 0, deblock_mode(deblock),
                                1 if me_full else -1, 1 if shared_copy else 0, int(src_width), int(src_height),
                                int(num_refs), {"h264": 0, "hevc": 1, "av1": 2}.get(codec, 0),
                                int(round(aq_strength * 16)), 0 if subpel else -1, 1 if intra4x4 else 0,
                                int(tile_cols_log2), int(tile_rows_log2),
                                RC_MODES[rate_control], int(bitrate_kbps))
        if codec not in ("h264", "hevc", "av1"):
            raise ValueError("codec must be 'h264', 'hevc' or 'av1'")
        self.codec = codec
        self.width, self.height = width, height
        self.backend = backend
        self._h = L.sk_h264_create(ctypes.byref(self.cfg))
        if not self._h:
            raise RuntimeError(f"sk_h264_create failed: {L.sk_last_error().decode()}")
        self._inflight = collections.deque()   # input frames kept alive until finish()
        self._staged = None

    def close(self):
        if getattr(self, "_h", None):
            lib().sk_h264_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def request_keyframe(self):
        lib().sk_h264_request_keyframe(self._h)

    def set_overlay(self, slot: int, bgra) -> None:
        """K12/K13: overlay image for slot 0 (watermark) or 1 (cursor), premultiplied BGRA
        uint8 (h, w, 4), at most 512x512; None clears it. Blended inside the colour
        conversion of every following frame (the captured frame is not modified)."""
        if bgra is None:
            rc = lib().sk_h264_set_overlay_image(self._h, int(slot), None, 0, 0)
        else:
            a = np.ascontiguousarray(bgra, dtype=np.uint8)
            if a.ndim != 3 or a.shape[2] != 4:
                raise ValueError("overlay must be (h, w, 4) BGRA")
            rc = lib().sk_h264_set_overlay_image(self._h, int(slot), a.ctypes.data, a.shape[1], a.shape[0])
        if rc < 0:
            raise ValueError("overlay not supported (slot / size / encoder)")

    def set_overlay_pos(self, slot: int, x: int, y: int, tile=None, enabled: bool = True) -> None:
        """Placement of overlay `slot` for the frames encoded from now on; tile=(dx, dy)
        repeats the image with that period to the right and downwards."""
        tdx, tdy = tile if tile else (0, 0)
        lib().sk_h264_set_overlay_pos(self._h, int(slot), int(bool(enabled)), int(x), int(y), int(tdx), int(tdy))

    def set_qp(self, qp: int, paint_qp: int = 0):
        """Rate control: QP for changed / paint-over stripes from the next frame (<= 0 keeps)."""
        lib().sk_h264_set_qp(self._h, int(qp), int(paint_qp))

    def encode(self, bgrx: np.ndarray, frame_id: int = 0) -> list[Packet]:
        """bgrx: uint8 array (H, W, 4) or (H, stride) rows. Returns 0x04 stripe packets."""
        if bgrx.dtype != np.uint8:
            raise TypeError("bgrx must be uint8")
        if not bgrx.flags["C_CONTIGUOUS"]:
            bgrx = np.ascontiguousarray(bgrx)
        stride = bgrx.strides[0]
        L = lib()
        n = L.sk_h264_encode(self._h, bgrx.ctypes.data, stride, frame_id & 0xFFFF)
        if n < 0:
            raise RuntimeError(f"encode failed: {L.sk_last_error().decode()}")
        out = []
        pk = SkPacket()
        for i in range(n):
            L.sk_h264_get_packet(self._h, i, ctypes.byref(pk))
            out.append(Packet(ctypes.string_at(pk.data, pk.size), pk.y, pk.w, pk.h, bool(pk.key)))
        return out

    def encode_yuv(self, fmt: str, y, u, v=None, frame_id: int = 0) -> list[Packet]:
        """Planar 4:2:0 input instead of BGRx (GStreamer NV12 / I420 caps): ``fmt`` "i420"
        (y, u, v planes) or "nv12" (y plane, interleaved uv as ``u``). Planes are numpy
        uint8 arrays (host) or torch uint8 tensors on this encoder's GPU (device input,
        no host copy) or :class:`DevicePlane`. W x H luma, ((W+1)/2) x ((H+1)/2) chroma
        (x2 wide for NV12 uv)."""
        code = {"i420": 1, "nv12": 2}[fmt.lower()]
        planes = [y, u] + ([v] if code == 1 else [u])
        on_dev = int(isinstance(y, DevicePlane) or (hasattr(y, "data_ptr") and bool(getattr(y, "is_cuda", False))))
        ptrs, strides = [], []
        for p in planes:
            if isinstance(p, DevicePlane):
                ptrs.append(p.dev_ptr)
                strides.append(p.stride)
            elif hasattr(p, "data_ptr"):
                if p.dim() != 2 or p.stride(1) != 1:
                    raise ValueError("planes must be 2-D with unit column stride")
                ptrs.append(p.data_ptr())
                strides.append(p.stride(0) * p.element_size())
            else:
                a = np.asarray(p)
                if a.dtype != np.uint8 or a.ndim != 2 or a.strides[1] != 1:
                    raise ValueError("planes must be 2-D uint8 arrays with unit column stride")
                ptrs.append(a.ctypes.data)
                strides.append(a.strides[0])
        L = lib()
        n = L.sk_h264_encode_yuv(self._h, code, ptrs[0], strides[0], ptrs[1], strides[1], ptrs[2], strides[2],
                                 on_dev, frame_id & 0xFFFF)
        if n < 0:
            raise RuntimeError(f"encode_yuv failed: {L.sk_last_error().decode()}")
        out = []
        pk = SkPacket()
        for i in range(n):
            L.sk_h264_get_packet(self._h, i, ctypes.byref(pk))
            out.append(Packet(ctypes.string_at(pk.data, pk.size), pk.y, pk.w, pk.h, bool(pk.key)))
        return out

    def submit(self, bgrx: np.ndarray, frame_id: int = 0) -> None:
        """Queues a frame and returns at once (HIP: upload + graph launch); the array
        is kept alive until :meth:`finish`. Submit several encoders, then finish them."""
        if bgrx.dtype != np.uint8:
            raise TypeError("bgrx must be uint8")
        if not bgrx.flags["C_CONTIGUOUS"]:
            bgrx = np.ascontiguousarray(bgrx)
        L = lib()
        if L.sk_h264_submit(self._h, bgrx.ctypes.data, bgrx.strides[0], frame_id & 0xFFFF) < 0:
            raise RuntimeError(f"submit failed: {L.sk_last_error().decode()}")
        self._inflight.append(bgrx)

    def upload(self, bgrx: np.ndarray, frame_id: int = 0) -> None:
        """First half of :meth:`submit`: stages the frame (HIP: H2D on the copy stream).
        Allowed while the previous frame is still in flight — its upload overlaps that
        frame's kernels. Then either :meth:`launch` it after :meth:`finish` of the previous
        frame, or launch it at once (two frames in flight: the GPU runs it while the host
        collects the previous frame's packets) and finish the older frame afterwards."""
        if bgrx.dtype != np.uint8:
            raise TypeError("bgrx must be uint8")
        if not bgrx.flags["C_CONTIGUOUS"]:
            bgrx = np.ascontiguousarray(bgrx)
        self._staged = bgrx
        L = lib()
        if L.sk_h264_upload(self._h, bgrx.ctypes.data, bgrx.strides[0], frame_id & 0xFFFF) < 0:
            self._staged = None
            raise RuntimeError(f"upload failed: {L.sk_last_error().decode()}")

    def upload_ptr(self, ptr: int, stride: int, frame_id: int = 0, keepalive=None, wait_stream: int = 0) -> None:
        """:meth:`upload` from a raw address: host memory or, on the HIP backend, device
        memory of this encoder's GPU (e.g. a torch tensor's ``data_ptr()``; the copy is
        then device-to-device). ``keepalive`` is held until the frame is finished.
        ``wait_stream``: a HIP stream handle of this device (``torch.cuda.Stream.cuda_stream``)
        whose queued work produces the source; the copy waits for it on the device."""
        self._staged = keepalive
        L = lib()
        if wait_stream and L.sk_h264_wait_stream(self._h, ctypes.c_void_p(int(wait_stream))) < 0:
            self._staged = None
            raise RuntimeError(f"wait_stream failed: {L.sk_last_error().decode()}")
        if L.sk_h264_upload(self._h, ctypes.c_void_p(int(ptr)), int(stride), frame_id & 0xFFFF) < 0:
            self._staged = None
            raise RuntimeError(f"upload failed: {L.sk_last_error().decode()}")

    def set_upload_rows(self, rows) -> None:
        """Damage of the next :meth:`upload`: ``[(y0, y1), ...]`` rows changed since the
        previous upload, or None (unknown: full copy)."""
        L = lib()
        if rows is None:
            L.sk_h264_set_upload_rows(self._h, None, -1)
            return
        a = np.ascontiguousarray(np.asarray(rows, np.int32).reshape(-1, 2))
        L.sk_h264_set_upload_rows(self._h, a.ctypes.data if a.size else None, a.shape[0])

    def launch(self) -> None:
        L = lib()
        if L.sk_h264_launch(self._h) < 0:
            raise RuntimeError(f"launch failed: {L.sk_last_error().decode()}")
        self._inflight.append(getattr(self, "_staged", None))
        self._staged = None

    def finish(self) -> list[Packet]:
        L = lib()
        n = L.sk_h264_finish(self._h)
        if self._inflight:
            self._inflight.popleft()
        if n < 0:
            raise RuntimeError(f"encode failed: {L.sk_last_error().decode()}")
        return self._packets(n)

    def _packets(self, n: int) -> list[Packet]:
        L = lib()
        out = []
        pk = SkPacket()
        for i in range(n):
            L.sk_h264_get_packet(self._h, i, ctypes.byref(pk))
            out.append(Packet(ctypes.string_at(pk.data, pk.size), pk.y, pk.w, pk.h, bool(pk.key)))
        return out

    # -- session state transfer (codec/h264_encoder.h StateHeader layout) -----------------
    def state_bytes(self) -> int:
        return int(lib().sk_h264_state_bytes(self._h))

    def export_state(self, out=None):
        """Snapshot of the session (reference, damage baseline, MV field, controller).
        ``out``: None (returns a host numpy array), a host numpy uint8 array, or a
        device tensor (``data_ptr()`` + ``is_cuda``) on this encoder's GPU."""
        n = self.state_bytes()
        if out is None:
            out = np.empty(n, np.uint8)
        on_dev, ptr = _buffer_ptr(out, n)
        if lib().sk_h264_export_state(self._h, ptr, on_dev) < 0:
            raise RuntimeError(f"export_state failed: {lib().sk_last_error().decode()}")
        return out

    def import_state(self, buf) -> None:
        """Continues the exported session here: the next frame is coded against the
        imported reference (no IDR), same controller state and QPs."""
        on_dev, ptr = _buffer_ptr(buf, self.state_bytes())
        if lib().sk_h264_import_state(self._h, ptr, on_dev) < 0:
            raise RuntimeError(f"import_state failed: {lib().sk_last_error().decode()}")

    def debug_buffer(self, name: str, dtype=np.uint8) -> np.ndarray:
        L = lib()
        n = L.sk_h264_debug_buffer(self._h, name.encode(), None, 0)
        if n < 0:
            raise KeyError(name)
        buf = np.empty(n, dtype=np.uint8)
        L.sk_h264_debug_buffer(self._h, name.encode(), buf.ctypes.data, n)
        return buf.view(dtype)

    def set_rate(self, mode: str = "crf", kbps: int = 0) -> None:
        """K10 rate control from the next frame: 'cqp', 'crf' or 'cbr' at `kbps`."""
        lib().sk_h264_set_rate(self._h, RC_MODES[mode], int(kbps))

    def rc_stats(self) -> dict:
        arr = (ctypes.c_int32 * 64)()
        n = lib().sk_h264_rc_stats(self._h, arr, 64)
        return {k: int(arr[i]) for i, k in enumerate(RC_FIELDS) if i < n}

    def stage_times(self, n: int = 16) -> list[float]:
        arr = (ctypes.c_float * n)()
        k = lib().sk_h264_stage_times(self._h, arr, n)
        return list(arr[:k])


class HevcEncoder(H264Encoder):
    """HEVC Main encoder session: full-frame pictures whose slices are stripes of whole
    32x32-CTB rows (WPP substreams), same front end as the H.264 encoder. Packets carry
    the 10-byte stripe header + Annex-B (VPS/SPS/PPS on IDR)."""

    def __init__(self, width: int, height: int, **kw):
        kw.pop("fullframe", None)
        super().__init__(width, height, codec="hevc", fullframe=True, **kw)


class Av1Encoder(H264Encoder):
    """AV1 Main (8-bit 4:2:0) encoder session: full-frame pictures coded as OBU
    temporal units (temporal delimiter, sequence header on key frames, one OBU_FRAME
    with all tiles), same front end as the H.264 encoder. Packets carry the 10-byte
    stripe header + the temporal unit (low-overhead bitstream format)."""

    def __init__(self, width: int, height: int, **kw):
        kw.pop("fullframe", None)
        super().__init__(width, height, codec="av1", fullframe=True, **kw)


class JpegEncoder(H264Encoder):
    """JPEG stripe encoder session; packets are [frame_id u16][y u16][JPEG]."""

    def __init__(self, width: int, height: int, *, stripe_height: int = 64, quality: int = 40,
                 paint_quality: int = 90, use_paint_over: bool = True, paint_over_trigger: int = 15,
                 device: int = 0, backend: str = "cpu"):
        L = lib()
        if backend not in ("cpu", "hip"):
            raise ValueError("backend must be 'cpu' or 'hip'")
        if backend == "hip":
            require_gpu()
        if stripe_height % 16:
            raise ValueError("JPEG stripe_height must be a multiple of 16")
        self.cfg = SkJpegConfig(width, height, stripe_height, quality, paint_quality, int(use_paint_over),
                                paint_over_trigger, device, 1 if backend == "hip" else 0)
        self.width, self.height = width, height
        self.backend = backend
        self._h = L.sk_jpeg_create(ctypes.byref(self.cfg))
        if not self._h:
            raise RuntimeError(f"sk_jpeg_create failed: {L.sk_last_error().decode()}")
