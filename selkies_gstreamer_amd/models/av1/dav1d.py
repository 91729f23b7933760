"""Conformance oracle for the AV1 encoder: dav1d, called through ctypes.

The image has no ffmpeg / libaom tools, but Pillow's AVIF plugin bundles libavif,
which links dav1d 1.5.x (the VideoLAN AV1 decoder used by Chrome and Firefox) and
exports its public C API (``dav1d_open``, ``dav1d_send_data``,
``dav1d_get_picture``...). This module feeds raw AV1 OBU temporal units
(low-overhead bitstream format, spec §5) straight into it and returns I420 planes.
It is a test/verification tool only; nothing in the serving path loads it.

Only the public, ABI-stable parts of the dav1d structs are touched:
``Dav1dSettings.n_threads`` / ``.max_frame_delay`` (offsets 0 / 4),
``Dav1dData.data`` / ``.sz`` (0 / 8), and ``Dav1dPicture.data[3]``,
``.stride[2]``, ``.p.{w,h,layout,bpc}`` (16, 40, 56..68).
"""
from __future__ import annotations

import ctypes
import glob
import os
from typing import Optional

import numpy as np

_LIB = None


def _find() -> Optional[str]:
    try:
        import PIL
    except ImportError:
        return None
    base = os.path.dirname(os.path.dirname(PIL.__file__))
    for pat in ("pillow.libs/libavif*.so*", "PIL/.libs/libavif*.so*"):
        hits = sorted(glob.glob(os.path.join(base, pat)))
        if hits:
            return hits[0]
    return None


def available() -> bool:
    try:
        _lib()
        return True
    except OSError:
        return False


def _lib():
    global _LIB
    if _LIB is None:
        path = _find()
        if path is None:
            raise OSError("no libavif/dav1d on this image")
        L = ctypes.CDLL(path)
        L.dav1d_version.restype = ctypes.c_char_p
        L.dav1d_default_settings.argtypes = [ctypes.c_void_p]
        L.dav1d_open.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p]
        L.dav1d_data_create.restype = ctypes.c_void_p
        L.dav1d_data_create.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.dav1d_send_data.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.dav1d_get_picture.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.dav1d_picture_unref.argtypes = [ctypes.c_void_p]
        L.dav1d_data_unref.argtypes = [ctypes.c_void_p]
        L.dav1d_close.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        L.dav1d_flush.argtypes = [ctypes.c_void_p]
        _LIB = L
    return _LIB


def version() -> str:
    return _lib().dav1d_version().decode()


EAGAIN = -11


class Dav1dError(RuntimeError):
    pass


class Decoder:
    """Feed one temporal unit at a time, get the shown frame back (low latency:
    max_frame_delay 1; `n_threads` > 1 lets dav1d decode the frame's tiles in parallel,
    what a browser's decoder does for 4K)."""

    def __init__(self, n_threads: int = 1):
        L = self.L = _lib()
        settings = ctypes.create_string_buffer(1024)
        L.dav1d_default_settings(settings)
        ctypes.c_int.from_buffer(settings, 0).value = max(1, int(n_threads))   # n_threads
        ctypes.c_int.from_buffer(settings, 4).value = 1   # max_frame_delay
        self.ctx = ctypes.c_void_p()
        rc = L.dav1d_open(ctypes.byref(self.ctx), settings)
        if rc < 0:
            raise Dav1dError(f"dav1d_open failed ({rc})")

    def close(self):
        if self.ctx:
            self.L.dav1d_close(ctypes.byref(self.ctx))
            self.ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, tu: bytes, planes: bool = True):
        """One temporal unit -> (Y, U, V) uint8 arrays, or None if no picture came out.
        planes=False: the picture is released without a copy and (w, h) is returned
        (latency measurements: the copy out of dav1d's buffers is not decoding)."""
        L = self.L
        data = ctypes.create_string_buffer(256)
        buf = L.dav1d_data_create(data, len(tu))
        if not buf:
            raise Dav1dError("dav1d_data_create failed")
        ctypes.memmove(buf, tu, len(tu))
        pics = []
        while True:
            sz = ctypes.c_size_t.from_buffer(data, 8).value
            if sz == 0:
                break
            rc = L.dav1d_send_data(self.ctx, data)
            if rc < 0 and rc != EAGAIN:
                L.dav1d_data_unref(data)
                raise Dav1dError(f"dav1d_send_data: error {rc}")
            p = self._get(planes)
            if p is not None:
                pics.append(p)
            if rc == EAGAIN:
                continue
        while True:
            p = self._get(planes)
            if p is None:
                break
            pics.append(p)
        return pics[-1] if pics else None

    def _get(self, planes: bool = True):
        L = self.L
        pic = ctypes.create_string_buffer(1024)
        rc = L.dav1d_get_picture(self.ctx, pic)
        if rc == EAGAIN:
            return None
        if rc < 0:
            raise Dav1dError(f"dav1d_get_picture: error {rc}")
        ptrs = [ctypes.c_void_p.from_buffer(pic, 16 + 8 * i).value for i in range(3)]
        strides = [ctypes.c_ssize_t.from_buffer(pic, 40 + 8 * i).value for i in range(2)]
        w, h, layout, bpc = (ctypes.c_int.from_buffer(pic, 56 + 4 * i).value for i in range(4))
        if bpc != 8:
            L.dav1d_picture_unref(pic)
            raise Dav1dError(f"unexpected bit depth {bpc}")
        if not planes:
            L.dav1d_picture_unref(pic)
            return (w, h)
        planes = []
        for i, (pw, ph) in enumerate(((w, h), ((w + 1) // 2, (h + 1) // 2), ((w + 1) // 2, (h + 1) // 2))):
            st = strides[0 if i == 0 else 1]
            raw = ctypes.string_at(ptrs[i], st * (ph - 1) + pw)
            a = np.frombuffer(raw + b"\0" * (st * ph - len(raw)), dtype=np.uint8).reshape(ph, st)[:, :pw].copy()
            planes.append(a)
        L.dav1d_picture_unref(pic)
        return tuple(planes)


def decode_stream(tus) -> list:
    d = Decoder()
    try:
        return [d.decode(tu) for tu in tus]
    finally:
        d.close()
