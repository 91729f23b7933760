"""pcmflux-compatible audio capture: PulseAudio monitor -> Opus packets.

Contract of the reference server (selkies.py:64-70, 939-1070): fill an
``AudioCaptureSettings``, wrap a function in ``AudioChunkCallback`` and call
``AudioCapture().start_capture(settings, cb)``; the callback receives an
``AudioChunkEncodeResult`` pointer (``.data``/``.size`` = one Opus packet) from
the capture thread, and the server broadcasts ``0x01 0x00 + opus`` frames.

The capture loop is native (``csrc/runtime/audio_capture.cpp`` in
libselkies_native.so), like the reference's C++ pcmflux: a C++ thread reads the
PulseAudio source (libpulse-simple), applies the silence gate, encodes with
libopus and calls back once per packet; Python holds the GIL only inside the
callback. Both libraries are dlopen'ed at ``start_capture`` time; when either is
missing (as in this build image) ``available()`` is False and ``start_capture``
raises, which the server treats as "audio unavailable", the same as the
reference when its pcmflux import fails.

Extensions (not in the reference API, used by tests and headless boxes):
``device_name=b"synthetic[:hz]"`` reads a paced sine tone instead of PulseAudio,
and ``start_capture(..., codec="pcm")`` delivers raw s16le frames instead of Opus.
"""
from __future__ import annotations

import ctypes
from typing import Optional


class AudioCaptureSettings(ctypes.Structure):
    _fields_ = [
        ("device_name", ctypes.c_char_p),
        ("sample_rate", ctypes.c_int),
        ("channels", ctypes.c_int),
        ("opus_bitrate", ctypes.c_int),
        ("frame_duration_ms", ctypes.c_int),
        ("use_vbr", ctypes.c_bool),
        ("use_silence_gate", ctypes.c_bool),
        ("debug_logging", ctypes.c_bool),
    ]


class AudioChunkEncodeResult(ctypes.Structure):
    _fields_ = [("size", ctypes.c_int), ("data", ctypes.POINTER(ctypes.c_ubyte))]


AudioChunkCallback = ctypes.CFUNCTYPE(None, ctypes.POINTER(AudioChunkEncodeResult), ctypes.c_void_p)

CODEC_OPUS, CODEC_PCM = 0, 1


class _SkAudioSettings(ctypes.Structure):   # sk_audio_settings (csrc/runtime/sk_api.h)
    _fields_ = [("device_name", ctypes.c_char_p), ("sample_rate", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("opus_bitrate", ctypes.c_int32), ("frame_duration_ms", ctypes.c_int32),
                ("use_vbr", ctypes.c_int32), ("use_silence_gate", ctypes.c_int32), ("codec", ctypes.c_int32),
                ("synthetic_silence_frames", ctypes.c_int32)]


_bound = None


def _native():
    global _bound
    if _bound is None:
        from selkies_gstreamer_amd.ops import native
        L = native.lib()
        L.sk_audio_available.restype = ctypes.c_int
        L.sk_audio_create.restype = ctypes.c_void_p
        L.sk_audio_destroy.argtypes = [ctypes.c_void_p]
        L.sk_audio_start.argtypes = [ctypes.c_void_p, ctypes.POINTER(_SkAudioSettings), AudioChunkCallback,
                                     ctypes.c_void_p]
        L.sk_audio_start.restype = ctypes.c_int
        L.sk_audio_stop.argtypes = [ctypes.c_void_p]
        L.sk_audio_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.sk_audio_error.argtypes = [ctypes.c_void_p]
        L.sk_audio_error.restype = ctypes.c_char_p
        _bound = L
    return _bound


def available() -> bool:
    """True when PulseAudio capture + Opus encoding can run on this machine."""
    return _native().sk_audio_available() == 3


class AudioCapture:
    def __init__(self):
        self._h: Optional[int] = None
        self._cb = None
        self._final: dict = {}

    def start_capture(self, settings: AudioCaptureSettings, callback, codec: str = "opus",
                      synthetic_silence_frames: int = 0) -> None:
        L = _native()
        if self._h is not None:
            raise RuntimeError("pcmflux: capture already running")
        if not isinstance(callback, AudioChunkCallback):
            callback = AudioChunkCallback(callback)
        self._cb = callback   # kept alive while the native thread may call it
        s = _SkAudioSettings(settings.device_name, int(settings.sample_rate or 48000), int(settings.channels or 2),
                             int(settings.opus_bitrate or 320000), int(settings.frame_duration_ms or 20),
                             int(bool(settings.use_vbr)), int(bool(settings.use_silence_gate)),
                             CODEC_PCM if codec == "pcm" else CODEC_OPUS, int(synthetic_silence_frames))
        h = L.sk_audio_create()
        rc = L.sk_audio_start(h, ctypes.byref(s), callback, None)
        if rc != 0:
            msg = L.sk_audio_error(h).decode(errors="replace")
            L.sk_audio_destroy(h)
            raise RuntimeError(f"pcmflux: {msg or 'audio capture failed'} ({rc})")
        self._h = h

    def stats(self) -> dict:
        """Counters of the running capture, or of the last one once stopped."""
        if self._h is None:
            return dict(self._final)
        out = (ctypes.c_double * 4)()
        _native().sk_audio_stats(self._h, out, 4)
        return {"frames": int(out[0]), "packets": int(out[1]), "bytes": int(out[2]), "gated": int(out[3])}

    def stop_capture(self) -> None:
        if self._h is not None:
            L = _native()
            L.sk_audio_stop(self._h)
            self._final = self.stats()
            L.sk_audio_destroy(self._h)
            self._h = None
