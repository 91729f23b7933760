"""pcmflux-compatible audio capture: PulseAudio monitor -> Opus packets.

Contract of the reference server (selkies.py:64-70, 939-1070): fill an
``AudioCaptureSettings``, wrap a function in ``AudioChunkCallback`` and call
``AudioCapture().start_capture(settings, cb)``; the callback receives an
``AudioChunkEncodeResult`` pointer (``.data``/``.size`` = one Opus packet) from
the capture thread, and the server broadcasts ``0x01 0x00 + opus`` frames.

Audio is a few hundred kbit/s and needs no GPU; the capture loop runs in a
native-released thread that calls libpulse-simple (``pa_simple_read``) and
libopus (``opus_encode``) through ctypes, so the GIL is held only to hand a
finished packet to the callback. Both libraries are resolved at ``start_capture``
time; when either is missing (as in this build image) ``available()`` is False
and ``start_capture`` raises, which the server treats as "audio unavailable",
the same as the reference when its pcmflux import fails.
"""
from __future__ import annotations

import ctypes
import ctypes.util
import threading
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

# libpulse / libopus constants
_PA_SAMPLE_S16LE = 3
_PA_STREAM_RECORD = 2
_OPUS_APPLICATION_AUDIO = 2049
_OPUS_SET_BITRATE_REQUEST = 4002
_OPUS_SET_VBR_REQUEST = 4006


class _PaSampleSpec(ctypes.Structure):
    _fields_ = [("format", ctypes.c_int), ("rate", ctypes.c_uint32), ("channels", ctypes.c_uint8)]


class _PaBufferAttr(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("maxlength", "tlength", "prebuf", "minreq", "fragsize")]


def _load(names) -> Optional[ctypes.CDLL]:
    for n in names:
        path = ctypes.util.find_library(n) or None
        for cand in ([path] if path else []) + [f"lib{n}.so.0"]:
            try:
                return ctypes.CDLL(cand)
            except OSError:
                continue
    return None


def _libs():
    pa = _load(["pulse-simple"])
    opus = _load(["opus"])
    return pa, opus


def available() -> bool:
    pa, opus = _libs()
    return pa is not None and opus is not None


class AudioCapture:
    def __init__(self):
        self._thread: Optional[threading.Thread] = None
        self._stop = threading.Event()
        self._cb = None
        self._err: Optional[str] = None

    def start_capture(self, settings: AudioCaptureSettings, callback) -> None:
        pa, opus = _libs()
        if pa is None or opus is None:
            raise RuntimeError("pcmflux: libpulse-simple and libopus are required for audio capture")
        if not isinstance(callback, AudioChunkCallback):
            callback = AudioChunkCallback(callback)
        self._cb = callback
        rate, ch = int(settings.sample_rate or 48000), int(settings.channels or 2)
        frame = rate * int(settings.frame_duration_ms or 20) // 1000
        spec = _PaSampleSpec(_PA_SAMPLE_S16LE, rate, ch)
        attr = _PaBufferAttr(0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, frame * ch * 2)
        pa.pa_simple_new.restype = ctypes.c_void_p
        pa.pa_simple_new.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                     ctypes.c_char_p, ctypes.POINTER(_PaSampleSpec), ctypes.c_void_p,
                                     ctypes.POINTER(_PaBufferAttr), ctypes.POINTER(ctypes.c_int)]
        pa.pa_simple_read.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_int)]
        pa.pa_simple_free.argtypes = [ctypes.c_void_p]
        err = ctypes.c_int(0)
        stream = pa.pa_simple_new(None, b"selkies", _PA_STREAM_RECORD, settings.device_name, b"desktop-audio",
                                  ctypes.byref(spec), None, ctypes.byref(attr), ctypes.byref(err))
        if not stream:
            raise RuntimeError(f"pcmflux: pa_simple_new failed ({err.value})")
        opus.opus_encoder_create.restype = ctypes.c_void_p
        opus.opus_encoder_create.argtypes = [ctypes.c_int32, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        opus.opus_encode.restype = ctypes.c_int32
        opus.opus_encode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int32]
        opus.opus_encoder_destroy.argtypes = [ctypes.c_void_p]
        enc = opus.opus_encoder_create(rate, ch, _OPUS_APPLICATION_AUDIO, ctypes.byref(err))
        if not enc:
            pa.pa_simple_free(stream)
            raise RuntimeError(f"pcmflux: opus_encoder_create failed ({err.value})")
        opus.opus_encoder_ctl(ctypes.c_void_p(enc), _OPUS_SET_BITRATE_REQUEST, ctypes.c_int32(settings.opus_bitrate))
        opus.opus_encoder_ctl(ctypes.c_void_p(enc), _OPUS_SET_VBR_REQUEST, ctypes.c_int32(int(settings.use_vbr)))
        gate = bool(settings.use_silence_gate)
        self._stop.clear()

        def run():
            pcm = (ctypes.c_int16 * (frame * ch))()
            out = (ctypes.c_ubyte * 4000)()
            res = AudioChunkEncodeResult()
            try:
                while not self._stop.is_set():
                    if pa.pa_simple_read(stream, pcm, ctypes.sizeof(pcm), ctypes.byref(err)) < 0:
                        self._err = f"pa_simple_read failed ({err.value})"
                        break
                    if gate and not any(pcm):
                        continue
                    n = opus.opus_encode(ctypes.c_void_p(enc), pcm, frame, out, len(out))
                    if n > 0:
                        res.size = n
                        res.data = ctypes.cast(out, ctypes.POINTER(ctypes.c_ubyte))
                        self._cb(ctypes.byref(res), None)
            finally:
                opus.opus_encoder_destroy(ctypes.c_void_p(enc))
                pa.pa_simple_free(stream)

        self._thread = threading.Thread(target=run, name="pcmflux-capture", daemon=True)
        self._thread.start()

    def stop_capture(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2.0)
            self._thread = None
