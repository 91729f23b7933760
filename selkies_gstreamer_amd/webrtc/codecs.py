"""Media codecs of the WebRTC stack and their RTP parameters.

Parity target: the vendored aiortc codec registry of the reference
(``src/selkies/webrtc/codecs/__init__.py``: ``CODECS``, ``get_encoder``,
``get_decoder``; ``g711.py``, ``g722.py``, ``h264.py``, ``opus.py``). The heavy
lifting is native: H.264 is the gfx950 HIP encoder (ops/native.H264Encoder),
G.711 / G.722 are host C++ (csrc/codec/telephony.cpp), Opus uses libopus when
the system has it (pcmflux).

Audio frames are int16 numpy arrays (mono). Encoders return one RTP payload per
``encode`` call; decoders take one payload.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from ..ops.native import lib as _native


@dataclass(frozen=True)
class RtpCodec:
    kind: str          # "audio" | "video"
    name: str          # rtpmap encoding name
    clock_rate: int
    channels: int = 1
    payload_type: int = 0
    fmtp: str = ""
    rtcp_fb: tuple = field(default_factory=tuple)

    @property
    def rtpmap(self) -> str:
        base = f"{self.name}/{self.clock_rate}"
        return base + (f"/{self.channels}" if self.kind == "audio" and self.channels > 1 else "")


# Offered in this order (the static payload types of RFC 3551 for PCMU/PCMA/G722).
CODECS = {
    "audio": [
        RtpCodec("audio", "opus", 48000, 2, 111, "minptime=10;useinbandfec=1;stereo=1;sprop-stereo=1"),
        RtpCodec("audio", "G722", 8000, 1, 9),   # RFC 3551: G.722 advertises 8000 for historic reasons
        RtpCodec("audio", "PCMU", 8000, 1, 0),
        RtpCodec("audio", "PCMA", 8000, 1, 8),
    ],
    "video": [
        RtpCodec("video", "H264", 90000, 1, 97,
                 "level-asymmetry-allowed=1;packetization-mode=1;profile-level-id=42e01f",
                 ("nack", "nack pli", "ccm fir", "goog-remb")),
    ],
}


def find_codec(kind: str, name: str) -> RtpCodec:
    for c in CODECS[kind]:
        if c.name.lower() == name.lower():
            return c
    raise KeyError(f"unsupported {kind} codec {name}")


def _api():
    L = _native()
    if not getattr(L, "_sk_tel_init", False):
        i16p = ctypes.POINTER(ctypes.c_int16)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.sk_g711_encode.argtypes = [ctypes.c_int, i16p, ctypes.c_int, u8p]
        L.sk_g711_decode.argtypes = [ctypes.c_int, u8p, ctypes.c_int, i16p]
        L.sk_g722_create.restype = ctypes.c_void_p
        L.sk_g722_destroy.argtypes = [ctypes.c_void_p]
        L.sk_g722_encode.argtypes = [ctypes.c_void_p, i16p, ctypes.c_int, u8p]
        L.sk_g722_decode.argtypes = [ctypes.c_void_p, u8p, ctypes.c_int, i16p]
        L._sk_tel_init = True
    return L


def _i16(a: np.ndarray):
    a = np.ascontiguousarray(a, dtype=np.int16)
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_int16))


class G711Encoder:
    """20 ms of 8 kHz mono -> 160-byte PCMU/PCMA payload."""

    def __init__(self, alaw: bool = False):
        self.alaw = int(alaw)

    def encode(self, pcm: np.ndarray) -> bytes:
        a, p = _i16(pcm)
        out = (ctypes.c_uint8 * a.size)()
        _api().sk_g711_encode(self.alaw, p, a.size, out)
        return bytes(out)


class G711Decoder:
    def __init__(self, alaw: bool = False):
        self.alaw = int(alaw)

    def decode(self, payload: bytes) -> np.ndarray:
        buf = (ctypes.c_uint8 * len(payload)).from_buffer_copy(payload)
        out = np.empty(len(payload), np.int16)
        _api().sk_g711_decode(self.alaw, buf, len(payload), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)))
        return out


class G722Encoder:
    """16 kHz mono PCM (even sample count) -> G.722 64 kbit/s payload (stateful)."""

    def __init__(self):
        self._h = _api().sk_g722_create()

    def encode(self, pcm: np.ndarray) -> bytes:
        a, p = _i16(pcm)
        if a.size % 2:
            raise ValueError("G.722 encodes pairs of 16 kHz samples")
        out = (ctypes.c_uint8 * (a.size // 2))()
        n = _api().sk_g722_encode(self._h, p, a.size, out)
        return bytes(out[:n])

    def __del__(self):
        if getattr(self, "_h", None):
            _api().sk_g722_destroy(self._h)
            self._h = None


class G722Decoder:
    def __init__(self):
        self._h = _api().sk_g722_create()

    def decode(self, payload: bytes) -> np.ndarray:
        buf = (ctypes.c_uint8 * len(payload)).from_buffer_copy(payload)
        out = np.empty(2 * len(payload), np.int16)
        _api().sk_g722_decode(self._h, buf, len(payload), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)))
        return out

    def __del__(self):
        if getattr(self, "_h", None):
            _api().sk_g722_destroy(self._h)
            self._h = None


def get_encoder(codec: RtpCodec):
    n = codec.name.lower()
    if n == "pcmu":
        return G711Encoder(alaw=False)
    if n == "pcma":
        return G711Encoder(alaw=True)
    if n == "g722":
        return G722Encoder()
    raise ValueError(f"no in-process encoder for {codec.name} (H.264: ops.native.H264Encoder, opus: pcmflux)")


def get_decoder(codec: RtpCodec):
    n = codec.name.lower()
    if n == "pcmu":
        return G711Decoder(alaw=False)
    if n == "pcma":
        return G711Decoder(alaw=True)
    if n == "g722":
        return G722Decoder()
    raise ValueError(f"no in-process decoder for {codec.name}")
