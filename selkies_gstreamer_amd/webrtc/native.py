"""ctypes binding of ``libselkies_rtc.so`` (csrc/rtc/rtc.cpp): DTLS-SRTP,
SRTP/SRTCP, RTP packetisation and CRC32c."""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path

_LIB_PATH = Path(__file__).resolve().parents[1] / "_lib" / "libselkies_rtc.so"
_lib = None
_mu = threading.Lock()


class RtpParams(ctypes.Structure):
    _fields_ = [("ssrc", ctypes.c_uint32), ("timestamp", ctypes.c_uint32), ("seq", ctypes.c_uint16),
                ("payload_type", ctypes.c_uint8), ("marker", ctypes.c_uint8), ("mtu", ctypes.c_int),
                ("playout_ext_id", ctypes.c_int), ("playout_min", ctypes.c_int), ("playout_max", ctypes.c_int)]


def lib():
    """Loads the library, building it in-tree first if it is missing."""
    global _lib
    with _mu:
        if _lib is not None:
            return _lib
        if not _LIB_PATH.exists():
            from selkies_gstreamer_amd.ops.build import build_rtc
            build_rtc()
        L = ctypes.CDLL(str(_LIB_PATH))
        vp, u8p, i32 = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int
        sig = {
            "rtc_dtls_create": (vp, [i32]), "rtc_dtls_destroy": (None, [vp]),
            "rtc_dtls_set_role": (None, [vp, i32]),
            "rtc_dtls_fingerprint": (i32, [vp, ctypes.c_char_p, i32]),
            "rtc_dtls_set_remote_fingerprint": (None, [vp, ctypes.c_char_p]),
            "rtc_dtls_start": (i32, [vp]), "rtc_dtls_feed": (i32, [vp, u8p, i32]),
            "rtc_dtls_pop": (i32, [vp, ctypes.c_void_p, i32]), "rtc_dtls_read": (i32, [vp, ctypes.c_void_p, i32]),
            "rtc_dtls_write": (i32, [vp, u8p, i32]), "rtc_dtls_state": (i32, [vp]),
            "rtc_dtls_timeout_ms": (i32, [vp]), "rtc_dtls_on_timeout": (i32, [vp]),
            "rtc_dtls_srtp_keys": (i32, [vp, ctypes.c_void_p, ctypes.c_void_p]),
            "rtc_dtls_error": (ctypes.c_char_p, [vp]), "rtc_dtls_close": (None, [vp]),
            "rtc_srtp_create": (vp, [u8p]), "rtc_srtp_destroy": (None, [vp]),
            "rtc_srtp_protect_rtp": (i32, [vp, ctypes.c_void_p, i32]),
            "rtc_srtp_protect_rtcp": (i32, [vp, ctypes.c_void_p, i32]),
            "rtc_srtp_unprotect_rtp": (i32, [vp, ctypes.c_void_p, i32]),
            "rtc_srtp_unprotect_rtcp": (i32, [vp, ctypes.c_void_p, i32]),
            "rtc_srtp_session_keys": (None, [vp, ctypes.c_void_p]),
            "rtc_h264_packetize": (i32, [vp, u8p, i32, ctypes.POINTER(RtpParams), ctypes.c_void_p, i32,
                                         ctypes.POINTER(ctypes.c_int), i32]),
            "rtc_h265_packetize": (i32, [vp, u8p, i32, ctypes.POINTER(RtpParams), ctypes.c_void_p, i32,
                                         ctypes.POINTER(ctypes.c_int), i32]),
            "rtc_av1_packetize": (i32, [vp, u8p, i32, ctypes.POINTER(RtpParams), ctypes.c_void_p, i32,
                                        ctypes.POINTER(ctypes.c_int), i32]),
            "rtc_rtp_packet": (i32, [vp, u8p, i32, ctypes.POINTER(RtpParams), ctypes.c_void_p, i32]),
            "rtc_crc32c": (ctypes.c_uint32, [u8p, i32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype, f.argtypes = res, args
        _lib = L
        return L


class DtlsError(Exception):
    pass


class Dtls:
    """One DTLS association. role 'server' (setup:passive) or 'client' (setup:active)."""

    NEW, CONNECTING, CONNECTED, FAILED, CLOSED = range(5)

    def __init__(self, role: str):
        self._L = lib()
        self.role = role
        self._h = self._L.rtc_dtls_create(1 if role == "server" else 0)
        if self.state == self.FAILED:
            raise DtlsError(self.error)
        buf = ctypes.create_string_buffer(128)
        n = self._L.rtc_dtls_fingerprint(self._h, buf, 128)
        self.fingerprint = buf.value[:n].decode()
        self._buf = ctypes.create_string_buffer(65536)

    def set_role(self, role: str) -> None:
        """Switches client/server before the handshake (same certificate and fingerprint)."""
        self.role = role
        self._L.rtc_dtls_set_role(self._h, 1 if role == "server" else 0)

    def set_remote_fingerprint(self, fp: str) -> None:
        self._L.rtc_dtls_set_remote_fingerprint(self._h, fp.encode())

    @property
    def state(self) -> int:
        return self._L.rtc_dtls_state(self._h)

    @property
    def error(self) -> str:
        return self._L.rtc_dtls_error(self._h).decode()

    def start(self) -> list[bytes]:
        if self._L.rtc_dtls_start(self._h) < 0:
            raise DtlsError(self.error)
        return self.pop()

    def feed(self, datagram: bytes) -> bool:
        """Returns True when this datagram completed the handshake."""
        r = self._L.rtc_dtls_feed(self._h, datagram, len(datagram))
        if r < 0:
            raise DtlsError(self.error)
        return r == 1

    def pop(self) -> list[bytes]:
        out = []
        while True:
            n = self._L.rtc_dtls_pop(self._h, self._buf, len(self._buf))
            if n <= 0:
                return out
            out.append(self._buf.raw[:n])

    def read(self) -> list[bytes]:
        out = []
        while True:
            n = self._L.rtc_dtls_read(self._h, self._buf, len(self._buf))
            if n <= 0:
                return out
            out.append(self._buf.raw[:n])

    def write(self, data: bytes) -> list[bytes]:
        if self._L.rtc_dtls_write(self._h, data, len(data)) < 0:
            raise DtlsError("write on a DTLS association that is not connected")
        return self.pop()

    def timeout_ms(self) -> int:
        return self._L.rtc_dtls_timeout_ms(self._h)

    def on_timeout(self) -> list[bytes]:
        self._L.rtc_dtls_on_timeout(self._h)
        return self.pop()

    def srtp_keys(self) -> tuple[bytes, bytes]:
        loc, rem = ctypes.create_string_buffer(30), ctypes.create_string_buffer(30)
        if self._L.rtc_dtls_srtp_keys(self._h, loc, rem) != 0:
            raise DtlsError("SRTP keys are not available before the handshake completes")
        return loc.raw, rem.raw

    def close(self) -> list[bytes]:
        if self._h:
            self._L.rtc_dtls_close(self._h)
            return self.pop()
        return []

    def __del__(self):
        try:
            if self._h:
                self._L.rtc_dtls_destroy(self._h)
                self._h = None
        except Exception:
            pass


class Srtp:
    """One direction's SRTP/SRTCP context (AES_CM_128_HMAC_SHA1_80)."""

    def __init__(self, key_salt: bytes):
        if len(key_salt) != 30:
            raise ValueError("SRTP master key + salt must be 30 bytes")
        self._L = lib()
        self._h = self._L.rtc_srtp_create(key_salt)
        self._buf = ctypes.create_string_buffer(65536)

    @property
    def handle(self):
        return self._h

    def _run(self, fn, pkt: bytes) -> bytes | None:
        ctypes.memmove(self._buf, pkt, len(pkt))
        n = fn(self._h, self._buf, len(pkt))
        return self._buf.raw[:n] if n >= 0 else None

    def protect_rtp(self, pkt: bytes) -> bytes:
        return self._run(self._L.rtc_srtp_protect_rtp, pkt)

    def protect_rtcp(self, pkt: bytes) -> bytes:
        return self._run(self._L.rtc_srtp_protect_rtcp, pkt)

    def unprotect_rtp(self, pkt: bytes) -> bytes | None:
        return self._run(self._L.rtc_srtp_unprotect_rtp, pkt)

    def unprotect_rtcp(self, pkt: bytes) -> bytes | None:
        return self._run(self._L.rtc_srtp_unprotect_rtcp, pkt)

    def session_keys(self) -> bytes:
        out = ctypes.create_string_buffer(100)
        self._L.rtc_srtp_session_keys(self._h, out)
        return out.raw

    def __del__(self):
        try:
            if self._h:
                self._L.rtc_srtp_destroy(self._h)
                self._h = None
        except Exception:
            pass


class RtpPacketizer:
    """Per-stream RTP state (SSRC, sequence numbers) + native packetisation."""

    def __init__(self, ssrc: int, payload_type: int, mtu: int = 1200, seq: int = 0):
        self._L = lib()
        self.params = RtpParams(ssrc, 0, seq & 0xFFFF, payload_type, 0, mtu, 0, 0, 0)
        self._out = ctypes.create_string_buffer(1 << 20)
        self._lens = (ctypes.c_int * 4096)()

    def set_playout_delay(self, ext_id: int, min_ms: int = 0, max_ms: int = 0) -> None:
        """Adds the playout-delay header extension (negotiated extmap id) to every packet;
        ext_id 0 removes it. Delays are carried in 10 ms units (max 40.95 s)."""
        self.params.playout_ext_id = ext_id
        self.params.playout_min = max(0, min(4095, min_ms // 10))
        self.params.playout_max = max(0, min(4095, max_ms // 10))

    @property
    def seq(self) -> int:
        return self.params.seq

    def h264(self, annexb: bytes, timestamp: int, srtp: Srtp | None = None) -> list[bytes]:
        self.params.timestamp = timestamp & 0xFFFFFFFF
        need = len(annexb) + 64 * (len(annexb) // 1000 + 8)
        if need > len(self._out):
            self._out = ctypes.create_string_buffer(need * 2)
        n = self._L.rtc_h264_packetize(srtp.handle if srtp else None, annexb, len(annexb),
                                       ctypes.byref(self.params), self._out, len(self._out), self._lens,
                                       len(self._lens))
        if n < 0:
            raise ValueError("access unit too large for the packetiser buffers")
        out, off, raw = [], 0, self._out.raw
        for i in range(n):
            out.append(raw[off:off + self._lens[i]])
            off += self._lens[i]
        return out

    def h265(self, annexb: bytes, timestamp: int, srtp: Srtp | None = None) -> list[bytes]:
        """RFC 7798 payloads (single NAL / aggregation / fragmentation units) of one access unit."""
        return self._packetize(self._L.rtc_h265_packetize, annexb, timestamp, srtp)

    def av1(self, tu: bytes, timestamp: int, srtp: Srtp | None = None) -> list[bytes]:
        """AV1 RTP payloads (aggregation header, OBU elements, fragments) of one temporal unit."""
        return self._packetize(self._L.rtc_av1_packetize, tu, timestamp, srtp)

    def _packetize(self, fn, annexb: bytes, timestamp: int, srtp: Srtp | None) -> list[bytes]:
        self.params.timestamp = timestamp & 0xFFFFFFFF
        need = len(annexb) + 64 * (len(annexb) // 1000 + 8)
        if need > len(self._out):
            self._out = ctypes.create_string_buffer(need * 2)
        n = fn(srtp.handle if srtp else None, annexb, len(annexb), ctypes.byref(self.params), self._out,
               len(self._out), self._lens, len(self._lens))
        if n < 0:
            raise ValueError("access unit too large for the packetiser buffers")
        out, off, raw = [], 0, self._out.raw
        for i in range(n):
            out.append(raw[off:off + self._lens[i]])
            off += self._lens[i]
        return out

    def raw(self, payload: bytes, timestamp: int, marker: bool = False, srtp: Srtp | None = None) -> bytes:
        self.params.timestamp = timestamp & 0xFFFFFFFF
        self.params.marker = 1 if marker else 0
        n = self._L.rtc_rtp_packet(srtp.handle if srtp else None, payload, len(payload), ctypes.byref(self.params),
                                   self._out, len(self._out))
        if n < 0:
            raise ValueError("payload too large")
        return self._out.raw[:n]


def crc32c(data: bytes) -> int:
    return lib().rtc_crc32c(data, len(data))
