"""STUN messages (RFC 5389) with the ICE (RFC 8445) and TURN (RFC 5766)
attributes — the wire format under the ICE agent (reference: the vendored
aiortc relies on aioice, webrtc/rtcicetransport.py; webrtcbin uses libnice)."""
from __future__ import annotations

import hashlib
import hmac
import ipaddress
import os
import struct
import zlib
from dataclasses import dataclass, field

MAGIC = 0x2112A442
FINGERPRINT_XOR = 0x5354554E

# methods
BINDING, ALLOCATE, REFRESH, SEND, DATA, CREATE_PERMISSION, CHANNEL_BIND = 0x001, 0x003, 0x004, 0x006, 0x007, 0x008, 0x009
# classes
REQUEST, INDICATION, SUCCESS, ERROR = 0x000, 0x010, 0x100, 0x110

# attributes
MAPPED_ADDRESS = 0x0001
USERNAME = 0x0006
MESSAGE_INTEGRITY = 0x0008
ERROR_CODE = 0x0009
CHANNEL_NUMBER = 0x000C
LIFETIME = 0x000D
XOR_PEER_ADDRESS = 0x0012
DATA_ATTR = 0x0013
REALM = 0x0014
NONCE = 0x0015
XOR_RELAYED_ADDRESS = 0x0016
REQUESTED_TRANSPORT = 0x0019
XOR_MAPPED_ADDRESS = 0x0020
PRIORITY = 0x0024
USE_CANDIDATE = 0x0025
SOFTWARE = 0x8022
FINGERPRINT = 0x8028
ICE_CONTROLLED = 0x8029
ICE_CONTROLLING = 0x802A

_ADDRESS_ATTRS = {MAPPED_ADDRESS}
_XOR_ADDRESS_ATTRS = {XOR_MAPPED_ADDRESS, XOR_PEER_ADDRESS, XOR_RELAYED_ADDRESS}
_U32_ATTRS = {PRIORITY, LIFETIME, FINGERPRINT}
_U64_ATTRS = {ICE_CONTROLLED, ICE_CONTROLLING}
_STR_ATTRS = {USERNAME, REALM, NONCE, SOFTWARE}


def is_stun(data: bytes) -> bool:
    """RFC 7983 demultiplexing: first byte 0..3 and the magic cookie."""
    return len(data) >= 20 and data[0] < 4 and struct.unpack_from("!I", data, 4)[0] == MAGIC


def _pad(n: int) -> int:
    return (4 - n % 4) % 4


def _enc_addr(addr, xor: bool, tid: bytes) -> bytes:
    host, port = addr[0], addr[1]
    ip = ipaddress.ip_address(host)
    fam = 1 if ip.version == 4 else 2
    raw = ip.packed
    if xor:
        port ^= MAGIC >> 16
        key = struct.pack("!I", MAGIC) + (tid if fam == 2 else b"")
        raw = bytes(a ^ b for a, b in zip(raw, key))
    return struct.pack("!BBH", 0, fam, port) + raw


def _dec_addr(v: bytes, xor: bool, tid: bytes):
    fam, port = v[1], struct.unpack_from("!H", v, 2)[0]
    raw = v[4:8] if fam == 1 else v[4:20]
    if xor:
        port ^= MAGIC >> 16
        key = struct.pack("!I", MAGIC) + (tid if fam == 2 else b"")
        raw = bytes(a ^ b for a, b in zip(raw, key))
    return (str(ipaddress.ip_address(raw)), port)


@dataclass
class Message:
    method: int
    cls: int
    tid: bytes = field(default_factory=lambda: os.urandom(12))
    attrs: dict = field(default_factory=dict)

    @property
    def msg_type(self) -> int:
        m, c = self.method, self.cls
        return (m & 0x000F) | ((m & 0x0070) << 1) | ((m & 0x0F80) << 2) | c

    def encode(self, integrity_key: bytes | None = None, fingerprint: bool = True) -> bytes:
        body = b""
        for t, v in self.attrs.items():
            if t in (MESSAGE_INTEGRITY, FINGERPRINT):
                continue
            if t in _XOR_ADDRESS_ATTRS:
                raw = _enc_addr(v, True, self.tid)
            elif t in _ADDRESS_ATTRS:
                raw = _enc_addr(v, False, self.tid)
            elif t in _U32_ATTRS:
                raw = struct.pack("!I", v)
            elif t in _U64_ATTRS:
                raw = struct.pack("!Q", v)
            elif t in _STR_ATTRS:
                raw = v.encode() if isinstance(v, str) else v
            elif t == ERROR_CODE:
                code, reason = v
                raw = struct.pack("!HBB", 0, code // 100, code % 100) + reason.encode()
            elif t == REQUESTED_TRANSPORT:
                raw = struct.pack("!B3x", v)
            elif t == CHANNEL_NUMBER:
                raw = struct.pack("!H2x", v)
            elif t == USE_CANDIDATE:
                raw = b""
            else:
                raw = bytes(v)
            body += struct.pack("!HH", t, len(raw)) + raw + b"\x00" * _pad(len(raw))
        if integrity_key is not None:
            hdr = struct.pack("!HHI", self.msg_type, len(body) + 24, MAGIC) + self.tid
            mac = hmac.new(integrity_key, hdr + body, hashlib.sha1).digest()
            body += struct.pack("!HH", MESSAGE_INTEGRITY, 20) + mac
        if fingerprint:
            hdr = struct.pack("!HHI", self.msg_type, len(body) + 8, MAGIC) + self.tid
            crc = (zlib.crc32(hdr + body) ^ FINGERPRINT_XOR) & 0xFFFFFFFF
            body += struct.pack("!HHI", FINGERPRINT, 4, crc)
        return struct.pack("!HHI", self.msg_type, len(body), MAGIC) + self.tid + body


class StunError(ValueError):
    pass


def decode(data: bytes) -> tuple[Message, dict]:
    """Returns (message, offsets) where offsets maps attribute type -> byte offset
    (used to verify MESSAGE-INTEGRITY / FINGERPRINT)."""
    if not is_stun(data):
        raise StunError("not a STUN message")
    mt, ln = struct.unpack_from("!HH", data, 0)
    if 20 + ln > len(data):
        raise StunError("truncated STUN message")
    tid = data[8:20]
    cls = mt & 0x0110
    m = mt & ~0x0110
    method = (m & 0x000F) | ((m & 0x00E0) >> 1) | ((m & 0x3E00) >> 2)
    msg = Message(method, cls, tid, {})
    offs = {}
    pos = 20
    while pos + 4 <= 20 + ln:
        t, alen = struct.unpack_from("!HH", data, pos)
        v = data[pos + 4:pos + 4 + alen]
        offs[t] = pos
        if t in _XOR_ADDRESS_ATTRS:
            msg.attrs[t] = _dec_addr(v, True, tid)
        elif t in _ADDRESS_ATTRS:
            msg.attrs[t] = _dec_addr(v, False, tid)
        elif t in _U32_ATTRS and alen == 4:
            msg.attrs[t] = struct.unpack("!I", v)[0]
        elif t in _U64_ATTRS and alen == 8:
            msg.attrs[t] = struct.unpack("!Q", v)[0]
        elif t in _STR_ATTRS:
            msg.attrs[t] = v.decode("utf-8", "replace")
        elif t == ERROR_CODE and alen >= 4:
            msg.attrs[t] = ((v[2] & 7) * 100 + v[3], v[4:].decode("utf-8", "replace"))
        elif t == USE_CANDIDATE:
            msg.attrs[t] = True
        elif t == CHANNEL_NUMBER and alen >= 2:
            msg.attrs[t] = struct.unpack_from("!H", v)[0]
        else:
            msg.attrs[t] = bytes(v)
        pos += 4 + alen + _pad(alen)
    return msg, offs


def check_integrity(data: bytes, offs: dict, key: bytes) -> bool:
    pos = offs.get(MESSAGE_INTEGRITY)
    if pos is None:
        return False
    mt = struct.unpack_from("!H", data, 0)[0]
    hdr = struct.pack("!HHI", mt, pos - 20 + 24, MAGIC) + data[8:20]
    mac = hmac.new(key, hdr + data[20:pos], hashlib.sha1).digest()
    return hmac.compare_digest(mac, data[pos + 4:pos + 24])


def check_fingerprint(data: bytes, offs: dict) -> bool:
    pos = offs.get(FINGERPRINT)
    if pos is None:
        return True  # optional
    mt = struct.unpack_from("!H", data, 0)[0]
    hdr = struct.pack("!HHI", mt, pos - 20 + 8, MAGIC) + data[8:20]
    crc = (zlib.crc32(hdr + data[20:pos]) ^ FINGERPRINT_XOR) & 0xFFFFFFFF
    return crc == struct.unpack_from("!I", data, pos + 4)[0]


def long_term_key(username: str, realm: str, password: str) -> bytes:
    """TURN long-term credential key (RFC 5389 §15.4)."""
    return hashlib.md5(f"{username}:{realm}:{password}".encode()).digest()
