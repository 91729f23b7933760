"""RTP / RTCP helpers: headers, sender reports, feedback parsing (PLI, FIR,
NACK, REMB, receiver reports) and an RFC 6184 H.264 depacketiser.

Reference: the vendored aiortc webrtc/rtp.py (RTCP packet classes,
unwrap/wrap of NACK and REMB) and webrtc/codecs/h264.py (depacketiser);
packetisation itself is native (rtc_h264_packetize, csrc/rtc/rtc.cpp).
"""
from __future__ import annotations

import struct
import time
from dataclasses import dataclass, field

RTCP_SR, RTCP_RR, RTCP_SDES, RTCP_BYE, RTCP_RTPFB, RTCP_PSFB = 200, 201, 202, 203, 205, 206
FB_NACK, FB_TWCC = 1, 15
FB_PLI, FB_FIR, FB_REMB = 1, 4, 15

NTP_EPOCH = 2208988800


def is_rtcp(data: bytes) -> bool:
    """RFC 5761 demultiplexing of RTCP from RTP on one port."""
    return len(data) >= 2 and 192 <= data[1] <= 223


@dataclass
class RtpHeader:
    payload_type: int
    seq: int
    timestamp: int
    ssrc: int
    marker: bool
    header_len: int


def parse_rtp(data: bytes) -> RtpHeader | None:
    if len(data) < 12 or data[0] >> 6 != 2:
        return None
    cc = data[0] & 15
    hl = 12 + 4 * cc
    if data[0] & 0x10:
        if len(data) < hl + 4:
            return None
        hl += 4 + 4 * struct.unpack_from("!H", data, hl + 2)[0]
    if hl > len(data):
        return None
    seq, ts, ssrc = struct.unpack_from("!HII", data, 2)
    return RtpHeader(data[1] & 0x7F, seq, ts, ssrc, bool(data[1] & 0x80), hl)


def ntp_now() -> tuple[int, int]:
    t = time.time() + NTP_EPOCH
    return int(t) & 0xFFFFFFFF, int((t % 1) * (1 << 32)) & 0xFFFFFFFF


def sender_report(ssrc: int, rtp_ts: int, packets: int, octets: int, cname: str = "selkies") -> bytes:
    """SR + SDES(CNAME) compound packet."""
    hi, lo = ntp_now()
    sr = struct.pack("!BBHIIIIII", 0x80, RTCP_SR, 6, ssrc, hi, lo, rtp_ts & 0xFFFFFFFF, packets & 0xFFFFFFFF,
                     octets & 0xFFFFFFFF)
    c = cname.encode()[:255]
    item = struct.pack("!IBB", ssrc, 1, len(c)) + c + b"\x00"
    item += b"\x00" * ((4 - len(item) % 4) % 4)
    sdes = struct.pack("!BBH", 0x81, RTCP_SDES, len(item) // 4) + item
    return sr + sdes


def pli(sender_ssrc: int, media_ssrc: int) -> bytes:
    return struct.pack("!BBHII", 0x80 | FB_PLI, RTCP_PSFB, 2, sender_ssrc, media_ssrc)


def fir(sender_ssrc: int, media_ssrc: int, seq: int) -> bytes:
    return struct.pack("!BBHIIIBxxx", 0x80 | FB_FIR, RTCP_PSFB, 4, sender_ssrc, 0, media_ssrc, seq & 0xFF)


def nack(sender_ssrc: int, media_ssrc: int, lost: list[int]) -> bytes:
    fci, lost = b"", sorted(set(lost))
    i = 0
    while i < len(lost):
        pid, blp = lost[i], 0
        j = i + 1
        while j < len(lost) and 0 < ((lost[j] - pid) & 0xFFFF) <= 16:
            blp |= 1 << (((lost[j] - pid) & 0xFFFF) - 1)
            j += 1
        fci += struct.pack("!HH", pid, blp)
        i = j
    return struct.pack("!BBHII", 0x80 | FB_NACK, RTCP_RTPFB, 2 + len(fci) // 4, sender_ssrc, media_ssrc) + fci


def remb(sender_ssrc: int, bitrate: int, ssrcs: list[int]) -> bytes:
    exp = 0
    mant = bitrate
    while mant >= (1 << 18):
        mant >>= 1
        exp += 1
    body = b"REMB" + struct.pack("!BBBB", len(ssrcs), (exp << 2) | (mant >> 16), (mant >> 8) & 0xFF, mant & 0xFF)
    body += b"".join(struct.pack("!I", s) for s in ssrcs)
    return struct.pack("!BBHII", 0x80 | FB_REMB, RTCP_PSFB, 2 + len(body) // 4, sender_ssrc, 0) + body


def receiver_report(ssrc: int, media_ssrc: int, fraction_lost: int, cum_lost: int, highest_seq: int,
                    jitter: int = 0) -> bytes:
    return struct.pack("!BBHIIIIIII", 0x81, RTCP_RR, 7, ssrc, media_ssrc,
                       ((fraction_lost & 0xFF) << 24) | (cum_lost & 0xFFFFFF), highest_seq & 0xFFFFFFFF, jitter,
                       0, 0)


@dataclass
class RtcpFeedback:
    pli: set = field(default_factory=set)          # media ssrcs that asked for a keyframe (PLI or FIR)
    nacks: dict = field(default_factory=dict)      # media ssrc -> [lost seqs]
    remb_bps: int | None = None
    reports: list = field(default_factory=list)    # (ssrc, fraction_lost, cum_lost, highest_seq, jitter, lsr, dlsr)
    bye: bool = False


def parse_rtcp(data: bytes) -> RtcpFeedback:
    fb = RtcpFeedback()
    pos = 0
    while pos + 4 <= len(data):
        v_p_c, pt, ln = struct.unpack_from("!BBH", data, pos)
        end = pos + 4 * (ln + 1)
        if v_p_c >> 6 != 2 or end > len(data):
            break
        fmt = v_p_c & 31
        if pt in (RTCP_SR, RTCP_RR):
            off = pos + 8 + (20 if pt == RTCP_SR else 0)
            for _ in range(fmt):
                if off + 24 > end:
                    break
                ssrc, lost_word, hs, jit, lsr, dlsr = struct.unpack_from("!IIIIII", data, off)
                cum = lost_word & 0xFFFFFF
                fb.reports.append((ssrc, lost_word >> 24, cum, hs, jit, lsr, dlsr))
                off += 24
        elif pt == RTCP_RTPFB and fmt == FB_NACK and end - pos >= 12:
            media = struct.unpack_from("!I", data, pos + 8)[0]
            lost = fb.nacks.setdefault(media, [])
            for off in range(pos + 12, end - 3, 4):
                pid, blp = struct.unpack_from("!HH", data, off)
                lost.append(pid)
                for b in range(16):
                    if blp & (1 << b):
                        lost.append((pid + b + 1) & 0xFFFF)
        elif pt == RTCP_PSFB and end - pos >= 12:
            media = struct.unpack_from("!I", data, pos + 8)[0]
            if fmt == FB_PLI:
                fb.pli.add(media)
            elif fmt == FB_FIR:
                for off in range(pos + 12, end - 7, 8):
                    fb.pli.add(struct.unpack_from("!I", data, off)[0])
            elif fmt == FB_REMB and end - pos >= 20 and data[pos + 12:pos + 16] == b"REMB":
                b1, b2, b3 = data[pos + 17], data[pos + 18], data[pos + 19]
                fb.remb_bps = ((b1 & 3) << 16 | b2 << 8 | b3) << (b1 >> 2)
        elif pt == RTCP_BYE:
            fb.bye = True
        pos = end
    return fb


class H264Depacketizer:
    """Reassembles RFC 6184 packets (single NAL, STAP-A, FU-A) into Annex-B access units."""

    def __init__(self):
        self._au: list = []
        self._fu: bytearray | None = None
        self._ts = None

    def push(self, payload: bytes, timestamp: int, marker: bool) -> bytes | None:
        if self._ts is not None and timestamp != self._ts and self._au:
            self._au, self._fu = [], None  # lost the end of the previous access unit
        self._ts = timestamp
        t = payload[0] & 0x1F
        if 1 <= t <= 23:
            self._au.append(payload)
        elif t == 24:
            pos = 1
            while pos + 2 <= len(payload):
                n = struct.unpack_from("!H", payload, pos)[0]
                self._au.append(payload[pos + 2:pos + 2 + n])
                pos += 2 + n
        elif t == 28 and len(payload) >= 2:
            s, e = payload[1] & 0x80, payload[1] & 0x40
            if s:
                self._fu = bytearray([(payload[0] & 0xE0) | (payload[1] & 0x1F)])
            if self._fu is not None:
                self._fu += payload[2:]
                if e:
                    self._au.append(bytes(self._fu))
                    self._fu = None
        if marker:
            au = b"".join(b"\x00\x00\x00\x01" + n for n in self._au)
            self._au = []
            return au
        return None


class H265Depacketizer:
    """Reassembles RFC 7798 packets (single NAL, AP type 48, FU type 49) into Annex-B access units."""

    def __init__(self):
        self._au: list = []
        self._fu: bytearray | None = None
        self._ts = None

    def push(self, payload: bytes, timestamp: int, marker: bool) -> bytes | None:
        if self._ts is not None and timestamp != self._ts and self._au:
            self._au, self._fu = [], None
        self._ts = timestamp
        if len(payload) < 3:
            return None
        t = (payload[0] >> 1) & 63
        if t == 48:
            pos = 2
            while pos + 2 <= len(payload):
                n = struct.unpack_from("!H", payload, pos)[0]
                self._au.append(payload[pos + 2:pos + 2 + n])
                pos += 2 + n
        elif t == 49:
            fu = payload[2]
            if fu & 0x80:
                self._fu = bytearray([(payload[0] & 0x81) | ((fu & 63) << 1), payload[1]])
            if self._fu is not None:
                self._fu += payload[3:]
                if fu & 0x40:
                    self._au.append(bytes(self._fu))
                    self._fu = None
        else:
            self._au.append(payload)
        if marker:
            au = b"".join(b"\x00\x00\x00\x01" + n for n in self._au)
            self._au = []
            return au
        return None


def _leb128(buf: bytes, pos: int) -> tuple[int, int]:
    """LEB128 at pos -> (value, next pos); ValueError when truncated or over 8 bytes."""
    v, sh = 0, 0
    for _ in range(8):
        if pos >= len(buf):
            raise ValueError("truncated leb128")
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << sh
        sh += 7
        if not b & 0x80:
            return v, pos
    raise ValueError("leb128 longer than 8 bytes")


def _put_leb128(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


class AV1Depacketizer:
    """Reassembles AV1 RTP packets (aggregation header Z/Y/W/N, OBU elements) into a
    temporal unit of low-overhead OBUs: a temporal delimiter, then every OBU with its
    size field restored (what a decoder such as dav1d takes)."""

    def __init__(self):
        self._obus: list = []
        self._frag: bytearray | None = None
        self._ts = None

    def push(self, payload: bytes, timestamp: int, marker: bool) -> bytes | None:
        if self._ts is not None and timestamp != self._ts and self._obus:
            self._obus, self._frag = [], None
        self._ts = timestamp
        if not payload:
            return None
        agg = payload[0]
        z, y, w = bool(agg & 0x80), bool(agg & 0x40), (agg >> 4) & 3
        pos, elems = 1, []
        k = 0
        try:
            while pos < len(payload):
                k += 1
                if w and k == w:            # last element: no length field
                    n = len(payload) - pos
                else:
                    n, pos = _leb128(payload, pos)
                if n == 0 or pos + n > len(payload):
                    raise ValueError("OBU element exceeds the packet")
                elems.append(payload[pos:pos + n])
                pos += n
        except ValueError:   # malformed packet: drop it and the fragment it may continue
            self._frag = None
            return None
        for i, e in enumerate(elems):
            cont = i == 0 and z
            more = i == len(elems) - 1 and y
            if cont:
                if self._frag is None:   # lost the head: drop the fragment
                    continue
                self._frag += e
                if not more:
                    self._obus.append(bytes(self._frag))
                    self._frag = None
            elif more:
                self._frag = bytearray(e)
            else:
                self._obus.append(bytes(e))
        if marker:
            out = bytearray(b"\x12\x00")   # temporal delimiter
            for o in self._obus:
                ext = (o[0] >> 2) & 1
                hl = 1 + ext
                if len(o) < hl:
                    continue
                if o[0] & 2:   # the sender kept obu_has_size_field: the OBU is complete as is
                    out += o
                    continue
                out += bytes([o[0] | 2]) + o[1:hl] + _put_leb128(len(o) - hl) + o[hl:]
            self._obus, self._frag = [], None
            return bytes(out)
        return None
