"""Video forward error correction: RED (RFC 2198) + ULPFEC (RFC 5109), the scheme
webrtcbin enables for the reference's video when ``video_packetloss_percent`` > 0
(legacy/gstwebrtc_app.py:996-1000, ``fec-type ulp-red`` with ``fec-percentage``).

Sender: every media packet travels RED-encapsulated (one primary block, the block
header carries the media payload type); after each access unit, ``ceil(n * pct /
100)`` ULPFEC packets protect consecutive groups of the unit's packets (level 0 only,
16-bit mask for groups <= 16 packets, 48-bit otherwise). Media and FEC packets share
the RED stream's SSRC and sequence space, so the FEC packets take the sequence
numbers right after the unit's media packets.

Receiver (test peer / browser-less clients): RED is unwrapped, media packets are
remembered, and a FEC packet whose group misses exactly one packet rebuilds it
(header bits, timestamp, length and payload by XOR).
"""
from __future__ import annotations

import math
import struct
from typing import Optional

import numpy as np

RED_PT = 123
ULPFEC_PT = 125
MAX_GROUP = 48


def rtp_header_len(pkt: bytes) -> int:
    cc = pkt[0] & 0x0F
    n = 12 + 4 * cc
    if pkt[0] & 0x10:
        n += 4 + 4 * struct.unpack_from("!H", pkt, n + 2)[0]
    return n


def red_wrap(pkt: bytes, red_pt: int = RED_PT) -> bytes:
    """Media RTP packet -> the same packet as a RED packet with one primary block."""
    h = rtp_header_len(pkt)
    return bytes([pkt[0], (pkt[1] & 0x80) | red_pt]) + pkt[2:h] + bytes([pkt[1] & 0x7F]) + pkt[h:]


def red_unwrap(pkt: bytes) -> Optional[bytes]:
    """RED packet with one primary block -> the inner media packet (block PT restored).
    Redundant blocks (F bit set) are skipped; None when malformed."""
    h = rtp_header_len(pkt)
    i = h
    while i < len(pkt) and pkt[i] & 0x80:   # 4-byte headers of redundant blocks
        i += 4
    if i >= len(pkt):
        return None
    blk_pt = pkt[i] & 0x7F
    red_len = sum(((pkt[j + 2] & 0x03) << 8 | pkt[j + 3]) for j in range(h, i, 4))
    primary = pkt[i + 1 + red_len:]
    return bytes([pkt[0], (pkt[1] & 0x80) | blk_pt]) + pkt[2:h] + primary


def _xor_into(acc: np.ndarray, data: bytes) -> None:
    acc[:len(data)] ^= np.frombuffer(data, np.uint8)


def ulpfec_packet(media: list, seq_base: int, ssrc: int, seq: int, timestamp: int,
                  fec_pt: int = ULPFEC_PT) -> bytes:
    """One ULPFEC RTP packet (media PT = ``fec_pt``, to be RED-wrapped by the caller)
    protecting ``media`` (plaintext media RTP packets with consecutive sequence numbers
    starting at ``seq_base``)."""
    long_mask = len(media) > 16
    bodies = [p[12:] for p in media]          # everything after the fixed header
    plen = max(len(b) for b in bodies)
    acc = np.zeros(plen, np.uint8)
    b01 = 0
    ts = 0
    ln = 0
    mask = 0
    for p, b in zip(media, bodies):
        b01 ^= (p[0] << 8) | p[1]
        ts ^= struct.unpack_from("!I", p, 4)[0]
        ln ^= len(b)
        _xor_into(acc, b)
        off = (struct.unpack_from("!H", p, 2)[0] - seq_base) & 0xFFFF
        mask |= 1 << ((47 if long_mask else 15) - off)
    # FEC header: E=0 | L | P X CC recovery (from byte 0) ; M PT recovery (byte 1)
    first = (0x40 if long_mask else 0) | (b01 >> 8 & 0x3F)
    hdr = struct.pack("!BBHIH", first, b01 & 0xFF, seq_base, ts, ln)
    lvl = struct.pack("!H", plen) + (mask.to_bytes(6, "big") if long_mask else mask.to_bytes(2, "big"))
    rtp_hdr = struct.pack("!BBHII", 0x80, fec_pt & 0x7F, seq, timestamp, ssrc)
    return rtp_hdr + hdr + lvl + acc.tobytes()


class FecEncoder:
    """Per-access-unit FEC generation for a RED stream."""

    def __init__(self, ssrc: int, percentage: int, red_pt: int = RED_PT, fec_pt: int = ULPFEC_PT):
        self.ssrc, self.percentage = ssrc, percentage
        self.red_pt, self.fec_pt = red_pt, fec_pt

    def protect(self, media: list, next_seq: int) -> list:
        """media: one access unit's plaintext media packets (consecutive seqs). Returns
        the RED-wrapped media packets followed by RED-wrapped FEC packets numbered from
        ``next_seq``; the caller advances its sequence counter by the FEC count."""
        out = [red_wrap(p, self.red_pt) for p in media]
        if self.percentage <= 0 or not media:
            return out
        k = min(len(media), max(1, math.ceil(len(media) * self.percentage / 100)))
        per = min(MAX_GROUP, math.ceil(len(media) / k))
        ts = struct.unpack_from("!I", media[0], 4)[0]
        seq = next_seq
        for g in range(0, len(media), per):
            grp = media[g:g + per]
            base = struct.unpack_from("!H", grp[0], 2)[0]
            out.append(red_wrap(ulpfec_packet(grp, base, self.ssrc, seq, ts, self.fec_pt), self.red_pt))
            seq = (seq + 1) & 0xFFFF
        return out


class FecDecoder:
    """Receiver: RED unwrap + single-loss recovery per FEC packet."""

    def __init__(self, fec_pt: int = ULPFEC_PT, history: int = 512):
        self.fec_pt = fec_pt
        self.media: dict = {}   # seq -> plaintext media packet
        self.history = history
        self.recovered = 0

    def _remember(self, pkt: bytes) -> None:
        seq = struct.unpack_from("!H", pkt, 2)[0]
        self.media[seq] = pkt
        while len(self.media) > self.history:
            self.media.pop(next(iter(self.media)))

    def push(self, red_pkt: bytes) -> tuple:
        """One RED packet in; returns (media packets to hand on: the unwrapped packet
        itself and/or one recovered with this FEC packet, sequence number of this packet
        when it is a FEC packet else None)."""
        inner = red_unwrap(red_pkt)
        if inner is None:
            return [], None
        seq = struct.unpack_from("!H", inner, 2)[0]
        if inner[1] & 0x7F != self.fec_pt:
            if seq in self.media:
                return [], None   # already recovered
            self._remember(inner)
            return [inner], None
        rec = self._recover(inner)
        return ([rec] if rec is not None else []), seq

    def _recover(self, fec: bytes) -> Optional[bytes]:
        ssrc = struct.unpack_from("!I", fec, 8)[0]
        f = fec[12:]
        long_mask = bool(f[0] & 0x40)
        b01 = ((f[0] & 0x3F) << 8) | f[1]
        seq_base, ts, ln = struct.unpack_from("!HIH", f, 2)
        plen = struct.unpack_from("!H", f, 10)[0]
        mbytes = 6 if long_mask else 2
        mask = int.from_bytes(f[12:12 + mbytes], "big")
        payload = f[12 + mbytes:]
        nbits = 48 if long_mask else 16
        seqs = [(seq_base + i) & 0xFFFF for i in range(nbits) if mask >> (nbits - 1 - i) & 1]
        missing = [s for s in seqs if s not in self.media]
        if len(missing) != 1:
            return None
        acc = np.zeros(plen, np.uint8)
        _xor_into(acc, payload[:plen])
        for s in seqs:
            if s == missing[0]:
                continue
            p = self.media[s]
            b01 ^= ((p[0] << 8) | p[1]) & 0x3FFF   # version bits are not recovered
            ts ^= struct.unpack_from("!I", p, 4)[0]
            ln ^= len(p) - 12
            _xor_into(acc, p[12:])
        if ln > plen:
            return None
        pkt = struct.pack("!BBHII", 0x80 | (b01 >> 8 & 0x3F), b01 & 0xFF, missing[0], ts, ssrc) + acc[:ln].tobytes()
        self._remember(pkt)
        self.recovered += 1
        return pkt
