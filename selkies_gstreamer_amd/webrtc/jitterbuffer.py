"""RTP jitter buffer: reorders packets by sequence number and releases whole frames.

Parity target: the vendored aiortc ``JitterBuffer`` of the reference
(``src/selkies/webrtc/jitterbuffer.py``): a power-of-two ring indexed by
``seq % capacity``; a frame (all packets sharing one RTP timestamp) is released
when every sequence number from its first packet to the packet that starts the
next timestamp is present; a jump larger than the capacity resets the buffer
and asks the sender for a keyframe (PLI).

Sequence numbers are 16 bit and wrap; every comparison is done on the unwrapped
difference.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional


@dataclass
class RtpPacket:
    seq: int
    timestamp: int
    marker: bool
    payload: bytes


@dataclass
class JitterFrame:
    timestamp: int
    packets: list   # RtpPacket in sequence order


def _seq_delta(a: int, b: int) -> int:
    """Signed distance a - b of two 16-bit sequence numbers."""
    d = (a - b) & 0xFFFF
    return d - 0x10000 if d >= 0x8000 else d


class JitterBuffer:
    def __init__(self, capacity: int = 128, is_video: bool = True):
        assert capacity & (capacity - 1) == 0, "capacity must be a power of 2"
        self.capacity = capacity
        self.is_video = is_video
        self._slots: list[Optional[RtpPacket]] = [None] * capacity
        self._origin: Optional[int] = None   # sequence number of the oldest retained packet
        self._released: Optional[int] = None  # timestamp of the last released frame
        self.stats = {"frames": 0, "resets": 0, "late": 0}

    def __len__(self) -> int:
        return sum(p is not None for p in self._slots)

    def _reset(self) -> None:
        self._slots = [None] * self.capacity
        self._origin = None
        self._released = None
        self.stats["resets"] += 1

    def add(self, pkt: RtpPacket) -> tuple[bool, list]:
        """Inserts a packet. Returns (pli_needed, frames completed by it, oldest first)."""
        pli = False
        if self._origin is None:
            self._origin = pkt.seq
        d = _seq_delta(pkt.seq, self._origin)
        if d < 0:
            if -d > self.capacity:          # sender restarted: start over
                self._reset()
                self._origin = pkt.seq
                d = 0
                pli = self.is_video
            elif self._released is None:
                self._origin = pkt.seq      # nothing released yet: the stream starts earlier
                d = 0
            else:
                self.stats["late"] += 1     # older than what was already released
                return False, []
        if d >= self.capacity:
            # too far ahead: drop what cannot complete, restart at this packet
            self._reset()
            self._origin = pkt.seq
            d = 0
            pli = self.is_video
        self._slots[pkt.seq % self.capacity] = pkt
        frames = []
        while True:
            f = self._pop_frame()
            if f is None:
                return pli, frames
            frames.append(f)

    def _pop_frame(self) -> Optional[JitterFrame]:
        """Releases the oldest frame whose packets are all present and that is
        followed by a packet of a later timestamp (or ends with the marker bit)."""
        # fillers (payload None: ULPFEC packets sharing the RED stream's sequence space)
        # between frames are consumed here so they never block the next frame
        while True:
            p = self._slots[self._origin % self.capacity]
            if p is None or p.seq != self._origin or p.payload is not None:
                break
            self._slots[self._origin % self.capacity] = None
            self._origin = (self._origin + 1) & 0xFFFF
        frame: list[RtpPacket] = []
        ts = None
        for i in range(self.capacity):
            seq = (self._origin + i) & 0xFFFF
            p = self._slots[seq % self.capacity]
            if p is None or p.seq != seq:
                return None                  # gap: wait for retransmission / reorder
            if p.payload is None:            # a filler ends the frame before it
                return self._release(frame, ts, seq) if frame else None
            if ts is None:
                ts = p.timestamp
            if p.timestamp != ts:
                return self._release(frame, ts, seq)
            frame.append(p)
            if p.marker:
                return self._release(frame, ts, (seq + 1) & 0xFFFF)
        return None

    def _release(self, frame: list, ts: int, next_seq: int) -> JitterFrame:
        for p in frame:
            self._slots[p.seq % self.capacity] = None
        self._origin = next_seq
        self._released = ts
        self.stats["frames"] += 1
        return JitterFrame(ts, frame)

    def missing(self, limit: int = 64) -> list[int]:
        """Sequence numbers absent between the origin and the newest packet (NACK list)."""
        if self._origin is None:
            return []
        newest = None
        for p in self._slots:
            if p is not None and (newest is None or _seq_delta(p.seq, newest) > 0):
                newest = p.seq
        if newest is None:
            return []
        out = []
        for i in range(_seq_delta(newest, self._origin)):
            seq = (self._origin + i) & 0xFFFF
            p = self._slots[seq % self.capacity]
            if p is None or p.seq != seq:
                out.append(seq)
                if len(out) >= limit:
                    break
        return out
