"""Receive-side congestion control (Google Congestion Control, delay-based part).

Parity target: the vendored aiortc estimator the reference ships
(``src/selkies/webrtc/rate.py``: ``AimdRateControl`` 68, ``OveruseDetector`` 300,
``OveruseEstimator`` 371, ``RemoteBitrateEstimator`` 505), which turns packet
arrival times into the REMB value a receiver reports. This module follows the
algorithm of draft-ietf-rmcat-gcc-02 directly:

1. ``InterArrival`` groups packets by send time (one video frame = one RTP
   timestamp, or a 5 ms burst when abs-send-time is used) and yields, per
   completed group, the inter-group send delta, arrival delta and size delta.
2. ``DelayGradientFilter`` (Kalman filter, §5.3) estimates the queuing-delay
   gradient m(i) from d(i) = arrival delta - send delta.
3. ``OveruseDetector`` (§5.4) compares m(i) (scaled by the number of deltas)
   against an adaptive threshold gamma(i) and signals overuse only after it has
   persisted for 10 ms with a non-decreasing gradient.
4. ``AimdRateController`` (§5.5) moves the estimate A: multiplicative increase
   (8 %/s) far from the last congestion point, additive near it, 0.85 x the
   measured incoming rate on overuse, hold on underuse; A <= 1.5 x incoming.
5. ``RemoteBitrateEstimator`` ties these together per SSRC set and decides when
   a REMB is due (every second, or at once after a >= 3 % drop).

All times are milliseconds (floats); rates are bit/s.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

BURST_MS = 5.0
OVERUSE_TIME_MS = 10.0
NORMAL, OVERUSE, UNDERUSE = "normal", "overuse", "underuse"
HOLD, INCREASE, DECREASE = "hold", "increase", "decrease"


class RateCounter:
    """Bits received over a sliding window (default 1 s), in bit/s."""

    def __init__(self, window_ms: float = 1000.0):
        self.window = window_ms
        self._samples: list[tuple[float, int]] = []
        self._bytes = 0
        self._first: Optional[float] = None

    def add(self, nbytes: int, now_ms: float) -> None:
        self._expire(now_ms)
        if self._first is None or not self._samples:
            self._first = now_ms   # first packet, or a silence longer than the window: re-learn
        self._samples.append((now_ms, nbytes))
        self._bytes += nbytes

    def _expire(self, now_ms: float) -> None:
        cut = now_ms - self.window
        i = 0
        while i < len(self._samples) and self._samples[i][0] <= cut:
            self._bytes -= self._samples[i][1]
            i += 1
        if i:
            del self._samples[:i]

    def rate(self, now_ms: float) -> Optional[int]:
        self._expire(now_ms)
        # valid once a whole window has been observed (a half-filled window under-reads)
        if self._first is None or now_ms - self._first < self.window or not self._samples:
            return None
        return int(self._bytes * 8000.0 / self.window)


@dataclass
class _Group:
    first_send: float
    send: float      # send time of the group's last packet
    arrival: float   # arrival time of the group's last packet
    size: int


class InterArrival:
    """Packet groups -> (send delta, arrival delta, size delta) per completed group.

    ``group_by_timestamp``: packets with the same send time stamp form a group
    (RTP timestamps of one video frame); otherwise packets whose send times lie
    within ``BURST_MS`` of the group's first packet do (abs-send-time)."""

    def __init__(self, group_by_timestamp: bool = True):
        self.by_ts = group_by_timestamp
        self._cur: Optional[_Group] = None
        self._prev: Optional[_Group] = None

    def _new_group(self, send: float) -> bool:
        if self._cur is None:
            return False
        if self.by_ts:
            return send != self._cur.first_send
        return send - self._cur.first_send > BURST_MS

    def add(self, send_ms: float, arrival_ms: float, size: int):
        """Returns (send_delta, arrival_delta, size_delta) when a group completes, else None."""
        if self._cur is not None and send_ms < self._cur.first_send and not self.by_ts:
            return None  # reordered packet of an older group
        out = None
        if self._new_group(send_ms):
            if self._prev is not None:
                out = (self._cur.send - self._prev.send, self._cur.arrival - self._prev.arrival,
                       self._cur.size - self._prev.size)
            self._prev = self._cur
            self._cur = None
        if self._cur is None:
            self._cur = _Group(send_ms, send_ms, arrival_ms, 0)
        self._cur.send = max(self._cur.send, send_ms)
        self._cur.arrival = max(self._cur.arrival, arrival_ms)
        self._cur.size += size
        return out


class DelayGradientFilter:
    """Scalar Kalman filter on the inter-group delay variation (gcc-02 §5.3)."""

    def __init__(self, q: float = 1e-3, e0: float = 0.1, chi: float = 0.01):
        self.q = q
        self.e = e0
        self.chi = chi
        self.m = 0.0          # queuing-delay gradient estimate, ms per group
        self.var_v = 50.0     # measurement noise variance estimate
        self.num_deltas = 0

    def update(self, send_delta: float, arrival_delta: float, fmax: float = 30.0) -> float:
        d = arrival_delta - send_delta
        self.num_deltas = min(self.num_deltas + 1, 60)
        z = d - self.m
        # noise variance: exponential average with a frame-rate dependent factor, outliers capped at 3 sigma
        alpha = (1.0 - self.chi) ** (30.0 / max(1.0, fmax))
        zc = min(abs(z), 3.0 * math.sqrt(self.var_v))
        self.var_v = max(alpha * self.var_v + (1.0 - alpha) * zc * zc, 1.0)
        k = (self.e + self.q) / (self.var_v + self.e + self.q)
        self.m += k * z
        self.e = (1.0 - k) * (self.e + self.q)
        return self.m


class OveruseDetector:
    """Adaptive-threshold over/under-use signal (gcc-02 §5.4)."""

    def __init__(self, k_up: float = 0.01, k_down: float = 0.00018, gamma0: float = 12.5):
        self.k_up, self.k_down = k_up, k_down
        self.gamma = gamma0
        self.state = NORMAL
        self._over_ms = -1.0
        self._over_count = 0
        self._prev_m = 0.0
        self._last_ms: Optional[float] = None

    def detect(self, m: float, num_deltas: int, send_delta: float, now_ms: float) -> str:
        t = min(num_deltas, 60) * m   # modified trend, as compared against gamma
        if t > self.gamma:
            self._over_ms = send_delta if self._over_ms < 0 else self._over_ms + send_delta
            self._over_count += 1
            if self._over_ms > OVERUSE_TIME_MS and self._over_count > 1 and m >= self._prev_m:
                self._over_ms = 0.0
                self._over_count = 0
                self.state = OVERUSE
        elif t < -self.gamma:
            self._over_ms = -1.0
            self._over_count = 0
            self.state = UNDERUSE
        else:
            self._over_ms = -1.0
            self._over_count = 0
            self.state = NORMAL
        self._prev_m = m
        self._adapt(t, now_ms)
        return self.state

    def _adapt(self, t: float, now_ms: float) -> None:
        if self._last_ms is None:
            self._last_ms = now_ms
        if abs(t) > self.gamma + 15.0:   # do not let a spike drag the threshold
            self._last_ms = now_ms
            return
        k = self.k_down if abs(t) < self.gamma else self.k_up
        dt = min(now_ms - self._last_ms, 100.0)
        self.gamma = min(max(self.gamma + k * (abs(t) - self.gamma) * dt, 6.0), 600.0)
        self._last_ms = now_ms


class AimdRateController:
    """Additive-increase / multiplicative-decrease estimate A(i) (gcc-02 §5.5)."""

    def __init__(self, start_bps: int = 300_000, min_bps: int = 30_000, max_bps: int = 100_000_000,
                 beta: float = 0.85, rtt_ms: float = 200.0):
        self.rate = float(start_bps)
        self.min_bps, self.max_bps = min_bps, max_bps
        self.beta = beta
        self.rtt_ms = rtt_ms
        self.state = HOLD
        self._last_ms: Optional[float] = None
        self._avg_max_kbps: Optional[float] = None   # incoming rate at past decreases (kbit/s)
        self._var_max = 0.4
        self.initialized = False

    def _near_max(self, incoming_kbps: float) -> bool:
        if self._avg_max_kbps is None:
            return False
        std = math.sqrt(self._var_max * self._avg_max_kbps)
        return abs(incoming_kbps - self._avg_max_kbps) <= 3.0 * std

    def _track_max(self, incoming_kbps: float) -> None:
        a = 0.05
        if self._avg_max_kbps is None:
            self._avg_max_kbps = incoming_kbps
        else:
            self._avg_max_kbps = (1 - a) * self._avg_max_kbps + a * incoming_kbps
        norm = max(self._avg_max_kbps, 1.0)
        self._var_max = min(max((1 - a) * self._var_max + a * (self._avg_max_kbps - incoming_kbps) ** 2 / norm,
                                0.4), 2.5)

    def update(self, signal: str, incoming_bps: Optional[int], now_ms: float) -> int:
        if not self.initialized and incoming_bps:
            self.rate = float(incoming_bps)   # first valid throughput measurement
            self.initialized = True
        # state machine: overuse -> decrease; underuse -> hold; normal -> increase (from hold)
        if signal == OVERUSE:
            self.state = DECREASE
        elif signal == UNDERUSE:
            self.state = HOLD
        elif self.state in (HOLD, DECREASE):
            self.state = INCREASE
        dt = 0.0 if self._last_ms is None else min(now_ms - self._last_ms, 1000.0)
        self._last_ms = now_ms
        inc_kbps = (incoming_bps or 0) / 1000.0
        if self.state == INCREASE and incoming_bps:
            before = self.rate
            if self._avg_max_kbps is not None and inc_kbps > self._avg_max_kbps + 3.0 * math.sqrt(
                    self._var_max * self._avg_max_kbps):
                self._avg_max_kbps = None   # link capacity moved up: go multiplicative again
            if self._near_max(inc_kbps):
                # additive: about one packet (1200 B) per response time (RTT + 100 ms)
                per_frame_bits = self.rate / 30.0
                pkts = max(1.0, per_frame_bits / (1200 * 8))
                avg_pkt_bits = per_frame_bits / pkts
                self.rate += max(1000.0, avg_pkt_bits) * dt / (self.rtt_ms + 100.0)
            else:
                self.rate *= 1.08 ** (dt / 1000.0)
            # throughput cap: limits increases to 1.5x what arrives, never lowers the estimate
            self.rate = min(self.rate, max(before, 1.5 * incoming_bps + 10_000))
        elif self.state == DECREASE and incoming_bps:
            new = self.beta * incoming_bps
            if new > self.rate:   # never increase on a decrease signal
                new = self.rate
            self._track_max(inc_kbps)
            self.rate = new
            self.state = HOLD
        self.rate = min(max(self.rate, self.min_bps), self.max_bps)
        return int(self.rate)


class RemoteBitrateEstimator:
    """Per-stream delay-based estimator; feed every received media packet.

    ``add(arrival_ms, send_ms, size)`` returns ``(bitrate, send_remb)`` once an
    estimate exists; ``send_remb`` is True when a REMB should go out now (first
    estimate, 1 s since the last one, or a drop of >= 3 %)."""

    def __init__(self, start_bps: int = 300_000, group_by_timestamp: bool = True):
        self.inter = InterArrival(group_by_timestamp)
        self.filter = DelayGradientFilter()
        self.detector = OveruseDetector()
        self.aimd = AimdRateController(start_bps)
        self.incoming = RateCounter(1000.0)
        self.estimate: Optional[int] = None
        self._last_remb_ms: Optional[float] = None
        self._last_remb_bps: Optional[int] = None
        self._last_update_ms: Optional[float] = None
        self.signal = NORMAL

    def set_rtt(self, rtt_ms: float) -> None:
        self.aimd.rtt_ms = rtt_ms

    def add(self, arrival_ms: float, send_ms: float, size: int):
        self.incoming.add(size, arrival_ms)
        deltas = self.inter.add(send_ms, arrival_ms, size)
        if deltas is not None:
            sd, ad, _ = deltas
            m = self.filter.update(sd, ad)
            self.signal = self.detector.detect(m, self.filter.num_deltas, sd, arrival_ms)
        incoming = self.incoming.rate(arrival_ms)
        # the controller runs on every overuse signal and at least every 100 ms
        if incoming is None:
            return None
        due = self._last_update_ms is None or arrival_ms - self._last_update_ms >= 100.0 or self.signal == OVERUSE
        if not due:
            return (self.estimate, False) if self.estimate is not None else None
        self._last_update_ms = arrival_ms
        self.estimate = self.aimd.update(self.signal, incoming, arrival_ms)
        send = (self._last_remb_ms is None or arrival_ms - self._last_remb_ms >= 1000.0 or
                (self._last_remb_bps is not None and self.estimate < 0.97 * self._last_remb_bps))
        if send:
            self._last_remb_ms = arrival_ms
            self._last_remb_bps = self.estimate
        return self.estimate, send
