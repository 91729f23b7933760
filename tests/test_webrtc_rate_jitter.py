"""GCC delay-based estimator (webrtc/rate.py) and RTP jitter buffer (webrtc/jitterbuffer.py).

The reference's aiortc copies are not importable here (no aiortc/av), so the
estimator is checked on its defining behaviour with simulated links — parity
unpinned to the reference's exact numbers: a link that keeps up must never
produce an overuse signal and lets the estimate grow (bounded by 1.5x the
incoming rate); a bottleneck whose queue grows must be detected within a
second and pull the estimate below the bottleneck rate.
"""
import random

import pytest

from selkies_gstreamer_amd.webrtc.jitterbuffer import JitterBuffer, RtpPacket
from selkies_gstreamer_amd.webrtc.rate import (OVERUSE, DelayGradientFilter, InterArrival, OveruseDetector,
                                               RemoteBitrateEstimator)


def _simulate(est, seconds, send_bps, link_bps, fps=30, pkt=1000, t0=0.0, state=None, jitter_ms=0.0, seed=1):
    """Frames of ``send_bps`` through a FIFO bottleneck of ``link_bps``; returns
    the estimates/REMB decisions and the link state to continue from."""
    rng = random.Random(seed)
    last_arrival = state if state is not None else 0.0
    per_frame = max(1, int(send_bps / fps / 8 / pkt))
    out = []
    signals = []
    for f in range(int(seconds * fps)):
        send = t0 + f * 1000.0 / fps
        for _ in range(per_frame):
            tx = pkt * 8 * 1000.0 / link_bps
            arrival = max(send + 20.0, last_arrival) + tx + rng.uniform(0, jitter_ms)
            last_arrival = arrival
            r = est.add(arrival, send, pkt)
            signals.append(est.signal)
            if r is not None:
                out.append(r)
    return out, signals, last_arrival, t0 + seconds * 1000.0


def test_interarrival_groups_by_timestamp():
    ia = InterArrival(group_by_timestamp=True)
    assert ia.add(0.0, 10.0, 100) is None
    assert ia.add(0.0, 11.0, 100) is None
    assert ia.add(33.0, 45.0, 100) is None          # second group starts
    d = ia.add(66.0, 80.0, 300)                     # completes group 2
    assert d == (33.0, 45.0 - 11.0, 100 - 200)


def test_kalman_tracks_constant_gradient():
    f = DelayGradientFilter()
    for _ in range(200):
        m = f.update(33.0, 35.0)   # queue grows 2 ms per group
    assert 1.5 < m < 2.5
    g = DelayGradientFilter()
    for _ in range(200):
        m = g.update(33.0, 33.0)
    assert abs(m) < 0.1


def test_detector_needs_persistence():
    d = OveruseDetector()
    # one spike above the threshold is not overuse
    assert d.detect(1.0, 60, 33.0, 0.0) != OVERUSE
    d2 = OveruseDetector()
    states = [d2.detect(0.5 + 0.01 * i, 60, 33.0, 33.0 * i) for i in range(5)]
    assert OVERUSE in states


def test_estimate_grows_on_a_clear_link():
    est = RemoteBitrateEstimator(start_bps=300_000)
    out, signals, *_ = _simulate(est, 8.0, 2_000_000, 50_000_000, jitter_ms=1.0)
    assert OVERUSE not in signals
    rates = [r for r, _ in out]
    assert rates[-1] >= 1_500_000                   # follows the incoming rate up
    assert rates[-1] <= 1.5 * 2_050_000 + 10_000    # never far above what arrives
    assert sum(send for _, send in out) >= 7       # about one REMB per second


def test_bottleneck_is_detected_and_estimate_drops():
    est = RemoteBitrateEstimator(start_bps=2_000_000)
    out, signals, state, t = _simulate(est, 1.0, 2_000_000, 50_000_000)
    out2, signals2, state, t = _simulate(est, 4.0, 2_000_000, 800_000, t0=t, state=state)
    assert OVERUSE in signals2[: 2 * 30 * 8]        # within ~2 s of the queue starting to grow
    assert out2[-1][0] < 800_000                   # below the bottleneck capacity
    drops = [r for r, send in out2 if send]
    assert len(drops) >= 2


def test_recovers_after_congestion():
    est = RemoteBitrateEstimator(start_bps=1_000_000)
    _, _, state, t = _simulate(est, 3.0, 1_500_000, 600_000)
    low = est.estimate
    assert low < 600_000
    # the sender backs off to the estimate and the bottleneck goes away: the queue
    # drains, then the estimate climbs again (capped by 1.5x the incoming rate)
    out, signals, state, t = _simulate(est, 12.0, 500_000, 50_000_000, t0=t, state=state)
    assert signals[-300:].count(OVERUSE) == 0
    assert low < est.estimate <= 1.5 * 510_000 + 10_000


# -- jitter buffer ------------------------------------------------------------------------------------

def _frames(n_frames, per_frame, seq0=0, ts0=0):
    pkts = []
    seq = seq0
    for f in range(n_frames):
        for i in range(per_frame):
            pkts.append(RtpPacket(seq & 0xFFFF, ts0 + 3000 * f, i == per_frame - 1, bytes([f, i])))
            seq += 1
    return pkts


def test_in_order_frames_release_on_marker():
    jb = JitterBuffer(capacity=64)
    got = []
    for p in _frames(5, 3):
        pli, frames = jb.add(p)
        assert not pli
        got += frames
    assert [f.timestamp for f in got] == [0, 3000, 6000, 9000, 12000]
    assert all(len(f.packets) == 3 for f in got)
    assert len(jb) == 0


@pytest.mark.parametrize("seq0", [0, 65530])
def test_reordered_and_wrapping(seq0):
    rng = random.Random(7)
    pkts = _frames(6, 4, seq0=seq0)
    # shuffle inside windows of 5 packets (network reordering)
    shuffled = []
    for i in range(0, len(pkts), 5):
        w = pkts[i:i + 5]
        rng.shuffle(w)
        shuffled += w
    jb = JitterBuffer(capacity=64)
    got = []
    for p in shuffled:
        got += jb.add(p)[1]
    assert [f.timestamp for f in got] == [3000 * f for f in range(6)]
    for f in got:
        assert [p.payload[1] for p in f.packets] == [0, 1, 2, 3]


def test_gap_waits_and_reports_missing():
    jb = JitterBuffer(capacity=64)
    pkts = _frames(3, 3)
    lost = pkts.pop(4)                  # middle packet of frame 1
    got = []
    for p in pkts:
        got += jb.add(p)[1]
    assert [f.timestamp for f in got] == [0]
    assert jb.missing() == [lost.seq]
    got = jb.add(lost)[1]               # retransmission completes frames 1 and 2
    assert [f.timestamp for f in got] == [3000, 6000]


def test_large_jump_resets_and_requests_keyframe():
    jb = JitterBuffer(capacity=16)
    for p in _frames(2, 2):
        jb.add(p)
    pli, frames = jb.add(RtpPacket(500, 99000, True, b"x"))
    assert pli and [f.timestamp for f in frames] == [99000]
    assert jb.stats["resets"] == 1
