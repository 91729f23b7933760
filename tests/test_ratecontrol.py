"""K10 rate control (csrc/codec/ratecontrol.h): CRF, CBR with a 1.5-frame VBV and the
CBR overflow guard (second coding pass), on the CPU reference and — gpu-marked —
bit-exact on the HIP encoder (k_rc_qp, k_rc_guard, k_rc_account).

Reference parity: the WebRTC mode's encoders run CBR with vbv-buf-capacity of 1.5
frame periods (legacy/gstwebrtc_app.py:101-105, 630-637); the websocket mode's
pixelflux encoder is CRF-driven (settings.py:48). The reference publishes no rate
traces, so the bounds here are the VBV contract itself: mean rate near the target and
no frame other than a key frame above 1.5 budgets."""
import os
import sys

import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _trace(**kw):
    import rc_trace
    return rc_trace.run(**kw)


@pytest.mark.parametrize("content", ["motion", "desktop"])
def test_cbr_rate_and_vbv_cpu(content):
    r = _trace(backend="cpu", width=320, height=192, frames=150, content=content, mode="cbr", kbps=480)
    assert 0.85 <= r["rate_ratio"] <= 1.10, r
    assert r["nonkey_over_1p5"] == 0, r          # the guard re-coded every overflow
    assert r["qp_max"] <= 51


def test_cbr_follows_a_new_target_cpu():
    """set_rate() mid-stream: the delivered rate moves to the new budget."""
    W, H, fps = 320, 192, 60.0
    src = SyntheticDesktop(W, H, kind="motion")
    enc = H264Encoder(W, H, backend="cpu", fps=fps, rate_control="cbr", bitrate_kbps=400)
    sizes = []
    for t in range(160):
        if t == 80:
            enc.set_rate("cbr", 900)
        sizes.append(sum(len(p.data) for p in enc.encode(src.frame(t), t)))
    lo = sum(sizes[30:80]) * 8 * fps / 50 / 1000
    hi = sum(sizes[110:160]) * 8 * fps / 50 / 1000
    assert 0.8 * 400 <= lo <= 1.15 * 400, lo
    assert 0.8 * 900 <= hi <= 1.15 * 900, hi
    st = enc.rc_stats()
    assert st["mode"] == 2 and st["budget"] == int(900 * 1000 / fps)


def test_crf_coarser_on_complex_frames_cpu():
    """CRF: QP follows the frame complexity around the CRF value (x264 qcompress-like
    offset, clipped to [-3, +6]); CQP keeps the constant QP."""
    W, H = 320, 192
    calm, busy = SyntheticDesktop(W, H, kind="desktop"), SyntheticDesktop(W, H, kind="noise")
    qps = {}
    for mode in ("crf", "cqp"):
        enc = H264Encoder(W, H, backend="cpu", qp=25, rate_control=mode, use_paint_over=False,
                          scenecut=False)
        q = []
        for t in range(60):
            f = calm.frame(t) if t < 40 else busy.frame(t)
            enc.encode(f, t)
            q.append(enc.rc_stats()["cur_qp"] if mode == "crf" else 25)
        qps[mode] = q
    crf = qps["crf"]
    assert all(22 <= q <= 31 for q in crf), crf
    assert max(crf[42:]) > 25 >= min(crf[5:40]), crf


def test_capture_session_cbr_cpu():
    """The capture session (csrc/runtime/capture.cpp) runs CBR from its settings and
    switches mode at run time (sk_capture_set_rate)."""
    import ctypes

    import pixelflux
    from selkies_gstreamer_amd.ops.native import PinnedBuffer
    W, H = 256, 128
    src = SyntheticDesktop(W, H, kind="motion", seed=3)
    pool = PinnedBuffer((4, H, W, 4))
    for i in range(4):
        src.frame(i, out=pool.array[i])
    sizes = []

    def on_frame(res, n, user):
        sizes.append(sum(res[i].size for i in range(n)))

    s = pixelflux.default_settings(W, H, use_cpu=1, source=pixelflux.SOURCE_POOL, step_mode=1, pool_frames=4,
                                   pool_stride=W * 4, h264_rc_mode=2, h264_bitrate_kbps=300)
    s.pool = pool.array.ctypes.data
    cap = pixelflux.ScreenCapture()
    cb = pixelflux.FrameCallback(on_frame)
    cap.start_frame_capture(s, cb)
    cap.run(40)
    assert cap.wait(120_000) == 0
    cap.set_rate("crf", 0)
    cap.run(10)
    assert cap.wait(120_000) == 0
    cap.close()
    assert len(sizes) == 50
    budget = 300 * 1000 / 60 / 8
    assert max(sizes[5:40]) <= 1.6 * budget + 10      # per-frame stripe headers on top of the payload cap
    del ctypes


def _parity(codec, mode, kbps, frames, W=320, H=192, content="motion"):
    from selkies_gstreamer_amd.ops.native import require_gpu
    require_gpu()
    src = SyntheticDesktop(W, H, kind=content)
    kw = dict(fullframe=codec != "h264", codec=codec, fps=60.0, rate_control=mode, bitrate_kbps=kbps)
    g = H264Encoder(W, H, backend="hip", **kw)
    c = H264Encoder(W, H, backend="cpu", **kw)
    for t in range(frames):
        f = src.frame(t)
        pg, pc = g.encode(f, t), c.encode(f, t)
        assert [p.data for p in pg] == [p.data for p in pc], (codec, mode, t)
    sg, sc = g.rc_stats(), c.rc_stats()
    assert sg == sc
    return sc


@pytest.mark.gpu
def test_gpu_cbr_guard_matches_cpu():
    """H.264 CBR on the HIP encoder: k_rc_qp / k_rc_guard (gated second pass) /
    k_rc_account reproduce the CPU controller frame by frame, re-encodes included."""
    st = _parity("h264", "cbr", 480, 90)
    assert st["redos"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["hevc", "av1"])
def test_gpu_rate_control_matches_cpu_fullframe(codec):
    """HEVC / AV1 CBR on the HIP encoder: the per-frame cap's gated re-code passes
    (k_rc_guard_sizes + the coding kernels again) reproduce the CPU encoder's second and
    third codings byte for byte (HEVC at 240 kbit/s, where it re-codes). (AV1's leaky bucket re-codes less: its case is the desktop
    content at 960 kbit/s, which overflows the 2.5-budget ceiling on window bursts.)"""
    st = _parity(codec, "cbr", 240, 90) if codec == "hevc" else _parity(codec, "cbr", 960, 90, content="desktop")
    assert st["redos"] > 0
    _parity(codec, "crf", 0, 20)


@pytest.mark.parametrize("codec", ["hevc", "av1"])
@pytest.mark.parametrize("content", ["motion", "desktop"])
def test_cbr_frame_cap_hevc_av1_cpu(codec, content):
    """The per-frame cap (ratecontrol.h rc_frame_cap) on the full-frame encoders: HEVC's
    1.5-frame VBV holds every non-key frame to 1.5 budgets; AV1's 120 ms leaky bucket never
    overflows and holds them to 2.5 budgets (svtav1enc maxsection-pct=250). The mean rate
    stays near the target."""
    r = _trace(backend="cpu", codec=codec, width=320, height=192, frames=150, content=content, mode="cbr", kbps=480)
    assert r["nonkey_over_cap"] == 0, r
    if codec == "hevc":
        assert r["nonkey_over_1p5"] == 0, r
        assert r["redos"] > 0, r
    else:
        assert r["nonkey_over_2p5"] == 0, r
    assert 0.85 <= r["rate_ratio"] <= 1.10, r


def test_av1_cbr_holds_its_budget_cpu():
    """AV1 CBR as svtav1enc runs it (120 ms buffer, no scene-cut key frames, qindex from
    the fractional QP): 960x544 at 120 fps, 2.5 Mbit/s -> the mean within 10 % of the
    target after the key frame, one key frame, no inter frame above 2.5 budgets."""
    r = _trace(backend="cpu", codec="av1", width=960, height=544, frames=60, content="motion", mode="cbr",
               kbps=2500, fps=120.0)
    t = r["trace"]
    budget = 2500 * 1000 / 120 / 8
    inter = t["bytes"][1:]
    assert r["keyframes"] == 1
    assert 0.85 <= sum(inter) / len(inter) / budget <= 1.10, r
    assert max(inter) <= 2.5 * 1.03 * budget, r


def test_fractional_qp_dither():
    """rc_dither_qp (ratecontrol.h) through the CPU controller: a frame at fractional QP
    lo + f/256 codes round(N f / 256) of its N rate-controlled stripes at lo + 1 and the
    rest at lo."""
    from selkies_gstreamer_amd.ops.native import H264Encoder
    W, H = 320, 512   # 8 stripes of 64 px
    enc = H264Encoder(W, H, backend="cpu", rate_control="cbr", bitrate_kbps=600, fps=60.0)
    src = SyntheticDesktop(W, H, kind="motion")
    seen_frac = 0
    for t in range(60):
        enc.encode(src.frame(t), t)
        st = enc.rc_stats()
        lo, f = st["cur_qpf"] >> 8, st["cur_qpf"] & 255
        tasks = enc.debug_buffer("tasks").view(np.int32).reshape(-1, 12)
        coded = [int(q) for a, q in zip(tasks[:, 10], tasks[:, 1]) if a in (1, 2)]   # final_action P / I
        if len(coded) != 8:
            continue
        assert set(coded) <= {lo, lo + 1}, (t, coded, lo)
        assert coded.count(lo + 1) == (8 * f + 128) >> 8, (t, coded, f)
        seen_frac += f > 0
    enc.close()
    assert seen_frac > 0   # the controller used fractional QPs
