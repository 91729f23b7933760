"""Production capture loop (csrc/runtime/capture.cpp): per-frame callback, step mode,
two frames in flight, pool source, latency record. The gpu-marked twins run the same
loop on the HIP encoder (the path the server uses on an MI355X) and decode every
stripe with the independent H.264 decoder."""
import ctypes
import threading
import time

import numpy as np
import pytest

from selkies_gstreamer_amd.models.h264.decoder import H264Decoder
from selkies_gstreamer_amd.ops.native import PinnedBuffer
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop


def _pool(W, H, n=4, kind="motion"):
    src = SyntheticDesktop(W, H, kind=kind, seed=3)
    pool = PinnedBuffer((n, H, W, 4))
    for i in range(n):
        src.frame(i, out=pool.array[i])
    return pool


def _run_step(use_cpu: int, W=256, H=128, frames=6, fullframe=0, kind="motion"):
    import pixelflux
    pool = _pool(W, H, kind=kind)
    got = []
    lock = threading.Lock()

    def on_frame(res, n, user):
        with lock:
            got.append([(res[i].frame_id, res[i].stripe_y_start, res[i].stripe_height,
                         ctypes.string_at(res[i].data, res[i].size)) for i in range(n)])

    s = pixelflux.default_settings(W, H, use_cpu=use_cpu, source=pixelflux.SOURCE_POOL, step_mode=1,
                                   pool_frames=4, pool_stride=W * 4, stripe_height=64,
                                   use_paint_over_quality=0, h264_fullframe=fullframe)
    s.pool = pool.array.ctypes.data
    cap = pixelflux.ScreenCapture()
    cb = pixelflux.FrameCallback(on_frame)
    cap.start_frame_capture(s, cb)
    cap.run(frames)
    assert cap.wait(120_000) == 0
    lat = cap.latencies()
    st = cap.stats()
    cap.close()
    return pool, got, lat, st


def _check_stream(pool, got, W, H, frames):
    assert len(got) == frames                       # one callback per frame, in order
    fids = [f[0][0] for f in got if f]
    assert fids == sorted(fids)
    decs = {}
    for t, fr in enumerate(got):
        for fid, y, h, data in fr:
            assert data[0] == 0x04 and int.from_bytes(data[2:4], "big") == fid
            if data[1] == 1:
                decs[y] = H264Decoder()
            assert len(decs[y].decode(data[10:])) == 1
    assert set(decs) == set(range(0, H, 64))


def test_step_mode_cpu():
    pool, got, lat, st = _run_step(use_cpu=1)
    _check_stream(pool, got, 256, 128, 6)
    assert len(lat) == 6 and all(x > 0 for x in lat)
    assert st["frames"] == 6


def test_paced_session_keeps_rate_cpu():
    import pixelflux
    n = [0]

    def on_frame(res, k, user):
        n[0] += 1

    s = pixelflux.default_settings(128, 64, use_cpu=1, source=2, target_fps=20.0, stripe_height=64)
    cap = pixelflux.ScreenCapture()
    cb = pixelflux.FrameCallback(on_frame)
    cap.start_frame_capture(s, cb)
    time.sleep(1.0)
    cap.stop_capture()
    cap.close()
    assert 10 <= n[0] <= 26


def test_step_wait_times_out_without_budget_cpu():
    import pixelflux
    pool = _pool(128, 64)
    s = pixelflux.default_settings(128, 64, use_cpu=1, source=pixelflux.SOURCE_POOL, step_mode=1,
                                   pool_frames=4, pool_stride=128 * 4, stripe_height=64)
    s.pool = pool.array.ctypes.data
    cap = pixelflux.ScreenCapture()
    cap.start_frame_capture(s, ctypes.cast(None, pixelflux.FrameCallback))
    assert cap.wait(50) == 0          # nothing granted: nothing pending
    cap.run(2)
    assert cap.wait(60_000) == 0
    assert cap.stats()["frames"] == 2
    cap.close()


@pytest.mark.gpu
def test_step_mode_hip_two_in_flight():
    from selkies_gstreamer_amd.ops.native import require_gpu
    require_gpu()
    pool, got, lat, st = _run_step(use_cpu=0, W=640, H=256, frames=12)
    _check_stream(pool, got, 640, 256, 12)
    assert st["frames"] == 12 and len(lat) == 12


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["motion", "desktop"])
def test_hip_capture_matches_cpu_capture(kind):
    """Same pool through the HIP and the CPU capture loops: byte-identical packets. On
    desktop content the HIP loop uploads only the rows the pool source reports as damaged
    (what XDamage gives a display): fewer rows cross PCIe, same bytes out."""
    from selkies_gstreamer_amd.ops.native import require_gpu
    require_gpu()
    _, g_hip, _, st = _run_step(use_cpu=0, W=320, H=192, frames=9, kind=kind)
    _, g_cpu, _, _ = _run_step(use_cpu=1, W=320, H=192, frames=9, kind=kind)
    assert [[d for *_, d in f] for f in g_hip] == [[d for *_, d in f] for f in g_cpu]
    if kind == "desktop":
        assert st["upload_fraction"] < 0.8, st["upload_fraction"]
    else:
        assert st["upload_fraction"] > 0.95


@pytest.mark.gpu
def test_paced_hip_session_synthetic_decodes():
    import pixelflux
    from selkies_gstreamer_amd.ops.native import require_gpu
    require_gpu()
    got = []

    def on_frame(res, n, user):
        got.append([(res[i].stripe_y_start, ctypes.string_at(res[i].data, res[i].size)) for i in range(n)])

    s = pixelflux.default_settings(640, 384, use_cpu=0, source=1, target_fps=60.0, stripe_height=64)
    cap = pixelflux.ScreenCapture()
    cb = pixelflux.FrameCallback(on_frame)
    cap.start_frame_capture(s, cb)
    time.sleep(1.0)
    cap.stop_capture()
    st = cap.stats()
    lat = cap.latencies()
    cap.close()
    assert 40 <= st["frames"] <= 70          # paced at 60 fps
    assert np.median(lat) < 16.7             # each frame done well inside its tick
    decs = {}
    for fr in got:
        for y, data in fr:
            if data[1] == 1:
                decs[y] = H264Decoder()
            assert len(decs[y].decode(data[10:])) == 1


def test_upload_ranges_clamp_bad_pairs():
    """Damage rows reach the HIP upload from the public API (set_upload_rows): negative,
    inverted, empty and out-of-frame pairs must not index outside the frame (the band
    union is clamped to [0, rows); bad pairs contribute nothing)."""
    from selkies_gstreamer_amd.ops.native import upload_ranges
    assert upload_ranges([(0, 16)], 64) == [(0, 16)]
    assert upload_ranges([(5, 20)], 64) == [(0, 32)]                  # 16-row bands
    assert upload_ranges([(-64, 8)], 64) == [(0, 16)]                 # negative start clamped
    assert upload_ranges([(-100, -20)], 64) == []                     # wholly before the frame
    assert upload_ranges([(40, 10), (30, 30)], 64) == []              # inverted / empty
    assert upload_ranges([(50, 1000)], 60) == [(48, 60)]              # past the end, partial band
    assert upload_ranges([(0, 8), (16, 20), (48, 50)], 64) == [(0, 32), (48, 64)]
    assert upload_ranges([(2**31 - 1, -2**31)], 64) == []
    assert upload_ranges([], 64) == []
