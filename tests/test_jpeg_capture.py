"""JPEG stripe encoder (CPU reference) and the pixelflux-compatible capture API.

JPEG stripes are decoded with PIL (libjpeg) and compared with a float JFIF
conversion of the source; the capture session runs with the synthetic source
and the CPU encoders so it is exercised without a GPU or an X server.
"""
import io
import threading
import time

import numpy as np
import pytest
from PIL import Image

from selkies_gstreamer_amd.ops.native import JpegEncoder
from tests.h264_util import StripeDecoder, synthetic_frames


def _rgb(bgrx):
    return bgrx[..., 2::-1].astype(np.float64)


def _psnr(a, ref):
    mse = np.mean((a.astype(np.float64) - ref) ** 2)
    return 10 * np.log10(255 ** 2 / max(mse, 1e-9))


def _decode_jpeg_packet(p):
    fid = int.from_bytes(p[0:2], "big")
    y = int.from_bytes(p[2:4], "big")
    img = Image.open(io.BytesIO(p[4:]))
    assert img.format == "JPEG" and img.mode == "RGB"
    return fid, y, np.asarray(img)


@pytest.mark.parametrize("w,h,sh", [(320, 200, 64), (250, 90, 32), (64, 16, 16)])
def test_jpeg_stripes_decode(w, h, sh):
    frames = list(synthetic_frames(w, h, 3, kind="desktop"))
    enc = JpegEncoder(w, h, stripe_height=sh, quality=85, paint_quality=95)
    canvas = np.zeros((h, w, 3), np.uint8)
    for t, f in enumerate(frames):
        pk = enc.encode(f, frame_id=t)
        if t == 0:
            assert len(pk) == (h + sh - 1) // sh  # everything is sent first
        for p in pk:
            fid, y, rgb = _decode_jpeg_packet(p.data)
            assert fid == t and y == p.y and rgb.shape == (p.h, w, 3)
            canvas[y:y + p.h] = rgb
        # same quality as libjpeg's own 4:2:0 encode of the frame (per stripe)
        ref = _rgb(f)
        pil = np.zeros_like(canvas)
        for y in range(0, h, sh):
            buf = io.BytesIO()
            Image.fromarray(np.ascontiguousarray(f[y:y + sh, :, 2::-1])).save(buf, "JPEG", quality=85,
                                                                            subsampling=2)
            pil[y:y + sh] = np.asarray(Image.open(buf))
        assert _psnr(canvas, ref) > _psnr(pil, ref) - 0.3


def test_jpeg_damage_and_paint_over():
    w, h = 128, 128
    f = next(synthetic_frames(w, h, 1, kind="desktop"))
    enc = JpegEncoder(w, h, stripe_height=32, quality=30, paint_quality=90, paint_over_trigger=3)
    assert len(enc.encode(f, 0)) == 4
    g = f.copy()
    g[40:50, 10:20, :3] ^= 0x55  # damage in stripe 1 only
    pk = enc.encode(g, 1)
    assert [p.y for p in pk] == [32]
    sizes = {}
    for t in range(2, 8):
        for p in enc.encode(g, t):
            sizes.setdefault(p.y, []).append((t, len(p.data)))
    # every stripe gets exactly one paint-over (higher quality -> bigger) after 3 static frames
    assert sorted(sizes) == [0, 32, 64, 96]
    for y, lst in sizes.items():
        assert len(lst) == 1
    enc.request_keyframe()
    assert len(enc.encode(g, 9)) == 4


def test_jpeg_quality_monotonic():
    w, h = 192, 64
    f = next(synthetic_frames(w, h, 1, kind="noise"))
    size = []
    for q in (10, 50, 95):
        enc = JpegEncoder(w, h, stripe_height=64, quality=q, use_paint_over=False)
        size.append(sum(len(p.data) for p in enc.encode(f, 0)))
    assert size[0] < size[1] < size[2]


def _collect(settings, seconds=0.6):
    import pixelflux
    got, lock = [], threading.Lock()

    def cb(res_ptr, user):
        r = res_ptr.contents
        with lock:
            got.append((r.type, r.frame_id, r.stripe_y_start, r.stripe_height, bytes(r.data[:r.size])))

    cap = pixelflux.ScreenCapture()
    cap.start_capture(settings, pixelflux.StripeCallback(cb))
    time.sleep(seconds)
    cap.stop_capture()
    st = cap.stats()  # after stop: no callback can race the counters
    cap.close()
    return got, st


def test_capture_session_h264_synthetic():
    import pixelflux
    s = pixelflux.default_settings(256, 128, use_cpu=1, source=2, target_fps=30.0, stripe_height=64)
    got, st = _collect(s)
    assert st["frames"] >= 3 and st["source"] == "synthetic"
    assert got and all(t == 1 for t, *_ in got)
    dec = StripeDecoder(256, 128)
    n = 0
    for _, fid, y, sh, data in got:
        assert data[0] == 0x04 and int.from_bytes(data[2:4], "big") == fid
        dec.feed(data)
        n += 1
    assert n == st["packets"]
    assert sum(st["encode_ms_counts"]) == st["frames"]   # native per-frame encode histogram


def test_encode_histogram_reaches_prometheus():
    import pixelflux
    from prometheus_client import generate_latest
    from selkies_gstreamer_amd.server.metrics import Metrics
    s = pixelflux.default_settings(256, 128, use_cpu=1, source=2, target_fps=30.0, stripe_height=64)
    cap = pixelflux.ScreenCapture()
    cap.start_capture(s, lambda r, u: None)
    import time
    time.sleep(0.4)
    cap.stop_capture()
    m = Metrics()
    m.capture_started("primary", cap)
    text = generate_latest(m.registry).decode()
    cap.close()
    assert 'selkies_encode_seconds_bucket{display="primary",le="+Inf"}' in text
    assert "selkies_encode_seconds_count" in text


def test_capture_session_jpeg_synthetic():
    import pixelflux
    s = pixelflux.default_settings(160, 96, use_cpu=1, source=1, target_fps=30.0, output_mode=0,
                                   stripe_height=32)
    got, st = _collect(s)
    assert got and all(t == 0 for t, *_ in got)
    for _, fid, y, sh, data in got:
        fid2, y2, rgb = _decode_jpeg_packet(data)
        assert (fid2, y2) == (fid & 0xFFFF, y) and rgb.shape[0] == sh


def test_capture_rejects_x11_only_without_display(monkeypatch):
    import pixelflux
    monkeypatch.delenv("DISPLAY", raising=False)
    s = pixelflux.default_settings(64, 64, use_cpu=1, source=0)
    cap = pixelflux.ScreenCapture()
    with pytest.raises(RuntimeError):
        cap.start_capture(s, lambda r, u: None)
    cap.close()


def test_pcmflux_contract():
    import pcmflux
    s = pcmflux.AudioCaptureSettings()
    s.device_name = b"output.monitor"
    s.sample_rate, s.channels, s.opus_bitrate, s.frame_duration_ms = 48000, 2, 320000, 20
    s.use_vbr = True
    cap = pcmflux.AudioCapture()
    if not pcmflux.available():
        with pytest.raises(RuntimeError):
            cap.start_capture(s, pcmflux.AudioChunkCallback(lambda r, u: None))
    cap.stop_capture()


def test_capture_watermark(tmp_path):
    import pixelflux
    png = tmp_path / "wm.png"
    wm = np.zeros((24, 40, 4), np.uint8)
    wm[..., 0] = 255   # opaque red
    wm[..., 3] = 255
    Image.fromarray(wm, "RGBA").save(png)
    s = pixelflux.default_settings(160, 96, use_cpu=1, source=2, target_fps=30.0, output_mode=0, stripe_height=32,
                                   watermark_path=str(png), watermark_location_enum=3)
    got, _ = _collect(s, 0.4)
    canvas = np.zeros((96, 160, 3), np.uint8)
    for _, fid, y, sh, data in got:
        canvas[y:y + sh] = _decode_jpeg_packet(data)[2]
    # bottom-right, 16 px margin: rows 56..79, cols 104..143
    patch = canvas[60:76, 108:140].astype(int)
    assert patch[..., 0].mean() > 200 and patch[..., 1].mean() < 60 and patch[..., 2].mean() < 60
    assert canvas[10:20, 10:40, 0].mean() < 200 or canvas[10:20, 10:40, 1].mean() > 60  # not red elsewhere


@pytest.mark.parametrize("use_cpu", [1, pytest.param(0, marks=pytest.mark.gpu)])
def test_capture_watermark_h264_in_encoder(tmp_path, use_cpu):
    """H.264 capture sessions blend the watermark inside the encoder's colour conversion
    (K12, overlay.h) instead of writing the grabbed buffer: a pool source (never written)
    gets the watermark in the decoded picture, bottom-right with a 16 px margin."""
    import pixelflux
    from selkies_gstreamer_amd.ops.native import PinnedBuffer, hip_device_count
    if not use_cpu and hip_device_count() < 1:
        pytest.skip("no HIP device")
    png = tmp_path / "wm.png"
    wm = np.zeros((24, 40, 4), np.uint8)
    wm[..., 0] = 255   # opaque red (RGBA)
    wm[..., 3] = 255
    Image.fromarray(wm, "RGBA").save(png)
    W, H = 160, 96
    pool = PinnedBuffer((2, H, W, 4))
    pool.array[:] = 40
    before = pool.array.copy()
    s = pixelflux.default_settings(W, H, use_cpu=use_cpu, source=pixelflux.SOURCE_POOL, step_mode=1, pool_frames=2,
                                   pool_stride=W * 4, stripe_height=32, output_mode=1, watermark_path=str(png),
                                   watermark_location_enum=3)
    s.pool = pool.array.ctypes.data
    got = []

    def cb(res_ptr, user):
        r = res_ptr.contents
        got.append((r.frame_id, r.stripe_y_start, bytes(r.data[:r.size])))
    cap = pixelflux.ScreenCapture()
    cap.start_capture(s, pixelflux.StripeCallback(cb))
    cap.run(3)
    assert cap.wait(30_000) == 0
    cap.stop_capture()
    cap.close()
    assert np.array_equal(pool.array, before), "the captured frames must not be written"
    dec = StripeDecoder(W, H)
    for fid, y, data in got:
        if fid == 0:
            dec.feed(data)
    from tests.h264_util import bgrx_to_y709
    red = np.zeros((1, 1, 4), np.uint8)
    red[..., 2] = 255
    ref_y = int(bgrx_to_y709(red)[0, 0])
    patch = dec.Y[60:76, 108:140].astype(int)
    assert abs(patch.mean() - ref_y) < 4 and abs(int(dec.Y[10, 10]) - int(bgrx_to_y709(before[0, :1, :1])[0, 0])) < 4
