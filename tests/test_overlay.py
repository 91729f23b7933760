"""K12 watermark / K13 cursor composite fused into the colour conversion: encoding a
frame with an encoder overlay must give exactly the bitstream of encoding the frame
composited beforehand with the same integer blend (csrc/codec/overlay.h), on both
backends, for placed, clipped, tiled and moving overlays. The input frame is never
written."""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder, HevcEncoder, hip_device_count
from tests.h264_util import synthetic_frames


def premul(rng, h, w):
    img = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    img[..., 3] = np.where(rng.random((h, w)) < 0.2, 0, img[..., 3])   # fully transparent pixels
    img[..., :3] = (img[..., :3].astype(np.uint32) * img[..., 3:4] // 255).astype(np.uint8)
    return img


def composite(frame, img, x, y, tile=None):
    out = frame.copy()
    H, W = frame.shape[:2]
    h, w = img.shape[:2]
    ys, xs = np.mgrid[0:H, 0:W]
    dx, dy = xs - x, ys - y
    ok = (dx >= 0) & (dy >= 0)
    if tile:
        dx, dy = dx % tile[0], dy % tile[1]
    ok &= (dx < w) & (dy < h)
    src = img[np.clip(dy, 0, h - 1), np.clip(dx, 0, w - 1)].astype(np.uint32)
    a = src[..., 3:4]
    d = out[..., :3].astype(np.uint32)
    blended = ((src[..., :3] + (d * (255 - a) + 127) // 255) & 255).astype(np.uint8)
    m = ok & (a[..., 0] > 0)
    out[..., :3][m] = blended[m]
    return out


@pytest.mark.parametrize("place", ["inside", "clipped", "tiled"])
def test_overlay_equals_precomposited_cpu(place):
    W, H = 200, 120
    rng = np.random.default_rng(3)
    img = premul(rng, 24, 40)
    x, y, tile = {"inside": (30, 20, None), "clipped": (180, 110, None), "tiled": (5, 7, (60, 40))}[place]
    a = H264Encoder(W, H, stripe_height=32, qp=24)
    b = H264Encoder(W, H, stripe_height=32, qp=24)
    a.set_overlay(0, img)
    for t, f in enumerate(synthetic_frames(W, H, 4, seed=2)):
        keep = f.copy()
        xx = x + 3 * t   # the overlay moves: damage follows it
        a.set_overlay_pos(0, xx, y, tile)
        pa = a.encode(f, t)
        assert np.array_equal(f, keep), "the captured frame must not be written"
        pb = b.encode(composite(f, img, xx, y, tile), t)
        assert [p.data for p in pa] == [p.data for p in pb], f"frame {t}"


def test_two_overlays_and_disable():
    W, H = 160, 96
    rng = np.random.default_rng(5)
    wm, cur = premul(rng, 16, 48), premul(rng, 20, 12)
    a, b = H264Encoder(W, H, qp=26), H264Encoder(W, H, qp=26)
    a.set_overlay(0, wm)
    a.set_overlay(1, cur)
    frames = list(synthetic_frames(W, H, 3, seed=4))
    a.set_overlay_pos(0, 100, 70)
    a.set_overlay_pos(1, 20, 30)
    assert [p.data for p in a.encode(frames[0], 0)] == \
        [p.data for p in b.encode(composite(composite(frames[0], wm, 100, 70), cur, 20, 30), 0)]
    a.set_overlay_pos(1, 0, 0, enabled=False)
    assert [p.data for p in a.encode(frames[1], 1)] == [p.data for p in b.encode(composite(frames[1], wm, 100, 70), 1)]
    a.set_overlay(0, None)
    assert [p.data for p in a.encode(frames[2], 2)] == [p.data for p in b.encode(frames[2], 2)]


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["h264", "hevc"])
def test_overlay_gpu_matches_cpu(codec):
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    W, H = 256, 144
    rng = np.random.default_rng(9)
    wm, cur = premul(rng, 30, 70), premul(rng, 32, 32)
    cls = H264Encoder if codec == "h264" else HevcEncoder
    kw = dict(stripe_height=32) if codec == "h264" else {}
    g, c = cls(W, H, backend="hip", **kw), cls(W, H, backend="cpu", **kw)
    for e in (g, c):
        e.set_overlay(0, wm)
        e.set_overlay(1, cur)
    for t, f in enumerate(synthetic_frames(W, H, 6, seed=8)):
        for e in (g, c):
            e.set_overlay_pos(0, 10, 5, (90, 50) if t % 2 else None)
            e.set_overlay_pos(1, 7 * t + 200, 4 * t, enabled=t != 3)   # moving cursor, clipped at the edge
        pg, pc = g.encode(f, t), c.encode(f, t)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}"
