"""K2: capture resampling fused into the K1 colour conversion (codec/color.h).

The encoder's converted luma must equal an independent numpy model of the same
bilinear integer math (centre-aligned, 8-bit weights, edge clamp) followed by the
BT.709 limited-range formula; the stream decodes to the resampled picture; the
HIP kernel matches the CPU reference byte for byte (gpu tier).
"""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder
from tests.h264_util import StripeDecoder, psnr, synthetic_frames


def np_scale(src: np.ndarray, dw: int, dh: int) -> np.ndarray:
    sh, sw = src.shape[:2]
    stx, sty = (sw << 16) // dw, (sh << 16) // dh

    def pos(d, step):
        p = (((2 * d + 1).astype(np.int64) * step) >> 1) - 0x8000
        return np.maximum(p, 0)
    px, py = pos(np.arange(dw), stx), pos(np.arange(dh), sty)
    x0 = np.minimum(px >> 16, sw - 1)
    y0 = np.minimum(py >> 16, sh - 1)
    x1, y1 = np.minimum(x0 + 1, sw - 1), np.minimum(y0 + 1, sh - 1)
    wx, wy = ((px >> 8) & 255)[None, :, None], ((py >> 8) & 255)[:, None, None]
    s = src.astype(np.int64)

    def lerp(a, b, w):
        return (a * (256 - w) + b * w + 128) >> 8
    top = lerp(s[y0][:, x0], s[y0][:, x1], wx)
    bot = lerp(s[y1][:, x0], s[y1][:, x1], wx)
    return lerp(top, bot, wy).astype(np.uint8)


def y709(bgrx):
    b, g, r = (bgrx[..., i].astype(np.int64) for i in range(3))
    return np.clip(((47 * r + 157 * g + 16 * b + 128) >> 8) + 16, 0, 255).astype(np.uint8)


@pytest.mark.parametrize("src,dst", [((320, 192), (160, 96)), ((200, 120), (160, 96)), ((130, 70), (192, 112))])
def test_scaled_luma_matches_model(src, dst):
    (sw, sh), (dw, dh) = src, dst
    enc = H264Encoder(dw, dh, stripe_height=32, qp=24, backend="cpu", src_width=sw, src_height=sh)
    sd = StripeDecoder(dw, dh)
    for t, f in enumerate(synthetic_frames(sw, sh, 3, seed=6)):
        pk = enc.encode(f, t)
        for p in pk:
            sd.feed(p.data)
        want = y709(np_scale(f, dw, dh))
        got = enc.debug_buffer("src_y").reshape(-1, (dw + 15) // 16 * 16)[:dh, :dw]
        assert np.array_equal(got, want), f"frame {t}"
        assert psnr(sd.Y, want) > 32


def test_identity_when_sizes_match():
    f = next(synthetic_frames(160, 96, 1, seed=1))
    a = H264Encoder(160, 96, stripe_height=32, backend="cpu")
    b = H264Encoder(160, 96, stripe_height=32, backend="cpu", src_width=160, src_height=96)
    assert [p.data for p in a.encode(f, 0)] == [p.data for p in b.encode(f, 0)]


@pytest.mark.gpu
def test_hip_scaling_matches_cpu():
    kw = dict(stripe_height=64, qp=25, src_width=1920, src_height=1080)
    cpu = H264Encoder(1280, 720, backend="cpu", **kw)
    gpu = H264Encoder(1280, 720, backend="hip", **kw)
    for t, f in enumerate(synthetic_frames(1920, 1080, 3, seed=2)):
        assert [p.data for p in gpu.encode(f, t)] == [p.data for p in cpu.encode(f, t)], f"frame {t}"
