"""Quarter-pel motion (K4c): the encoder refines P vectors to quarter-sample precision
with the 6-tap interpolation (h264_core.h luma_qpel_sample); the independent decoder
(models/h264/decoder.py, its own vectorised Table 8-12) must reconstruct exactly the
encoder's reference picture, and sub-pixel motion must cost fewer bits than with
integer vectors only."""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder, ME_DTYPE, hip_device_count
from tests.h264_util import StripeDecoder


def subpixel_scene(W, H, n, step=0.37):
    """Smooth texture translating by a non-integer number of pixels per frame."""
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    out = []
    for t in range(n):
        x = xx - step * t * 2.0
        y = yy - step * t
        v = 128 + 60 * np.sin(x / 5.3) * np.cos(y / 7.1) + 40 * np.sin((x + y) / 11.0)
        f = np.zeros((H, W, 4), np.uint8)
        f[..., 0] = np.clip(v, 0, 255)
        f[..., 1] = np.clip(255 - v, 0, 255)
        f[..., 2] = np.clip(v * 0.5 + 60, 0, 255)
        out.append(f)
    return out


@pytest.mark.parametrize("fullframe", [False, True])
def test_subpel_reconstruction_matches_decoder(fullframe):
    W, H = 192, 128
    enc = H264Encoder(W, H, stripe_height=32, fullframe=fullframe, qp=24, use_paint_over=False)
    dec = StripeDecoder(W, H)
    frac = 0
    for t, f in enumerate(subpixel_scene(W, H, 6)):
        for p in enc.encode(f, t):
            dec.feed(p.data)
        me = enc.debug_buffer("me", ME_DTYPE)
        frac += int(np.count_nonzero((me["fx"] != 0) | (me["fy"] != 0)))
        ref = np.frombuffer(enc.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, (W + 15) // 16 * 16)[:H, :W]
        assert np.array_equal(dec.Y, ref), f"frame {t}: decoder != encoder reconstruction"
    assert frac > 20   # the refinement is really used


def test_subpel_saves_bits_on_subpixel_motion():
    W, H = 192, 128
    frames = subpixel_scene(W, H, 8)
    bits = {}
    for sp in (False, True):
        enc = H264Encoder(W, H, stripe_height=32, qp=26, use_paint_over=False, subpel=sp)
        bits[sp] = sum(len(p.data) for t, f in enumerate(frames) for p in enc.encode(f, t) if t > 0)
    assert bits[True] < 0.95 * bits[False], bits


@pytest.mark.gpu
@pytest.mark.parametrize("num_refs", [1, 2])
def test_subpel_gpu_matches_cpu(num_refs):
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    W, H = 256, 160
    g = H264Encoder(W, H, stripe_height=32, qp=24, backend="hip", num_refs=num_refs)
    c = H264Encoder(W, H, stripe_height=32, qp=24, backend="cpu", num_refs=num_refs)
    for t, f in enumerate(subpixel_scene(W, H, 8)):
        pg, pc = g.encode(f, t), c.encode(f, t)
        mg, mc = g.debug_buffer("me", ME_DTYPE), c.debug_buffer("me", ME_DTYPE)
        assert np.array_equal(mg["fx"], mc["fx"]) and np.array_equal(mg["fy"], mc["fy"]), f"frame {t}"
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}"


def _frac_count(enc):
    me = enc.debug_buffer("me", ME_DTYPE)
    return int(np.count_nonzero((me["fx"] != 0) | (me["fy"] != 0)))


def _texture(W, H, dx, dy):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    x, y = xx - dx, yy - dy
    v = 128 + 60 * np.sin(x / 5.3) * np.cos(y / 7.1) + 40 * np.sin((x + y) / 11.0)
    f = np.zeros((H, W, 4), np.uint8)
    f[..., 0] = np.clip(v, 0, 255)
    f[..., 1] = np.clip(255 - v, 0, 255)
    f[..., 2] = np.clip(v * 0.5 + 60, 0, 255)
    return f


def test_subpel_gate_skips_integer_motion_and_probes():
    """Adaptive refinement (h264_frame.h subpel_gate): after a probe frame that found no
    fractional vector, the refinement is off until the next probe (every 8th P frame of
    a stripe, frame_num % 8 == 1); once a probe finds fractional motion it stays on."""
    W, H = 192, 128
    # frame 1 (first P = probe): a whole-pixel shift; then sub-pixel motion from frame 2 on
    shifts = [(0.0, 0.0), (2.0, 0.0)] + [(2.0 + 0.74 * k, 0.37 * k) for k in range(1, 13)]
    enc = H264Encoder(W, H, stripe_height=32, qp=12, use_paint_over=False)
    counts = []
    for t, (dx, dy) in enumerate(shifts):
        enc.encode(_texture(W, H, dx, dy), t)
        counts.append(_frac_count(enc))
    assert counts[1] * 128 < W * H // 256, counts   # probe: integer motion -> gate closes
    assert all(c == 0 for c in counts[2:9]), counts  # gate closed: sub-pixel motion ignored
    assert counts[9] > 0, counts                     # frame_num 9: probe finds the sub-pixel motion
    assert all(c > 0 for c in counts[10:]), counts   # and the gate stays open


def test_subpel_gate_survives_state_migration():
    W, H = 192, 128
    frames = subpixel_scene(W, H, 6)
    a = H264Encoder(W, H, stripe_height=32, qp=24, use_paint_over=False)
    b = H264Encoder(W, H, stripe_height=32, qp=24, use_paint_over=False)
    for t in range(3):
        a.encode(frames[t], t)
    b.import_state(a.export_state())
    for t in range(3, 6):
        pa = [p.data for p in a.encode(frames[t], t)]
        pb = [p.data for p in b.encode(frames[t], t)]
        assert pa == pb
