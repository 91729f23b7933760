"""HEVC quarter-pel motion: the shared K4c refinement (k_subpel / subpel_refine) gives
P CUs fractional vectors, and the HEVC back ends predict them with the spec's 8-tap luma
filters (hevc_core.h luma_mc_sample, the LDS-staged separable pass in k_hevc_inter). The
independent decoder (models/hevc/decoder.py, its own Table 8-12 filters) must rebuild the
encoder's reconstruction exactly; sub-pixel motion must cost fewer bits than integer-only
vectors; the HIP back end must write the CPU reference's bytes."""
import numpy as np
import pytest

from selkies_gstreamer_amd.models.hevc.decoder import HevcDecoder
from selkies_gstreamer_amd.ops.native import ME_DTYPE, HevcEncoder, hip_device_count
from tests.test_h264_subpel import subpixel_scene


def _rec_y(enc, W, H):
    pw = (W + 15) // 16 * 16
    return np.frombuffer(enc.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, pw)[:H, :W]


def _frac(enc):
    me = enc.debug_buffer("me", ME_DTYPE)
    return int(np.count_nonzero((me["fx"] != 0) | (me["fy"] != 0)))


def test_hevc_subpel_reconstruction_matches_decoder():
    W, H = 192, 128
    enc = HevcEncoder(W, H, backend="cpu", qp=24, use_paint_over=False)
    dec = HevcDecoder()
    frac = 0
    for t, f in enumerate(subpixel_scene(W, H, 6)):
        pk = enc.encode(f, t)
        Y = dec.decode(pk[0].data[10:])[0][0]
        assert np.array_equal(Y, _rec_y(enc, W, H)), f"frame {t}: decoder != encoder reconstruction"
        if t:
            frac += _frac(enc)
    assert frac > 20   # fractional vectors are really coded


def test_hevc_subpel_saves_bits_on_subpixel_motion():
    W, H = 192, 128
    frames = subpixel_scene(W, H, 8)
    bits = {}
    for sp in (False, True):
        enc = HevcEncoder(W, H, backend="cpu", qp=26, use_paint_over=False, subpel=sp)
        bits[sp] = sum(len(p.data) for t, f in enumerate(frames) for p in enc.encode(f, t) if t > 0)
    assert bits[True] < 0.95 * bits[False], bits


@pytest.mark.gpu
def test_hevc_subpel_gpu_matches_cpu():
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    W, H = 256, 160
    g = HevcEncoder(W, H, qp=24, backend="hip", use_paint_over=False)
    c = HevcEncoder(W, H, qp=24, backend="cpu", use_paint_over=False)
    frac = 0
    for t, f in enumerate(subpixel_scene(W, H, 8)):
        pg, pc = g.encode(f, t), c.encode(f, t)
        mg, mc = g.debug_buffer("me", ME_DTYPE), c.debug_buffer("me", ME_DTYPE)
        if t:
            assert np.array_equal(mg["fx"], mc["fx"]) and np.array_equal(mg["fy"], mc["fy"]), f"frame {t}"
            frac += _frac(g)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}"
    assert frac > 20
