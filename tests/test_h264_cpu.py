"""CPU reference H.264 encoder: conformance against the independent decoder."""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder, MB_INFO_DTYPE
from tests.h264_util import StripeDecoder, synthetic_frames, bgrx_to_y709, psnr


@pytest.mark.parametrize("num_refs", [1, 2])
@pytest.mark.parametrize("deblock", [False, True])
@pytest.mark.parametrize("fullframe", [False, True])
@pytest.mark.parametrize("kind", ["desktop", "noise"])
def test_cpu_roundtrip_bitexact(fullframe, kind, deblock, num_refs):
    W, H = 160, 96
    enc = H264Encoder(W, H, stripe_height=32, fullframe=fullframe, qp=26, backend="cpu", deblock=deblock,
                      num_refs=num_refs)
    sd = StripeDecoder(W, H)
    for t, f in enumerate(synthetic_frames(W, H, 5, kind=kind)):
        pk = enc.encode(f, t)
        for p in pk:
            sd.feed(p.data)
        ref = enc.debug_buffer("ref_y").reshape(-1, (W + 15) // 16 * 16)[:H, :W]
        assert np.array_equal(sd.Y, ref), f"frame {t}: decoder output != encoder reconstruction"
        for name, plane in (("ref_u", sd.U), ("ref_v", sd.V)):
            buf = enc.debug_buffer(name)
            refc = buf.reshape((H + 15) // 16 * 8, -1)[:H // 2, :W // 2]
            assert np.array_equal(plane, refc), f"frame {t}: decoder {name} != encoder reconstruction"
        assert psnr(sd.Y, bgrx_to_y709(f)) > 30


def test_cpu_odd_size_and_crop():
    W, H = 130, 70  # not MB aligned: cropping in SPS, last stripe shorter
    enc = H264Encoder(W, H, stripe_height=48, qp=22, backend="cpu")
    sd = StripeDecoder(W, H)
    for t, f in enumerate(synthetic_frames(W, H, 3)):
        for p in enc.encode(f, t):
            assert p.h == min(48, H - p.y)
            sd.feed(p.data)
        assert psnr(sd.Y, bgrx_to_y709(f)) > 32


def test_static_stripes_are_not_resent():
    W, H = 128, 128
    enc = H264Encoder(W, H, stripe_height=32, use_paint_over=False, backend="cpu")
    f = next(synthetic_frames(W, H, 1))
    assert len(enc.encode(f, 0)) == 4        # first frame: every stripe, IDR
    assert enc.encode(f, 1) == []            # nothing changed
    g = f.copy()
    g[40:50, 10:20, :3] = 255                # touch stripe 1 only
    pk = enc.encode(g, 2)
    assert [p.y for p in pk] == [32] and not pk[0].key


def test_paint_over_burst():
    W, H = 64, 32
    enc = H264Encoder(W, H, stripe_height=32, qp=30, paint_qp=20, paint_over_trigger=3,
                      paint_over_burst=2, backend="cpu")
    f = next(synthetic_frames(W, H, 1))
    sent = [len(enc.encode(f, t)) for t in range(8)]
    # frame 0 IDR, static for 3 frames -> 2 paint-over frames, then quiet
    assert sent == [1, 0, 0, 1, 1, 0, 0, 0]


def test_keyframe_request_and_frame_id():
    W, H = 64, 64
    enc = H264Encoder(W, H, stripe_height=64, backend="cpu")
    f = next(synthetic_frames(W, H, 1))
    enc.encode(f, 7)
    enc.request_keyframe()
    pk = enc.encode(f, 0x1234)
    assert len(pk) == 1 and pk[0].key
    d = pk[0].data
    assert d[0] == 4 and d[1] == 1 and d[2:4] == b"\x12\x34"
    assert d[10:15] == b"\x00\x00\x00\x01\x67"  # SPS first on keyframes


def test_qp_escalation_bounds_macroblock_size():
    W, H = 64, 64
    enc = H264Encoder(W, H, stripe_height=64, qp=0, paint_qp=0, backend="cpu")
    f = next(synthetic_frames(W, H, 1, kind="noise"))
    pk = enc.encode(f, 0)
    mbs = enc.debug_buffer("mbs", MB_INFO_DTYPE)
    assert mbs["qp"].max() > 0  # noise at QP 0 must escalate
    sd = StripeDecoder(W, H)
    sd.feed(pk[0].data)


def _toggle_frames(W, H, n):
    """A desktop whose caret blinks and a button toggles hover state: frame t
    equals frame t - 2 (what the second reference picture captures)."""
    base = next(synthetic_frames(W, H, 1, seed=4))
    on = base.copy()
    on[20:36, 40:42, :3] = 10                       # caret
    on[60:76, 90:130, :3] = (230, 160, 40)          # highlighted button
    return [base if t % 2 == 0 else on for t in range(n)]


@pytest.mark.parametrize("fullframe", [False, True])
def test_two_reference_pictures_code_toggling_content(fullframe):
    W, H = 160, 96
    frames = _toggle_frames(W, H, 8)
    sizes = {}
    for refs in (1, 2):
        enc = H264Encoder(W, H, stripe_height=32, fullframe=fullframe, qp=24, use_paint_over=False,
                          backend="cpu", num_refs=refs)
        sd = StripeDecoder(W, H)
        total = 0
        for t, f in enumerate(frames):
            pk = enc.encode(f, t)
            for p in pk:
                sd.feed(p.data)
                if t >= 2:
                    total += len(p.data)
            ref = enc.debug_buffer("ref_y").reshape(-1, (W + 15) // 16 * 16)[:H, :W]
            assert np.array_equal(sd.Y, ref), f"refs={refs} frame {t}: decoder != encoder reconstruction"
        sizes[refs] = total
    assert sizes[2] < 0.6 * sizes[1], sizes      # the toggle is a near-free ref_idx 1 copy


def test_cpu_backend_queues_two_submitted_frames():
    """The synchronous backends queue each submitted frame's packets, so the
    two-frames-in-flight call pattern (submit n+1 before finish n) works on them too."""
    W, H = 160, 96
    frames = list(synthetic_frames(W, H, 5, seed=9))
    a = H264Encoder(W, H, stripe_height=32, qp=26, backend="cpu")
    ref = [[p.data for p in a.encode(f, t)] for t, f in enumerate(frames)]
    b = H264Encoder(W, H, stripe_height=32, qp=26, backend="cpu")
    got = []
    b.submit(frames[0], 0)
    for t in range(len(frames)):
        if t + 1 < len(frames):
            b.submit(frames[t + 1], t + 1)
        got.append([p.data for p in b.finish()])
    assert got == ref
    with pytest.raises(RuntimeError):
        b.finish()


def _deblock_idc(nal: bytes) -> int:
    """disable_deblocking_filter_idc of a P / I slice NAL of this encoder's streams
    (Baseline, POC type 2, frame_num 16 bits: codec/h264_syntax.h write_slice_header)."""
    from selkies_gstreamer_amd.models.h264.decoder import BitReader, unescape
    r = BitReader(unescape(nal[1:]))
    r.ue()                                    # first_mb_in_slice
    st = r.ue() % 5                           # slice_type
    r.ue()                                    # pic_parameter_set_id
    r.u(16)                                   # frame_num
    idr = (nal[0] & 31) == 5
    if idr:
        r.ue()                                # idr_pic_id
    if st == 0:
        if r.u(1):                            # num_ref_idx_active_override_flag
            r.ue()
        r.u(1)                                # ref_pic_list_modification_flag_l0 (0)
    r.u(2 if idr else 1)                      # dec_ref_pic_marking
    r.se()                                    # slice_qp_delta
    return r.ue()


@pytest.mark.parametrize("qp,idc", [(26, 1), (38, 2)])
def test_auto_deblock_follows_slice_qp(qp, idc):
    """deblock='auto' (the default): slices coded at QP >= 34 are deblocked (idc 2), those
    below are not (idc 1, the CRF-25 default stays x264-ultrafast-like); the independent
    decoder reproduces the encoder's reference either way."""
    W, H = 160, 96
    enc = H264Encoder(W, H, stripe_height=32, qp=qp, paint_qp=qp, use_paint_over=False, backend="cpu")
    sd = StripeDecoder(W, H)
    seen = set()
    for t, f in enumerate(synthetic_frames(W, H, 4, kind="desktop")):
        for p in enc.encode(f, t):
            sd.feed(p.data)
            for nal in p.data[10:].split(b"\x00\x00\x00\x01")[1:]:
                if nal[0] & 31 in (1, 5):
                    seen.add(_deblock_idc(nal))
        ref = enc.debug_buffer("ref_y").reshape(-1, (W + 15) // 16 * 16)[:H, :W]
        assert np.array_equal(sd.Y, ref), f"frame {t}"
    assert seen == {idc}
