"""HEVC Main encoder (CPU reference backend) against the independent test decoder
(models/hevc/decoder.py): every packet must decode, the decoder's picture must equal
the encoder's reconstruction bit-exactly (so encoder and decoder agree on every
normative process), and the picture must be close to the source."""
import numpy as np
import pytest

from selkies_gstreamer_amd.models.hevc.decoder import HevcDecoder, psnr, split_annexb
from selkies_gstreamer_amd.ops.native import HevcEncoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop


CUINFO = 40   # sizeof(hevc::CuInfo)


def _rec_y(enc, W, H):
    pw = (W + 15) // 16 * 16
    return np.frombuffer(enc.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, pw)[:H, :W]


def _luma(f):
    # BT.709 limited range, same as the encoder's K1 conversion up to rounding
    return (0.2126 * f[..., 2] + 0.7152 * f[..., 1] + 0.0722 * f[..., 0]) * 219 / 255 + 16


def _run(W, H, kind, frames, **kw):
    src = SyntheticDesktop(W, H, kind=kind)
    enc = HevcEncoder(W, H, backend="cpu", **kw)
    dec = HevcDecoder()
    out = []
    for t in range(frames):
        f = src.frame(t)
        pk = enc.encode(f, t)
        assert len(pk) == 1 and pk[0].y == 0 and pk[0].w == W and pk[0].h == H
        pics = dec.decode(pk[0].data[10:])
        assert len(pics) == 1
        Y, U, V = pics[0]
        assert Y.shape == (H, W) and U.shape == ((H + 1) // 2, (W + 1) // 2)
        assert np.array_equal(Y, _rec_y(enc, W, H)), f"frame {t}: decoder != encoder reconstruction"
        out.append((pk[0], Y, psnr(Y, _luma(f))))
    enc.close()
    return out


@pytest.mark.parametrize("W,H,kind", [(64, 32, "motion"), (256, 144, "motion"), (200, 100, "desktop"),
                                      (128, 64, "noise")])
def test_hevc_cpu_roundtrip(W, H, kind):
    res = _run(W, H, kind, 4)
    assert res[0][0].key and not res[1][0].key
    for pk, Y, q in res:
        assert q > 30, q


def test_hevc_bitstream_structure():
    W, H = 160, 96            # 10 x 6 CTBs, stripes of 4 CTB rows -> 2 slices
    enc = HevcEncoder(W, H, backend="cpu", stripe_height=64)
    src = SyntheticDesktop(W, H, kind="motion")
    key = enc.encode(src.frame(0), 0)[0].data[10:]
    types = [(n[0] >> 1) & 63 for n in split_annexb(key)]
    assert types == [32, 33, 34, 19, 19]            # VPS SPS PPS + two IDR_W_RADL slices
    p = enc.encode(src.frame(1), 1)[0].data[10:]
    assert [(n[0] >> 1) & 63 for n in split_annexb(p)] == [1, 1]   # TRAIL_R slices
    enc.request_keyframe()
    k2 = enc.encode(src.frame(2), 2)[0]
    assert k2.key and [(n[0] >> 1) & 63 for n in split_annexb(k2.data[10:])][:3] == [32, 33, 34]
    enc.close()


def test_hevc_static_content_is_all_skip():
    W, H = 128, 64
    enc = HevcEncoder(W, H, backend="cpu")
    f = SyntheticDesktop(W, H, kind="desktop").frame(0)
    dec = HevcDecoder()
    first = enc.encode(f, 0)[0]
    dec.decode(first.data[10:])
    sizes = []
    for t in range(1, 4):
        pk = enc.encode(f, t)[0]
        Y = dec.decode(pk.data[10:])[0][0]
        assert np.array_equal(Y, _rec_y(enc, W, H))
        sizes.append(len(pk.data))
    assert max(sizes) < 60   # skip-all slices: a few bytes each
    cus = np.frombuffer(enc.debug_buffer("cus", np.uint8), np.uint8).reshape(-1, CUINFO)
    assert (cus[:, 0] == 0).all()   # CU_SKIP
    assert (cus[:, 22] & 1).all()   # complete CTBs: one skipped 32x32 CU each
    enc.close()


def test_hevc_qp_changes_size():
    W, H = 128, 64
    a = _run(W, H, "noise", 2, qp=22)
    b = _run(W, H, "noise", 2, qp=38)
    assert len(b[1][0].data) < len(a[1][0].data)
    assert a[1][2] > b[1][2]


@pytest.mark.parametrize("kind,qp", [("motion", 22), ("noise", 30), ("desktop", 37)])
def test_hevc_chunk_parallel_cabac_model_is_exact(kind, qp, monkeypatch):
    """The chunk-parallel substream coder (codec/hevc_pcabac.h: context chains, range
    maps, composition, per-CTB coding from V = 0, tail merge) -- the algorithm the HIP
    back end runs -- writes the same bytes as the serial CABAC coder."""
    W, H = 192, 128
    src = SyntheticDesktop(W, H, kind=kind)
    ref = HevcEncoder(W, H, backend="cpu", stripe_height=64, qp=qp)
    monkeypatch.setenv("SK_HEVC_PCABAC", "1")
    par = HevcEncoder(W, H, backend="cpu", stripe_height=64, qp=qp)
    for t in range(4):
        f = src.frame(t)
        a = [p.data for p in ref.encode(f, t)]
        b = [p.data for p in par.encode(f, t)]
        assert a == b, f"frame {t}"


def _diagonal(W, H):
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    v = 128 + 90 * np.sin((xx * 0.8 + yy * 0.45) / 3.1)
    f = np.zeros((H, W, 4), np.uint8)
    f[..., 0] = f[..., 1] = f[..., 2] = np.clip(v, 0, 255)
    return f


def test_hevc_directional_intra_modes():
    """All 35 luma modes are searched (hevc_core.h HEVC_INTRA_ORDER): oriented texture picks
    directional modes, the decoder's 8.4.4.2.6 prediction rebuilds the encoder's picture,
    and the key frame is far smaller than with planar / DC / H / V alone (it was 9996
    bytes at QP 22 with the four modes, profiles/r3_hevc_tools.md)."""
    W, H = 384, 256
    f = _diagonal(W, H)
    enc = HevcEncoder(W, H, backend="cpu", qp=22)
    pk = enc.encode(f, 0)[0]
    Y = HevcDecoder().decode(pk.data[10:])[0][0]
    assert np.array_equal(Y, _rec_y(enc, W, H))
    modes = np.frombuffer(enc.debug_buffer("cus", np.uint8), np.uint8).reshape(-1, CUINFO)[:, 24:40]
    assert np.count_nonzero(~np.isin(modes, [0, 1, 10, 26])) > modes.size // 2
    assert len(pk.data) < 7500, len(pk.data)   # (levels round to 0.47: a little more detail, PSNR > 45)
    assert psnr(Y, _luma(f)) > 45


def _cus(enc):
    c = np.frombuffer(enc.debug_buffer("cus", np.uint8), np.uint8).reshape(-1, CUINFO)
    tu = c[:, 6]
    tsy = c[:, 18].astype(np.int64) | (c[:, 19].astype(np.int64) << 8)
    return c[:, 0], tu, tsy, c[:, 20]


def test_hevc_transform_tree_tools():
    """Residual quadtree (hevc_core.h code_cu, max_transform_hierarchy_depth 2): on text-like
    content the RD choices use 16x16, 8x8 and 4x4 TUs (DST for intra 4x4 luma), transform
    skip on 4x4 luma and chroma, in I and P pictures, and the decoder's Y, Cb and Cr equal
    the encoder's reconstruction (inner TU edges deblocked on both sides alike)."""
    W, H = 256, 144
    src = SyntheticDesktop(W, H, kind="motion")
    enc = HevcEncoder(W, H, backend="cpu", qp=27)
    dec = HevcDecoder()
    cw = (W + 1) // 2
    seen = {"split": 0, "whole": 0, "split8": 0, "ts": 0, "inter_split": 0}
    for t in range(3):
        pk = enc.encode(src.frame(t), t)[0]
        Y, U, V = dec.decode(pk.data[10:])[0]
        assert np.array_equal(Y, _rec_y(enc, W, H))
        pcw = (W + 15) // 16 * 8
        for name, P in (("ref_u", U), ("ref_v", V)):
            rec = np.frombuffer(enc.debug_buffer(name, np.uint8), np.uint8).reshape(-1, pcw)[:(H + 1) // 2, :cw]
            assert np.array_equal(P, rec), name
        mode, tu, tsy, tsc = _cus(enc)
        split = (tu & 16) != 0
        seen["split"] += int(split.sum())
        seen["whole"] += int((~split & (mode != 0)).sum())
        seen["split8"] += int(((tu & 15) != 0).sum())
        seen["ts"] += int(((tsy != 0) | (tsc != 0)).sum())
        if t:
            seen["inter_split"] += int((split & (mode != 3)).sum())
    assert all(v > 0 for v in seen.values()), seen
    enc.close()


@pytest.mark.parametrize("kind", ["desktop", "motion", "noise"])
def test_hevc_split_intra_slices(kind, monkeypatch):
    """Intra slices cut every CTB row into slices (hevc_core.h SliceMap; 20 CTBs of 32x32 at
    full size, 2 here via SK_HEVC_SEG_CTBS so a 320-wide picture splits 5 ways): mid-row
    slice starts under entropy_coding_sync, no top neighbours, no deblocking or SAO
    across the cuts. The independent decoder returns the encoder's reconstruction
    bit-exactly for key frames and the P frames predicted from them, and the serial and
    chunk-parallel CABAC models agree on the split layout."""
    monkeypatch.setenv("SK_HEVC_SEG_CTBS", "2")
    W, H = 320, 192
    res = _run(W, H, kind, 5, qp=27)
    key = res[0][0].data[10:]
    types = [(n[0] >> 1) & 63 for n in split_annexb(key)]
    assert types[:3] == [32, 33, 34] and types[3:] == [19] * (6 * 5)   # 6 CTB rows x 5 segments
    assert all(q > 30 for _, _, q in res)
    src = SyntheticDesktop(W, H, kind=kind)
    ref = HevcEncoder(W, H, backend="cpu", qp=27)
    monkeypatch.setenv("SK_HEVC_PCABAC", "1")
    par = HevcEncoder(W, H, backend="cpu", qp=27)
    for t in range(2):
        f = src.frame(t)
        assert [p.data for p in ref.encode(f, t)] == [p.data for p in par.encode(f, t)]


def _structure(enc):
    c = np.frombuffer(enc.debug_buffer("cus", np.uint8), np.uint8).reshape(-1, CUINFO)
    c32, cu8 = c[:, 22], c[:, 21]
    return {"cu32": int((c32 & 1).sum()) // 4, "tu32": int(((c32 & 9) == 9).sum()) // 4,
            "2NxN": int(((c32 & 1) & (((c32 >> 1) & 3) == 1)).sum()) // 4,
            "Nx2N": int(((c32 & 1) & (((c32 >> 1) & 3) == 2)).sum()) // 4,
            "cu8": int(((cu8 >> 4) & 1).sum()), "nxn": int(sum(bin(int(v) & 15).count("1") for v in cu8 if v & 16))}


@pytest.mark.parametrize("W,H,kind,qp", [(256, 144, "motion", 27), (200, 100, "desktop", 32), (336, 208, "motion", 22)])
def test_hevc_coding_quadtree(W, H, kind, qp):
    """CTB 32 coding quadtree (hevc_core.h): key frames use intra CU16s and CU8s with
    PART_NxN (four 4x4 PUs, own modes and MPM lists), P frames 32x32 CUs with PART_2Nx2N /
    2NxN / Nx2N over the unit motion field, under a 32x32 TU or a split root; picture sizes
    with odd unit counts leave partial CTBs (split_cu_flag inferred). The independent
    decoder returns the encoder's reconstruction (all planes) for every picture."""
    src = SyntheticDesktop(W, H, kind=kind)
    enc = HevcEncoder(W, H, backend="cpu", qp=qp, paint_qp=qp, use_paint_over=False, rate_control="cqp")
    dec = HevcDecoder()
    seen = {}
    cw, pcw = (W + 1) // 2, (W + 15) // 16 * 8
    for t in range(5):
        pk = enc.encode(src.frame(t), t)[0]
        Y, U, V = dec.decode(pk.data[10:])[0]
        assert np.array_equal(Y, _rec_y(enc, W, H)), f"frame {t}"
        for name, P in (("ref_u", U), ("ref_v", V)):
            rec = np.frombuffer(enc.debug_buffer(name, np.uint8), np.uint8).reshape(-1, pcw)[:(H + 1) // 2, :cw]
            assert np.array_equal(P, rec), (name, t)
        for k, v in _structure(enc).items():
            seen[k] = seen.get(k, 0) + v
    for k in ("cu32", "tu32", "cu8", "nxn"):
        assert seen[k] > 0, seen
    assert seen["2NxN"] + seen["Nx2N"] > 0, seen

