"""AV1 encoder (codec/av1_cpu.cpp) against an independent, conformant decoder:
dav1d 1.5 (the decoder in Chrome / Firefox), reached through Pillow's bundled
libavif (models/av1/dav1d.py). Every decoded frame must equal the encoder's own
reconstruction bit for bit (Y, U and V) — that pins the default CDF tables, the
syntax, the inverse transforms, intra / inter prediction and the MV stack — and
stay close to the source (PSNR)."""
import numpy as np
import pytest

from selkies_gstreamer_amd.models.av1 import dav1d
from selkies_gstreamer_amd.ops.native import Av1Encoder
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop

pytestmark = pytest.mark.skipif(not dav1d.available(), reason="dav1d (Pillow libavif) not available")


def planes(enc, W, H):
    sy = (W + 15) // 16 * 16
    sc = sy // 2
    ry = enc.debug_buffer("ref_y").reshape(-1, sy)[:H, :W]
    ru = enc.debug_buffer("ref_u").reshape(-1, sc)[:(H + 1) // 2, :(W + 1) // 2]
    rv = enc.debug_buffer("ref_v").reshape(-1, sc)[:(H + 1) // 2, :(W + 1) // 2]
    src = enc.debug_buffer("src_y").reshape(-1, sy)[:H, :W]
    return ry, ru, rv, src


def psnr(a, b):
    mse = np.mean((a.astype(np.float64) - b) ** 2)
    return 99.0 if mse == 0 else 10 * np.log10(255.0 ** 2 / mse)


def run(W, H, kind, frames, backend="cpu", **kw):
    enc = Av1Encoder(W, H, backend=backend, **kw)
    src = SyntheticDesktop(W, H, kind=kind)
    dec = dav1d.Decoder()
    out = []
    for t in range(frames):
        pk = enc.encode(src.frame(t), t)
        assert len(pk) == 1 and pk[0].data[0] == 0x04
        tu = pk[0].data[10:]
        assert tu[:2] == b"\x12\x00"          # temporal delimiter OBU
        pic = dec.decode(tu)
        assert pic is not None, f"frame {t}: dav1d produced no picture"
        ry, ru, rv, s = planes(enc, W, H)
        for name, a, b in zip("YUV", pic, (ry, ru, rv)):
            bad = np.argwhere(a != b)
            assert len(bad) == 0, f"frame {t} plane {name}: {len(bad)} samples differ, first {bad[:3].tolist()}"
        out.append((bool(pk[0].key), len(tu), psnr(pic[0], s)))
    dec.close()
    return out


@pytest.mark.parametrize("W,H", [(64, 64), (256, 128), (200, 120), (640, 360)])
def test_key_and_inter_frames_decode_exactly(W, H):
    res = run(W, H, "motion", 4, qp=25)
    assert res[0][0] and not any(k for k, _, _ in res[1:])
    assert min(p for _, _, p in res) > 30


def test_auto_tiles_from_3072_px_decode_exactly():
    """Frames 48+ superblocks wide take 16 tile columns (av1_core.h auto_tiles: the 4K key
    frame's per-tile wavefront fits 16 waves); dav1d decodes them exactly."""
    res = run(3072, 192, "motion", 2, qp=30)
    assert res[0][0] and min(p for _, _, p in res) > 30


def test_noise_cuts_stay_inter_frames():
    """No scene-cut key frames (svtav1enc in the reference runs intra-period -1 with
    no scene-change detection, legacy/gstwebrtc_app.py:733-739): a frame of new noise
    is an inter frame, still decoded bit-exactly by dav1d."""
    res = run(192, 128, "noise", 3, qp=30)
    assert res[0][0] and not any(k for k, _, _ in res[1:])


@pytest.mark.parametrize("tc,tr", [(0, 0), (2, 1), (1, 2), (3, 3)])
def test_tile_layouts(tc, tr):
    res = run(512, 320, "motion", 3, qp=28, tile_cols_log2=tc, tile_rows_log2=tr)
    assert len(res) == 3


@pytest.mark.parametrize("qp", [10, 22, 40, 51])
def test_quantisers(qp):
    res = run(128, 96, "motion", 3, qp=qp)
    if qp <= 22:
        assert res[0][2] > 38


def test_static_content_collapses_to_skip_superblocks():
    """A desktop that does not change codes every inter frame as 64x64 GLOBALMV skips."""
    W, H = 256, 192
    enc = Av1Encoder(W, H, backend="cpu", qp=25)
    frame = SyntheticDesktop(W, H, kind="motion").frame(0)
    dec = dav1d.Decoder()
    sizes = []
    for t in range(4):
        pk = enc.encode(frame, t)
        pic = dec.decode(pk[0].data[10:])
        ry, _, _, _ = planes(enc, W, H)
        assert (pic[0] == ry).all()
        sizes.append(len(pk[0].data) - 10)
    blk = enc.debug_buffer("blk").reshape(-1, 12)
    assert set(blk[:, 0].tolist()) == {4}            # every cell in a 64x64 block (after two refining frames)
    assert sizes[3] < 64                              # a handful of bytes per frame


def test_1080p_frames():
    res = run(1920, 1080, "motion", 2, qp=25)
    assert res[0][2] > 34 and res[1][1] < res[0][1] / 4


@pytest.mark.parametrize("mtu", [1200, 300])
def test_av1_rtp_roundtrip(mtu):
    """rtc_av1_packetize (csrc/rtc/rtc.cpp, AV1 RTP payload format) -> AV1Depacketizer
    (webrtc/rtp.py) rebuilds every temporal unit byte for byte; fragments at a small
    MTU; N only on the key frame's first packet; marker on the last packet."""
    from selkies_gstreamer_amd.webrtc import rtp
    from selkies_gstreamer_amd.webrtc.native import RtpPacketizer
    W, H = 320, 192
    src = SyntheticDesktop(W, H, kind="motion")
    enc = Av1Encoder(W, H, backend="cpu")
    pk = RtpPacketizer(ssrc=1234, payload_type=96, mtu=mtu)
    dep = rtp.AV1Depacketizer()
    for t in range(4):
        (p,) = enc.encode(src.frame(t), t)
        tu = p.data[10:]
        pkts = pk.av1(tu, 3000 * t)
        assert pkts and all(len(x) <= mtu for x in pkts)
        hdrs = [rtp.parse_rtp(x) for x in pkts]
        assert [h.marker for h in hdrs] == [False] * (len(pkts) - 1) + [True]
        aggs = [x[h.header_len] for x, h in zip(pkts, hdrs)]
        assert bool(aggs[0] & 0x08) == p.key and not any(a & 0x08 for a in aggs[1:])
        out = None
        for x, h in zip(pkts, hdrs):
            out = dep.push(x[h.header_len:], h.timestamp, h.marker)
        assert out == tu


def test_av1_depacketizer_malformed_and_sized_obus():
    """Truncated / oversized elements are dropped without raising; an OBU the sender
    kept obu_has_size_field on passes through unchanged (no second size field)."""
    from selkies_gstreamer_amd.webrtc import rtp
    dep = rtp.AV1Depacketizer()
    assert dep.push(bytes([0x00, 0x85]), 1, True) is None          # leb128 cut short
    assert dep.push(bytes([0x00, 0x05, 0x30, 0x01]), 2, True) is None  # element longer than the packet
    sized = bytes([0x32, 0x02, 0xAA, 0xBB])                        # OBU_FRAME with has_size + size 2
    out = dep.push(bytes([0x10]) + sized, 3, True)                  # W=1: one element, no length
    assert out == b"\x12\x00" + sized
    bare = bytes([0x30, 0xAA, 0xBB])                               # no size field: one is added
    assert dep.push(bytes([0x10]) + bare, 4, True) == b"\x12\x00" + bytes([0x32, 0x02, 0xAA, 0xBB])


def test_idtx_blocks_on_text_decode_exactly():
    """IDTX (identity transform) is chosen by RD cost where it pays - dense synthetic
    text - in key and inter frames, and dav1d reconstructs every such block exactly."""
    W, H = 320, 192
    enc = Av1Encoder(W, H, backend="cpu", qp=30)
    src = SyntheticDesktop(W, H, kind="desktop")
    dec = dav1d.Decoder()
    idtx = []
    for t in range(3):
        pk = enc.encode(src.frame(t), t)
        pic = dec.decode(pk[0].data[10:])
        ry, ru, rv, _ = planes(enc, W, H)
        assert all(np.array_equal(a, b) for a, b in zip(pic, (ry, ru, rv)))
        blk = enc.debug_buffer("blk").view(np.int16).reshape(-1, 6)
        idtx.append(int((blk[:, 4] == 1).sum()))
    dec.close()
    assert idtx[0] > 0, idtx   # key frame


def test_palette_key_frames_decode_exactly_and_save_bytes(monkeypatch):
    """Screen content tools on key frames (allow_screen_content_tools, luma palettes of
    2..8 colours; av1_core.h code_palette_mode_info / code_palette_tokens): blocks of
    text and flat UI become exact palettes. dav1d decodes them to the encoder's
    reconstruction, and the key frame is smaller and closer to the source than the
    same encoder with palettes off (SK_AV1_PALETTE=0)."""
    W, H = 640, 360
    enc = Av1Encoder(W, H, backend="cpu", qp=22)
    enc.encode(SyntheticDesktop(W, H, kind="desktop").frame(0), 0)
    blk = enc.debug_buffer("blk").reshape(-1, 12)
    pal_n = blk[:, 10]
    assert (pal_n > 0).sum() > 50 and pal_n.max() <= 8 and pal_n[pal_n > 0].min() >= 2
    on = run(W, H, "desktop", 3, qp=22)
    monkeypatch.setenv("SK_AV1_PALETTE", "0")
    off = run(W, H, "desktop", 3, qp=22)
    assert on[0][1] < 0.85 * off[0][1] and on[0][2] > off[0][2] + 5
