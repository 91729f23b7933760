"""HEVC on the MI355X: the HIP back end must be byte-identical to the CPU reference
(codec/hevc_cpu.cpp) — CU decisions, levels and packets — and its stream must decode
with the independent test decoder (models/hevc/decoder.py) to the encoder's
reconstruction."""
import numpy as np
import pytest

from selkies_gstreamer_amd.models.hevc.decoder import HevcDecoder
from selkies_gstreamer_amd.ops.native import HevcEncoder, hip_device_count
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _need_gpu():
    if hip_device_count() < 1:
        pytest.skip("no HIP device")


def _pair(W, H, **kw):
    return HevcEncoder(W, H, backend="hip", device=0, **kw), HevcEncoder(W, H, backend="cpu", **kw)


@pytest.mark.parametrize("W,H,kind,frames", [(128, 64, "motion", 5), (256, 144, "desktop", 4),
                                             (200, 100, "noise", 3), (320, 192, "motion", 18)])
def test_hevc_hip_matches_cpu(W, H, kind, frames):
    gpu, cpu = _pair(W, H)
    src = SyntheticDesktop(W, H, kind=kind)
    dec = HevcDecoder()
    pw = (W + 15) // 16 * 16
    for t in range(frames):
        f = src.frame(t)
        pg, pc = gpu.encode(f, t), cpu.encode(f, t)
        cg = np.frombuffer(gpu.debug_buffer("cus", np.uint8), np.uint8)
        cc = np.frombuffer(cpu.debug_buffer("cus", np.uint8), np.uint8)
        assert np.array_equal(cg, cc), f"frame {t}: CU decisions differ"
        lg = np.frombuffer(gpu.debug_buffer("coefs", np.uint8), np.int16)
        lc = np.frombuffer(cpu.debug_buffer("coefs", np.uint8), np.int16)
        assert np.array_equal(lg, lc), f"frame {t}: levels differ"
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}: packets differ"
        Y = dec.decode(pg[0].data[10:])[0][0]
        rec = np.frombuffer(gpu.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, pw)[:H, :W]
        assert np.array_equal(Y, rec)
    gpu.close()
    cpu.close()


def test_hevc_hip_keyframe_and_qp():
    W, H = 192, 128
    gpu, cpu = _pair(W, H)
    src = SyntheticDesktop(W, H, kind="motion")
    for t in range(6):
        if t == 3:
            gpu.request_keyframe()
            cpu.request_keyframe()
        if t == 4:
            gpu.set_qp(34)
            cpu.set_qp(34)
        f = src.frame(t)
        pg, pc = gpu.encode(f, t), cpu.encode(f, t)
        assert [p.data for p in pg] == [p.data for p in pc], t
        assert pg[0].key == (t in (0, 3))
    gpu.close()
    cpu.close()


def test_hevc_hip_1080p_parity():
    W, H = 1920, 1080
    gpu, cpu = _pair(W, H)
    src = SyntheticDesktop(W, H, kind="motion")
    for t in range(4):
        f = src.frame(t)
        pg, pc = gpu.encode(f, t), cpu.encode(f, t)
        assert [p.data for p in pg] == [p.data for p in pc], t
    gpu.close()
    cpu.close()


@pytest.mark.parametrize("kind,seg", [("motion", "4"), ("noise", "3"), ("desktop", "7")])
def test_hevc_hip_split_intra_slices(kind, seg, monkeypatch):
    """Split intra slices (hevc_core.h SliceMap) on the GPU: k_hevc_intra_seg (one wave
    per row segment), per-segment substreams through the chunk-parallel CABAC, one slice
    NAL per segment from k_hevc_hdr - byte-identical to the CPU, key frames on request
    included, and decoded to the encoder's reconstruction."""
    monkeypatch.setenv("SK_HEVC_SEG_CTBS", seg)
    W, H = 336, 208   # 21 x 13 units = 11 x 7 CTBs: partial CTBs, uneven segments, a partial last slice
    gpu, cpu = _pair(W, H, qp=27)
    src = SyntheticDesktop(W, H, kind=kind)
    dec = HevcDecoder()
    pw = (W + 15) // 16 * 16
    for t in range(6):
        if t == 3:
            gpu.request_keyframe()
            cpu.request_keyframe()
        f = src.frame(t)
        pg, pc = gpu.encode(f, t), cpu.encode(f, t)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}"
        Y = dec.decode(pg[0].data[10:])[0][0]
        rec = np.frombuffer(gpu.debug_buffer("ref_y", np.uint8), np.uint8).reshape(-1, pw)[:H, :W]
        assert np.array_equal(Y, rec), f"frame {t}"
    gpu.close()
    cpu.close()


def test_hevc_hip_4k_keyframe_parity():
    """3840x2160 key frames (12 segments per CTB row, 816 slices) and the P frames after
    them: GPU == CPU."""
    W, H = 3840, 2160
    gpu, cpu = _pair(W, H)
    src = SyntheticDesktop(W, H, kind="desktop")
    for t in range(3):
        f = src.frame(t)
        pg, pc = gpu.encode(f, t), cpu.encode(f, t)
        assert [p.data for p in pg] == [p.data for p in pc], t
    gpu.close()
    cpu.close()
