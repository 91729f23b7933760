"""Spatial (band) parallelism of one session across devices (parallel/banded.py).

Stripes are independent streams, so a banded encoder must produce exactly the
packets a single encoder of the whole frame produces, with the stripe y rebased.
CPU backend here; the HIP variant (two bands on one GPU, the same code path a
multi-GPU node takes with distinct devices) is marked gpu.
"""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder
from selkies_gstreamer_amd.parallel.banded import BandedH264Encoder, split_bands
from tests.h264_util import synthetic_frames


def test_split_bands_whole_stripes():
    assert split_bands(1080, 64, 1) == [(0, 1080)]
    b = split_bands(1080, 64, 4)
    assert b[0][0] == 0 and b[-1][1] == 1080
    assert all(y0 % 64 == 0 for y0, _ in b)
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    sizes = [(y1 - y0 + 63) // 64 for y0, y1 in b]
    assert max(sizes) - min(sizes) <= 1 and sum(sizes) == 17
    assert len(split_bands(100, 64, 8)) == 2        # never more bands than stripes


def _compare(backend, devices, W=160, H=200, sh=32, n=5, **kw):
    single = H264Encoder(W, H, stripe_height=sh, backend=backend, qp=27, **kw)
    banded = BandedH264Encoder(W, H, devices, stripe_height=sh, backend=backend, qp=27, **kw)
    try:
        for t, f in enumerate(synthetic_frames(W, H, n, seed=4)):
            a = sorted((p.y, p.data) for p in single.encode(f, t))
            b = sorted((p.y, p.data) for p in banded.encode(f, t))
            assert a == b, f"frame {t}"
            if t == 2:
                single.request_keyframe()
                banded.request_keyframe()
    finally:
        banded.close()


@pytest.mark.parametrize("parts", [2, 3])
def test_banded_matches_single_encoder_cpu(parts):
    _compare("cpu", [0] * parts)


def test_banded_rejects_fullframe():
    with pytest.raises(ValueError):
        BandedH264Encoder(64, 64, [0, 0], backend="cpu", fullframe=True)


@pytest.mark.gpu
def test_banded_matches_single_encoder_hip():
    _compare("hip", [0, 0], W=640, H=360, sh=64, n=4)
