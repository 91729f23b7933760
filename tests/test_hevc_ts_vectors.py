"""Transform-skip residuals of the test HEVC decoder (models/hevc/decoder.py
residual_from_levels) against values worked out by hand from the spec text, not
from this repo's encoder: 8.6.3 scaling (m = 16, levelScale = {40, 45, 51, 57, 64,
72}, bdShift = BitDepth + Log2(nTbS) - 5 = 5 for 8-bit 4x4) and 8.6.4.2 (transform
skip: r = d << 7, then bdShift = 20 - BitDepth = 12).

No independent HEVC decoder is importable on this image (no PyAV / libde265 /
ffmpeg), so whole-bitstream conformance of the residual quadtree and transform skip
stays parity-unpinned; these vectors pin the arithmetic the decoder applies."""
import numpy as np

from selkies_gstreamer_amd.models.hevc.decoder import residual_from_levels


def _one(level, qp, pos=(0, 0)):
    lv = np.zeros((4, 4), np.int64)
    lv[pos] = level
    return residual_from_levels(lv, qp, 2, True, False)


def test_transform_skip_hand_vectors():
    # level 1, qP 4: 1 * 16 * 64 = 1024; (1024 + 16) >> 5 = 32; (32 * 128 + 2048) >> 12 = 1
    assert _one(1, 4)[0, 0] == 1
    # level -3, qP 30: levelScale[0] = 40, << 5: -3 * 16 * 40 * 32 = -61440;
    # (-61440 + 16) >> 5 = -1920; (-1920 * 128 + 2048) >> 12 = floor(-59.5) = -60
    assert _one(-3, 30)[0, 0] == -60
    # level 7, qP 22 at (2, 3): levelScale[4] = 64, << 3: 7 * 16 * 64 * 8 = 57344;
    # (57344 + 16) >> 5 = 1792; (1792 * 128 + 2048) >> 12 = 56.5 -> 56
    r = _one(7, 22, (2, 3))
    assert r[2, 3] == 56 and np.count_nonzero(r) == 1   # no spreading: the sample stays put
    # clipping of d to 16 bits: level 2000, qP 51 -> d = 32767 -> (32767 * 128 + 2048) >> 12 = 1024
    assert _one(2000, 51)[0, 0] == 1024


def test_dct_path_differs_from_transform_skip():
    lv = np.zeros((4, 4), np.int64)
    lv[0, 0] = 10
    dct = residual_from_levels(lv, 22, 2, False, False)
    assert np.count_nonzero(dct) == 16 and len(set(dct.ravel().tolist())) == 1   # a DC-only block is flat
