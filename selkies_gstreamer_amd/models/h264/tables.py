"""H.264 CAVLC tables for the Python verification decoder.

Single source of truth: the tables are parsed from the native header
``csrc/codec/h264_tables.h`` (the encoder's tables), so a typo cannot hide in a
second copy. Their structural validity (prefix-free, Kraft sums) is asserted in
``tests/test_h264_tables.py``.
"""
from __future__ import annotations

import re
from functools import lru_cache
from pathlib import Path

HEADER = Path(__file__).resolve().parents[3] / "csrc" / "codec" / "h264_tables.h"


@lru_cache(maxsize=1)
def _source() -> str:
    return HEADER.read_text()


def table(name: str):
    """Returns the table `name` as a (nested) list of ints."""
    m = re.search(re.escape(name) + r"\s*(\[[^=]*\])\s*=\s*\{(.*?)\};", _source(), re.S)
    if not m:
        raise KeyError(name)
    body = m.group(2)
    rows = re.findall(r"\{([^{}]*)\}", body)
    nums = lambda s: [int(x) for x in re.findall(r"-?\d+", s)]  # noqa: E731
    if rows:
        return [nums(r) for r in rows]
    return nums(body)


def vlc_codes(lens, codes):
    """[(length, code, index)] for entries with length > 0."""
    return [(l, c, i) for i, (l, c) in enumerate(zip(lens, codes)) if l > 0]


@lru_cache(maxsize=None)
def coeff_token_map(vlc: int):
    """dict (length, code) -> (TotalCoeff, TrailingOnes). vlc 0..3, or -1 for chroma DC."""
    if vlc == -1:
        lens, codes = table("H264_CDC_COEFF_TOKEN_LEN"), table("H264_CDC_COEFF_TOKEN_CODE")
    else:
        lens, codes = table("H264_COEFF_TOKEN_LEN")[vlc], table("H264_COEFF_TOKEN_CODE")[vlc]
    out = {}
    for l, c, i in vlc_codes(lens, codes):
        if i == 0:
            out[(l, c)] = (0, 0)
        else:
            tc, t1 = divmod(i, 4)
            out[(l, c)] = (tc, t1)
    return out


@lru_cache(maxsize=None)
def total_zeros_map(total_coeff: int, chroma_dc: bool):
    if chroma_dc:
        lens = table("H264_CDC_TOTAL_ZEROS_LEN")[total_coeff - 1][: 4 - total_coeff + 1]
        codes = table("H264_CDC_TOTAL_ZEROS_CODE")[total_coeff - 1][: 4 - total_coeff + 1]
    else:
        lens = table("H264_TOTAL_ZEROS_LEN")[total_coeff - 1]
        codes = table("H264_TOTAL_ZEROS_CODE")[total_coeff - 1]
    return {(l, c): i for i, (l, c) in enumerate(zip(lens, codes))}


@lru_cache(maxsize=None)
def run_before_map(zeros_left: int):
    t = min(zeros_left, 7) - 1
    lens = table("H264_RUN_BEFORE_LEN")[t]
    codes = table("H264_RUN_BEFORE_CODE")[t]
    return {(l, c): i for i, (l, c) in enumerate(zip(lens, codes))}


ZIGZAG = table("H264_ZIGZAG4x4")
BLK_X = table("H264_BLK_X")
BLK_Y = table("H264_BLK_Y")
DEQUANT_V = table("H264_DEQUANT_V")
POS_CLASS = table("H264_POS_CLASS")
CHROMA_QP = table("H264_CHROMA_QP")
CBP_TO_CODE_INTRA = table("H264_CBP_TO_CODE_INTRA")
CBP_TO_CODE_INTER = table("H264_CBP_TO_CODE_INTER")
CODE_TO_CBP_INTRA = [CBP_TO_CODE_INTRA.index(c) for c in range(48)]
CODE_TO_CBP_INTER = [CBP_TO_CODE_INTER.index(c) for c in range(48)]
