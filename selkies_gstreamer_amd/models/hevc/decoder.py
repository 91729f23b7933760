"""H.265 / HEVC Main decoder used to verify the encoder (test oracle).

There is no ffmpeg/PyAV/libde265 in the build environment, so the
HIP HEVC encoder is checked against this independent implementation of the decoding
process of ITU-T H.265: clause 7 (VPS/SPS/PPS/slice segment header syntax), 9.3
(CABAC parsing: context initialisation, WPP storage/synchronisation, arithmetic
decoding, binarisations and context selection) and 8 (intra sample prediction with
reference substitution and filtering, merge / AMVP motion vector prediction, 8-tap
luma and 4-tap chroma interpolation, scaling, inverse DCT/DST, reconstruction).

Supported: Main 8-bit 4:2:0, any CTB/CB/TB sizes with quadtree splits, intra
PART_2Nx2N / PART_NxN CUs and inter PART_2Nx2N / 2NxN / Nx2N CUs, I and P slices with one
reference list, multiple slices, entropy_coding_sync (WPP) substreams, transform skip.
NotImplementedError for the rest (B slices, tiles, AMP and inter NxN partitions, PCM,
scaling lists, TMVP, long-term references, sign data hiding, cu_qp_delta). The
deblocking filter (8.7.2) runs on the completed picture: transform and prediction block
edges on the 8x8 grid, boundary strength (the coefficient rule on transform edges only),
luma decisions and strong / normal filters, chroma on bS 2. Sample adaptive
offset (7.3.8.3 syntax, 8.7.3 band / edge offsets with the picture and slice boundary
rules) then runs on the deblocked picture.

Written from the specification text, not from the encoder's tables; numpy for the
sample processes, plain Python for parsing. Intended for test-sized pictures.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from ..h264.decoder import split_annexb, unescape


class BitstreamError(ValueError):
    pass


# ---------------------------------------------------------------------------
class Bits:
    def __init__(self, data: bytes, pos: int = 0):
        self.d = data
        self.p = pos   # bit position

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            byte = self.d[self.p >> 3] if (self.p >> 3) < len(self.d) else 0
            v = (v << 1) | ((byte >> (7 - (self.p & 7))) & 1)
            self.p += 1
        return v

    def ue(self) -> int:
        z = 0
        while self.u(1) == 0:
            z += 1
            if z > 32:
                raise BitstreamError("bad ue(v)")
        return (1 << z) - 1 + self.u(z)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)


# ---------------------------------------------------------------------------
# CABAC tables (9.3.4.3.2): rangeTabLps and transIdxLps.
RANGE_LPS = [
    (128, 176, 208, 240), (128, 167, 197, 227), (128, 158, 187, 216), (123, 150, 178, 205),
    (116, 142, 169, 195), (111, 135, 160, 185), (105, 128, 152, 175), (100, 122, 144, 166),
    (95, 116, 137, 158), (90, 110, 130, 150), (85, 104, 123, 142), (81, 99, 117, 135),
    (77, 94, 111, 128), (73, 89, 105, 122), (69, 85, 100, 116), (66, 80, 95, 110),
    (62, 76, 90, 104), (59, 72, 86, 99), (56, 69, 81, 94), (53, 65, 77, 89),
    (51, 62, 73, 85), (48, 59, 69, 80), (46, 56, 66, 76), (43, 53, 63, 72),
    (41, 50, 59, 69), (39, 48, 56, 65), (37, 45, 54, 62), (35, 43, 51, 59),
    (33, 41, 48, 56), (32, 39, 46, 53), (30, 37, 43, 50), (29, 35, 41, 48),
    (27, 33, 39, 45), (26, 31, 37, 43), (24, 30, 35, 41), (23, 28, 33, 39),
    (22, 27, 32, 37), (21, 26, 30, 35), (20, 24, 29, 33), (19, 23, 27, 31),
    (18, 22, 26, 30), (17, 21, 25, 28), (16, 20, 23, 27), (15, 19, 22, 25),
    (14, 18, 21, 24), (14, 17, 20, 23), (13, 16, 19, 22), (12, 15, 18, 21),
    (12, 14, 17, 20), (11, 14, 16, 19), (11, 13, 15, 18), (10, 12, 15, 17),
    (10, 12, 14, 16), (9, 11, 13, 15), (9, 11, 12, 14), (8, 10, 12, 14),
    (8, 9, 11, 13), (7, 9, 11, 12), (7, 9, 10, 12), (7, 8, 10, 11),
    (6, 8, 9, 11), (6, 7, 9, 10), (6, 7, 8, 9), (2, 2, 2, 2)]
TRANS_LPS = [0, 0, 1, 2, 2, 4, 4, 5, 6, 7, 8, 9, 9, 11, 11, 12, 13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21,
             22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33, 33, 33, 34, 34, 35,
             35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63]

# initValue per syntax element, indexed [initType][ctxIdx-within-element] (Tables 9-5..9-37).
INIT = {
    "split_cu_flag": [[139, 141, 157], [107, 139, 126], [107, 139, 126]],
    "cu_skip_flag": [[154, 154, 154], [197, 185, 201], [197, 185, 201]],
    "pred_mode_flag": [[154], [149], [134]],
    "part_mode": [[184, 154, 154, 154], [154, 139, 154, 154], [154, 139, 154, 154]],
    "prev_intra_luma_pred_flag": [[184], [154], [183]],
    "intra_chroma_pred_mode": [[63], [152], [152]],
    "rqt_root_cbf": [[154], [79], [79]],
    "merge_flag": [[154], [110], [154]],
    "merge_idx": [[154], [122], [137]],
    "inter_pred_idc": [[154] * 5, [95, 79, 63, 31, 31], [95, 79, 63, 31, 31]],
    "ref_idx": [[154, 154], [153, 153], [153, 153]],
    "mvp_flag": [[154], [168], [168]],
    "split_transform_flag": [[153, 138, 138], [124, 138, 94], [224, 167, 122]],
    "cbf_luma": [[111, 141], [153, 111], [153, 111]],
    "cbf_chroma": [[94, 138, 182, 154], [149, 107, 167, 154], [149, 92, 167, 154]],
    "abs_mvd_greater0_flag": [[154], [140], [169]],
    "abs_mvd_greater1_flag": [[154], [198], [198]],
    "cu_qp_delta_abs": [[154, 154], [154, 154], [154, 154]],
    "transform_skip_flag": [[139, 139], [139, 139], [139, 139]],
    "last_x_prefix": [
        [110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63],
        [125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108],
        [125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93]],
    "coded_sub_block_flag": [[91, 171, 134, 141], [121, 140, 61, 154], [121, 140, 61, 154]],
    "sig_coeff_flag": [
        [111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153,
         125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139, 111, 136,
         139, 111],
        [155, 154, 139, 153, 139, 123, 123, 63, 153, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153,
         154, 166, 183, 140, 136, 153, 154, 170, 153, 138, 138, 122, 121, 122, 121, 167, 151, 183, 140, 151,
         183, 140],
        [170, 154, 139, 153, 139, 123, 123, 63, 124, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153,
         154, 166, 183, 140, 136, 153, 154, 170, 153, 123, 123, 107, 121, 107, 121, 167, 151, 183, 140, 151,
         183, 140]],
    "coeff_abs_level_greater1_flag": [
        [140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166, 182, 140,
         227, 122, 197],
        [154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137, 169, 194, 166, 167,
         154, 167, 137, 182],
        [154, 196, 167, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 122, 169, 208, 166, 167,
         154, 152, 167, 182]],
    "coeff_abs_level_greater2_flag": [[138, 153, 136, 167, 152, 152], [107, 167, 91, 122, 107, 167],
                                      [107, 167, 91, 107, 107, 167]],
}
INIT["last_y_prefix"] = INIT["last_x_prefix"]
INIT["sao_merge_flag"] = [[153], [153], [153]]          # sao_merge_left_flag / sao_merge_up_flag
INIT["sao_type_idx"] = [[200], [185], [160]]            # sao_type_idx_luma / _chroma (first bin)


def init_contexts(init_type: int, qp: int) -> dict:
    ctx = {}
    q = min(max(qp, 0), 51)
    for name, tabs in INIT.items():
        states = []
        for iv in tabs[init_type]:
            m = (iv >> 4) * 5 - 45
            n = ((iv & 15) << 3) - 16
            pre = min(max(((m * q) >> 4) + n, 1), 126)
            mps = 1 if pre > 63 else 0
            states.append([pre - 64 if mps else 63 - pre, mps])
        ctx[name] = states
    return ctx


def copy_contexts(ctx: dict) -> dict:
    return {k: [list(s) for s in v] for k, v in ctx.items()}


class Cabac:
    """Arithmetic decoding engine (9.3.4.3) over one substream (RBSP bytes)."""

    def __init__(self, data: bytes):
        self.b = Bits(data)
        self.range = 510
        self.offset = self.b.u(9)

    def decision(self, st: list) -> int:
        p, mps = st
        lps = RANGE_LPS[p][(self.range >> 6) & 3]
        self.range -= lps
        if self.offset >= self.range:
            binv = 1 - mps
            self.offset -= self.range
            self.range = lps
            if p == 0:
                st[1] = 1 - mps
            st[0] = TRANS_LPS[p]
        else:
            binv = mps
            st[0] = min(p + 1, 62)
        while self.range < 256:
            self.range <<= 1
            self.offset = (self.offset << 1) | self.b.u(1)
        return binv

    def bypass(self) -> int:
        self.offset = (self.offset << 1) | self.b.u(1)
        if self.offset >= self.range:
            self.offset -= self.range
            return 1
        return 0

    def bypass_bits(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.bypass()
        return v

    def terminate(self) -> int:
        self.range -= 2
        if self.offset >= self.range:
            return 1
        while self.range < 256:
            self.range <<= 1
            self.offset = (self.offset << 1) | self.b.u(1)
        return 0


# ---------------------------------------------------------------------------
# Transforms (8.6.4.2) and intra tables.
_C64 = [64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64, 61, 57, 54, 50, 46, 43, 38, 36,
        31, 25, 22, 18, 13, 9, 4, 0]


def _cosv(m: int) -> int:
    m %= 128
    if m <= 32:
        return _C64[m]
    if m < 64:
        return -_C64[64 - m]
    if m <= 96:
        return -_C64[m - 64]
    return _C64[128 - m]


def dct_matrix(n: int) -> np.ndarray:
    s = 32 // n
    t = np.zeros((n, n), dtype=np.int64)
    t[0, :] = 64
    for k in range(1, n):
        for j in range(n):
            t[k, j] = _cosv((2 * j + 1) * k * s)
    return t


_DCT = {n: dct_matrix(n) for n in (4, 8, 16, 32)}
_DST = np.array([[29, 55, 74, 84], [74, 74, 0, -74], [84, -29, -74, 55], [55, -84, 74, -29]], dtype=np.int64)

INTRA_ANGLE = [0, 0, 32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26, -32, -26, -21, -17, -13,
               -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32]
INV_ANGLE = {11: -4096, 12: -1638, 13: -910, 14: -630, 15: -482, 16: -390, 17: -315, 18: -256, 19: -315,
             20: -390, 21: -482, 22: -630, 23: -910, 24: -1638, 25: -4096}
LUMA_FILTER = [[0, 0, 0, 64, 0, 0, 0, 0], [-1, 4, -10, 58, 17, -5, 1, 0], [-1, 4, -11, 40, 40, -11, 4, -1],
               [0, 1, -5, 17, 58, -10, 4, -1]]
CHROMA_FILTER = [[0, 64, 0, 0], [-2, 58, 10, -2], [-4, 54, 16, -2], [-6, 46, 28, -4], [-4, 36, 36, -4],
                 [-4, 28, 46, -6], [-2, 16, 54, -4], [-2, 10, 58, -2]]
LEVEL_SCALE = [40, 45, 51, 57, 64, 72]
QPC_TABLE = {30: 29, 31: 30, 32: 31, 33: 32, 34: 33, 35: 33, 36: 34, 37: 34, 38: 35, 39: 35, 40: 36, 41: 36,
             42: 37, 43: 37}


def inverse_transform(d: np.ndarray, n: int, dst: bool) -> np.ndarray:
    """d[y][x] scaled coefficients -> residual (8-bit video)."""
    m = _DST if dst else _DCT[n]
    e = m.T @ d.astype(np.int64)                    # columns: e[y][x] = sum_j m[j][y] d[j][x]
    g = np.clip((e + 64) >> 7, -32768, 32767)
    r = g @ m                                       # rows: r[y][x] = sum_j g[y][j] m[j][x]
    return (r + 2048) >> 12


def residual_from_levels(levels: np.ndarray, qp: int, log2: int, ts: bool, dst: bool) -> np.ndarray:
    """TransCoeffLevel -> residual of one n x n TB, 8-bit video: scaling (8.6.3, flat
    m = 16, bdShift = BitDepth + log2 - 5), then transform skip (8.6.4.2: r = d << 7) or
    the inverse DCT / DST, and the final (r + 2^11) >> 12 (bdShift 20 - BitDepth)."""
    n = 1 << log2
    bd = 8 + log2 - 5
    scale = 16 * LEVEL_SCALE[qp % 6] << (qp // 6)
    d = np.clip((np.asarray(levels, np.int64) * scale + (1 << (bd - 1))) >> bd, -32768, 32767)
    if ts:
        return ((d << 7) + (1 << 11)) >> 12
    return inverse_transform(d, n, dst)


def scan_diag(n: int) -> list:
    out = []
    x = y = 0
    while len(out) < n * n:
        while y >= 0:
            if x < n and y < n:
                out.append((x, y))
            y -= 1
            x += 1
        y = x
        x = 0
    return out


def scan_order(n: int, scan_idx: int) -> list:
    if scan_idx == 0:
        return scan_diag(n)
    if scan_idx == 1:   # horizontal
        return [(x, y) for y in range(n) for x in range(n)]
    return [(x, y) for x in range(n) for y in range(n)]   # vertical


# ---------------------------------------------------------------------------
@dataclass
class Sps:
    width: int = 0
    height: int = 0
    crop: tuple = (0, 0, 0, 0)
    log2_min_cb: int = 3
    log2_ctb: int = 4
    log2_min_tb: int = 2
    log2_max_tb: int = 5
    max_th_inter: int = 0
    max_th_intra: int = 0
    log2_poc_lsb: int = 8
    num_st_rps: int = 0
    st_rps: list = None
    amp: bool = False
    sao: bool = False
    pcm: bool = False
    tmvp: bool = False
    strong_smoothing: bool = False
    scaling_list: bool = False
    long_term: bool = False


@dataclass
class Pps:
    dependent_slices: bool = False
    output_flag_present: bool = False
    extra_bits: int = 0
    sign_hiding: bool = False
    cabac_init_present: bool = False
    num_ref_l0: int = 1
    init_qp: int = 26
    constrained_intra: bool = False
    transform_skip: bool = False
    cu_qp_delta: bool = False
    cb_qp_offset: int = 0
    cr_qp_offset: int = 0
    slice_chroma_qp_offsets: bool = False
    tiles: bool = False
    wpp: bool = False
    loop_filter_across_slices: bool = False
    deblock_override: bool = False
    deblock_disabled: bool = False
    beta_offset: int = 0
    tc_offset: int = 0
    lists_modification: bool = False
    log2_par_mrg: int = 2
    slice_header_ext: bool = False


class HevcDecoder:
    def __init__(self):
        self.sps: Sps | None = None
        self.pps: Pps | None = None
        self.ref = None          # previous decoded picture (Y, U, V) for P slices
        self.poc = 0
        self.frames = []
        self.cur = None

    # ---------------- parameter sets ----------------
    @staticmethod
    def _ptl(b: Bits, max_sub_layers_minus1: int):
        b.u(2); b.u(1); b.u(5); b.u(32); b.u(4); b.u(32); b.u(12)
        b.u(8)   # general_level_idc
        if max_sub_layers_minus1 > 0:
            raise NotImplementedError("sub-layers")

    def _parse_sps(self, r: bytes):
        b = Bits(r)
        b.u(4)
        msl = b.u(3)
        b.u(1)
        self._ptl(b, msl)
        b.ue()
        if b.ue() != 1:
            raise NotImplementedError("only 4:2:0")
        s = Sps()
        s.width, s.height = b.ue(), b.ue()
        if b.u(1):
            s.crop = (b.ue(), b.ue(), b.ue(), b.ue())
        if b.ue() != 0 or b.ue() != 0:
            raise NotImplementedError("only 8-bit")
        s.log2_poc_lsb = b.ue() + 4
        sub = b.u(1)
        for _ in range(0 if sub else msl, msl + 1):
            b.ue(); b.ue(); b.ue()
        s.log2_min_cb = b.ue() + 3
        s.log2_ctb = s.log2_min_cb + b.ue()
        s.log2_min_tb = b.ue() + 2
        s.log2_max_tb = s.log2_min_tb + b.ue()
        s.max_th_inter = b.ue()
        s.max_th_intra = b.ue()
        s.scaling_list = bool(b.u(1))
        if s.scaling_list:
            raise NotImplementedError("scaling lists")
        s.amp = bool(b.u(1))
        s.sao = bool(b.u(1))
        s.pcm = bool(b.u(1))
        if s.pcm:
            raise NotImplementedError("PCM")
        s.num_st_rps = b.ue()
        s.st_rps = []
        for i in range(s.num_st_rps):
            s.st_rps.append(self._st_rps(b, i, s.st_rps))
        s.long_term = bool(b.u(1))
        if s.long_term:
            raise NotImplementedError("long-term refs")
        s.tmvp = bool(b.u(1))
        s.strong_smoothing = bool(b.u(1))
        self.sps = s

    @staticmethod
    def _st_rps(b: Bits, idx: int, prev: list) -> list:
        if idx != 0 and b.u(1):
            raise NotImplementedError("inter RPS prediction")
        nneg, npos = b.ue(), b.ue()
        deltas = []
        poc = 0
        for _ in range(nneg):
            poc -= b.ue() + 1
            deltas.append((poc, b.u(1)))
        poc = 0
        for _ in range(npos):
            poc += b.ue() + 1
            deltas.append((poc, b.u(1)))
        return deltas

    def _parse_pps(self, r: bytes):
        b = Bits(r)
        b.ue(); b.ue()
        p = Pps()
        p.dependent_slices = bool(b.u(1))
        p.output_flag_present = bool(b.u(1))
        p.extra_bits = b.u(3)
        p.sign_hiding = bool(b.u(1))
        p.cabac_init_present = bool(b.u(1))
        p.num_ref_l0 = b.ue() + 1
        b.ue()
        p.init_qp = 26 + b.se()
        p.constrained_intra = bool(b.u(1))
        p.transform_skip = bool(b.u(1))
        p.cu_qp_delta = bool(b.u(1))
        if p.cu_qp_delta:
            raise NotImplementedError("cu_qp_delta")
        p.cb_qp_offset, p.cr_qp_offset = b.se(), b.se()
        p.slice_chroma_qp_offsets = bool(b.u(1))
        if b.u(1) or b.u(1):
            raise NotImplementedError("weighted prediction")
        if b.u(1):
            raise NotImplementedError("transquant bypass")
        p.tiles = bool(b.u(1))
        if p.tiles:
            raise NotImplementedError("tiles")
        p.wpp = bool(b.u(1))
        p.loop_filter_across_slices = bool(b.u(1))
        if b.u(1):
            p.deblock_override = bool(b.u(1))
            p.deblock_disabled = bool(b.u(1))
            if not p.deblock_disabled:
                p.beta_offset, p.tc_offset = 2 * b.se(), 2 * b.se()
        if b.u(1):
            raise NotImplementedError("PPS scaling lists")
        p.lists_modification = bool(b.u(1))
        p.log2_par_mrg = b.ue() + 2
        p.slice_header_ext = bool(b.u(1))
        if p.sign_hiding:
            raise NotImplementedError("sign data hiding")
        self.pps = p

    # ---------------- pictures ----------------
    def decode(self, annexb: bytes) -> list:
        """Decodes an Annex-B stream; returns the pictures completed by it as (Y, U, V)
        arrays cropped to the conformance window."""
        out = []
        for nal in split_annexb(annexb):
            if len(nal) < 2:
                continue
            t = (nal[0] >> 1) & 63
            if t == 32:
                continue
            if t == 33:
                self._parse_sps(unescape(nal[2:]))
            elif t == 34:
                self._parse_pps(unescape(nal[2:]))
            elif t in (0, 1, 19, 20, 21):
                done = self._slice(nal, t)
                if done is not None:
                    out.append(done)
            elif t in (35, 36, 37, 38, 39, 40):
                continue
            else:
                raise NotImplementedError(f"NAL type {t}")
        if self.cur is not None:
            out.append(self._finish_picture())
        return out

    def _finish_picture(self):
        s = self.sps
        if any(v[0] for v in self.cur["dbk_slices"].values()):
            self._deblock()
        if self.cur["sao"]:
            self._sao_filter()
        Y, U, V = self.cur["Y"], self.cur["U"], self.cur["V"]
        self.ref = (Y.copy(), U.copy(), V.copy())
        self.cur = None
        cl, cr, ct, cb = s.crop
        return (Y[2 * ct:s.height - 2 * cb, 2 * cl:s.width - 2 * cr].copy(),
                U[ct:s.height // 2 - cb, cl:s.width // 2 - cr].copy(),
                V[ct:s.height // 2 - cb, cl:s.width // 2 - cr].copy())

    def _deblock(self):
        c = self.cur
        c["cb_off"], c["cr_off"] = self.pps.cb_qp_offset, self.pps.cr_qp_offset
        planes = (c["Y"], c["U"], c["V"])
        _deblock_pass(c, planes, True, c["dbk_slices"])
        _deblock_pass(c, planes, False, c["dbk_slices"])

    def _new_picture(self):
        s = self.sps
        nmin = (s.width // 4) * (s.height // 4)
        self.cur = {
            "Y": np.zeros((s.height, s.width), np.uint8),
            "U": np.zeros((s.height // 2, s.width // 2), np.uint8),
            "V": np.zeros((s.height // 2, s.width // 2), np.uint8),
            # per 4x4 block: slice address (-1 = not decoded), pred mode (0 inter, 1 intra), skip,
            # intra mode, mv, ct depth
            "slice": np.full((s.height // 4, s.width // 4), -1, np.int64),
            "intra": np.zeros((s.height // 4, s.width // 4), np.int64),
            "skip": np.zeros((s.height // 4, s.width // 4), np.int64),
            "ipm": np.ones((s.height // 4, s.width // 4), np.int64),
            "mv": np.zeros((s.height // 4, s.width // 4, 2), np.int64),
            "depth": np.zeros((s.height // 4, s.width // 4), np.int64),
            # deblocking side info per 4x4 block: transform / prediction edge on the left / top
            # boundary, luma cbf of the transform block, QpY
            "ev": np.zeros((s.height // 4, s.width // 4), bool),
            "eh": np.zeros((s.height // 4, s.width // 4), bool),
            "tev": np.zeros((s.height // 4, s.width // 4), bool),   # transform block edges
            "teh": np.zeros((s.height // 4, s.width // 4), bool),
            "cbf": np.zeros((s.height // 4, s.width // 4), bool),
            "qp": np.zeros((s.height // 4, s.width // 4), np.int64),
            "dbk_slices": {},
            "sao": {},         # (rx, ry) -> SAO parameters of the CTB
            "sao_slices": {},  # slice address -> (slice_sao_luma_flag, slice_sao_chroma_flag)
        }
        del nmin

    # ---------------- slice ----------------
    def _slice(self, nal: bytes, nut: int):
        s, p = self.sps, self.pps
        if s is None or p is None:
            raise BitstreamError("slice before parameter sets")
        payload = nal[2:]
        r = unescape(payload)
        b = Bits(r)
        first = b.u(1)
        if 16 <= nut <= 23:
            b.u(1)
        b.ue()
        ctb = 1 << s.log2_ctb
        wc = (s.width + ctb - 1) // ctb
        hc = (s.height + ctb - 1) // ctb
        addr = 0
        if not first:
            if p.dependent_slices:
                raise NotImplementedError("dependent slices")
            nbits = max(1, (wc * hc - 1).bit_length())
            addr = b.u(nbits)
        if first:
            if self.cur is not None:
                done = self._finish_picture()
            else:
                done = None
            self._new_picture()
        else:
            done = None
            if self.cur is None:
                raise BitstreamError("slice without a picture")
        b.u(p.extra_bits)
        slice_type = b.ue()
        if slice_type == 0:
            raise NotImplementedError("B slices")
        if p.output_flag_present:
            b.u(1)
        idr = nut in (19, 20)
        if not idr:
            b.u(s.log2_poc_lsb)
            if not b.u(1):
                self._st_rps(b, s.num_st_rps, s.st_rps)
            elif s.num_st_rps > 1:
                b.u(max(1, (s.num_st_rps - 1).bit_length()))
            if s.tmvp:
                if b.u(1):
                    raise NotImplementedError("TMVP")
        sao_luma = sao_chroma = False
        if s.sao:
            sao_luma = bool(b.u(1))
            sao_chroma = bool(b.u(1))   # ChromaArrayType != 0
        self.cur["sao_slices"][addr] = (sao_luma, sao_chroma)
        num_ref = p.num_ref_l0
        max_merge = 5
        if slice_type == 1:
            if b.u(1):
                num_ref = b.ue() + 1
            if p.lists_modification:
                raise NotImplementedError("list modification")
            cabac_init = b.u(1) if p.cabac_init_present else 0
            max_merge = 5 - b.ue()
        else:
            cabac_init = 0
        qp = p.init_qp + b.se()
        if p.slice_chroma_qp_offsets:
            b.se(); b.se()
        deblock_disabled = p.deblock_disabled
        beta_off, tc_off = p.beta_offset, p.tc_offset
        if p.deblock_override and b.u(1):
            deblock_disabled = bool(b.u(1))
            if not deblock_disabled:
                beta_off, tc_off = 2 * b.se(), 2 * b.se()
        across = p.loop_filter_across_slices
        if p.loop_filter_across_slices and (sao_luma or sao_chroma or not deblock_disabled):
            across = bool(b.u(1))
        # per-slice deblocking parameters, looked up by the slice map at filtering time
        self.cur["dbk_slices"][addr] = (not deblock_disabled, beta_off, tc_off, across)
        entry = []
        if p.tiles or p.wpp:
            n = b.ue()
            if n:
                ln = b.ue() + 1
                entry = [b.u(ln) + 1 for _ in range(n)]
        if p.slice_header_ext:
            b.u(8 * b.ue())
        # byte_alignment()
        if b.u(1) != 1:
            raise BitstreamError("byte_alignment")
        while b.p & 7:
            b.u(1)
        hdr_rbsp = b.p >> 3
        # map the RBSP header length to the escaped payload (entry points count EP bytes)
        pos, rb, zeros = 0, 0, 0
        while rb < hdr_rbsp:
            byte = payload[pos]
            if zeros >= 2 and byte == 3:
                zeros = 0
                pos += 1
                continue
            zeros = zeros + 1 if byte == 0 else 0
            pos += 1
            rb += 1
        starts = [pos]
        for e in entry:
            starts.append(starts[-1] + e)
        subs = [unescape(payload[starts[k]:(starts[k + 1] if k + 1 < len(starts) else len(payload))])
                for k in range(len(starts))]
        self._slice_data(addr, slice_type, qp, cabac_init, num_ref, max_merge, subs, wc, hc)
        return done

    # ---------------- slice data ----------------
    def _avail(self, xc, yc, xn, yn) -> bool:
        """z-scan availability (6.4.1) via the decoded map: inside the picture, decoded, same slice."""
        s = self.sps
        if xn < 0 or yn < 0 or xn >= s.width or yn >= s.height:
            return False
        sa = self.cur["slice"][yn >> 2, xn >> 2]
        return sa >= 0 and sa == self.slice_addr

    def _slice_data(self, addr, slice_type, qp, cabac_init, num_ref, max_merge, subs, wc, hc):
        s, p = self.sps, self.pps
        self.slice_addr = addr
        self.slice_type = slice_type
        self.qp = qp
        self.max_merge = max_merge
        self.num_ref = num_ref
        init_type = 0 if slice_type == 2 else (2 if cabac_init else 1)
        self.init_type = init_type
        ctb = 1 << s.log2_ctb
        self.ctx = init_contexts(init_type, qp)
        sub_i = 0
        self.cabac = Cabac(subs[0])
        sync = None
        a = addr
        while True:
            cx, cy = a % wc, a // wc
            if p.wpp and cx == 0 and a != addr:
                # new substream: arithmetic decoder restart, contexts from the WPP storage
                sub_i += 1
                if sub_i >= len(subs):
                    raise BitstreamError("missing WPP substream")
                self.cabac = Cabac(subs[sub_i])
                tr_x, tr_y = ctb, (cy - 1) * ctb
                if sync is not None and self._avail(0, cy * ctb, tr_x, tr_y):
                    self.ctx = copy_contexts(sync)
                else:
                    self.ctx = init_contexts(init_type, qp)
            elif p.wpp and cx == 0 and a == addr:
                pass
            luma, chroma = self.cur["sao_slices"][addr]
            if luma or chroma:
                self._sao_syntax(cx, cy, a, wc, luma, chroma)
            self._coding_quadtree(cx * ctb, cy * ctb, s.log2_ctb, 0)
            if p.wpp and cx == 1:
                sync = copy_contexts(self.ctx)
            if p.wpp and wc == 1:
                sync = None
            end = self.cabac.terminate()
            a += 1
            if end:
                break
            if p.wpp and a % wc == 0:
                if self.cabac.terminate() != 1:
                    raise BitstreamError("end_of_subset_one_bit")
            if a >= wc * hc:
                raise BitstreamError("slice runs past the picture")

    # ---------------- SAO ----------------
    def _sao_syntax(self, rx, ry, ctb_addr, wc, luma, chroma):
        """sao(rx, ry) (7.3.8.3): merge flags, per-component type / offsets / band position /
        edge class; stores SaoTypeIdx, SaoOffsetVal[1..4], band position and class."""
        c = self.cur
        merge_left = merge_up = 0
        if rx > 0 and ctb_addr - 1 >= self.slice_addr:
            merge_left = self._dec("sao_merge_flag")
        if ry > 0 and not merge_left and ctb_addr - wc >= self.slice_addr:
            merge_up = self._dec("sao_merge_flag")
        if merge_left:
            c["sao"][(rx, ry)] = c["sao"][(rx - 1, ry)]
            return
        if merge_up:
            c["sao"][(rx, ry)] = c["sao"][(rx, ry - 1)]
            return
        prm = {"type": [0, 0, 0], "off": [[0] * 4 for _ in range(3)], "band": [0, 0, 0], "cls": [0, 0, 0]}
        cab = self.cabac
        for ci in range(3):
            if not ((luma and ci == 0) or (chroma and ci > 0)):
                continue
            if ci < 2:
                t = 0
                if self._dec("sao_type_idx"):
                    t = 2 if cab.bypass() else 1     # TR cMax 2: "10" band, "11" edge
                prm["type"][ci] = t
            else:
                prm["type"][2] = prm["type"][1]
                prm["cls"][2] = prm["cls"][1]
            t = prm["type"][ci]
            if t == 0:
                continue
            absv = []
            for _ in range(4):                     # sao_offset_abs: TR cMax 7, bypass
                v = 0
                while v < 7 and cab.bypass():
                    v += 1
                absv.append(v)
            if t == 1:
                sg = [(-1 if cab.bypass() else 1) if a else 1 for a in absv]
                prm["band"][ci] = cab.bypass_bits(5)
                prm["off"][ci] = [a * g for a, g in zip(absv, sg)]
            else:
                if ci < 2:
                    prm["cls"][ci] = cab.bypass_bits(2)
                prm["off"][ci] = [absv[0], absv[1], -absv[2], -absv[3]]
        c["sao"][(rx, ry)] = prm

    def _sao_filter(self):
        """8.7.3 on the deblocked picture: band offsets by (sample >> 3) relative to the band
        position, edge offsets from the sign pattern against the class's two neighbours;
        samples whose edge neighbour lies outside the picture or across a slice boundary
        that may not be filtered stay unchanged."""
        c = self.cur
        s = self.sps
        ctb = 1 << s.log2_ctb
        hpos = {0: (-1, 1), 1: (0, 0), 2: (-1, 1), 3: (1, -1)}
        vpos = {0: (0, 0), 1: (-1, 1), 2: (-1, 1), 3: (-1, 1)}
        slice_map = c["slice"]
        across = {a: v[3] for a, v in c["dbk_slices"].items()}
        for ci, name in enumerate(("Y", "U", "V")):
            sh = 0 if ci == 0 else 1
            src = c[name].astype(np.int64)
            out = c[name]
            H, W = src.shape
            n = ctb >> sh
            ys_all, xs_all = np.mgrid[0:H, 0:W]
            sl = slice_map[(ys_all << sh) >> 2, (xs_all << sh) >> 2]
            for (rx, ry), prm in c["sao"].items():
                t = prm["type"][ci]
                y0, x0 = ry * n, rx * n
                if t == 0 or y0 >= H or x0 >= W:
                    continue
                sao_l, sao_c = c["sao_slices"][int(sl[y0, x0])]
                if not (sao_l if ci == 0 else sao_c):
                    continue
                ys, xs = ys_all[y0:y0 + n, x0:x0 + n], xs_all[y0:y0 + n, x0:x0 + n]
                v = src[y0:y0 + n, x0:x0 + n]
                off = prm["off"][ci]
                if t == 1:
                    k = ((v >> 3) - prm["band"][ci]) & 31
                    res = v.copy()
                    for i in range(4):
                        res[k == i] += off[i]
                else:
                    cls = prm["cls"][ci]
                    ok = np.ones_like(v, bool)
                    nb = []
                    cur_sl = sl[y0:y0 + n, x0:x0 + n]
                    for i in range(2):
                        yy, xx = ys + vpos[cls][i], xs + hpos[cls][i]
                        inside = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
                        yyc, xxc = np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)
                        nsl = sl[yyc, xxc]
                        # across a slice boundary: the later slice's flag decides (MinTbAddrZs order)
                        later = np.where(nsl < cur_sl, cur_sl, nsl)
                        allow = np.vectorize(lambda a: across.get(int(a), False))(later) if (nsl != cur_sl).any() \
                            else np.ones_like(v, bool)
                        ok &= inside & ((nsl == cur_sl) | allow)
                        nb.append(src[yyc, xxc])
                    e = 2 + np.sign(v - nb[0]) + np.sign(v - nb[1])
                    e = np.where(e <= 2, np.where(e == 2, 0, e + 1), e)
                    e = np.where(ok, e, 0)
                    res = v.copy()
                    for i in range(1, 5):
                        res[e == i] += off[i - 1]
                out[y0:y0 + n, x0:x0 + n] = np.clip(res, 0, 255)

    # ---------------- coding tree ----------------
    def _dec(self, name, idx=0):
        return self.cabac.decision(self.ctx[name][idx])

    def _coding_quadtree(self, x0, y0, log2, depth):
        s = self.sps
        size = 1 << log2
        if x0 + size <= s.width and y0 + size <= s.height and log2 > s.log2_min_cb:
            al, aa = self._avail(x0, y0, x0 - 1, y0), self._avail(x0, y0, x0, y0 - 1)
            cond = split_cu_ctx_inc(al, int(self.cur["depth"][y0 >> 2, (x0 - 1) >> 2]) if al else 0,
                                    aa, int(self.cur["depth"][(y0 - 1) >> 2, x0 >> 2]) if aa else 0, depth)
            split = self._dec("split_cu_flag", cond)
        else:
            split = 1 if log2 > s.log2_min_cb else 0
        if split:
            h = size >> 1
            for dy in (0, h):
                for dx in (0, h):
                    if x0 + dx < s.width and y0 + dy < s.height:
                        self._coding_quadtree(x0 + dx, y0 + dy, log2 - 1, depth + 1)
            return
        self._coding_unit(x0, y0, log2, depth)

    def _mark(self, x0, y0, n, **vals):
        sl = (slice(y0 >> 2, (y0 + n) >> 2), slice(x0 >> 2, (x0 + n) >> 2))
        for k, v in vals.items():
            self.cur[k][sl] = v

    def _coding_unit(self, x0, y0, log2, depth):
        s = self.sps
        n = 1 << log2
        self._block_edges(x0, y0, n)
        self._mark(x0, y0, n, qp=self.qp, cbf=0)
        skip = 0
        if self.slice_type != 2:
            cond = 0
            if self._avail(x0, y0, x0 - 1, y0) and self.cur["skip"][y0 >> 2, (x0 - 1) >> 2]:
                cond += 1
            if self._avail(x0, y0, x0, y0 - 1) and self.cur["skip"][(y0 - 1) >> 2, x0 >> 2]:
                cond += 1
            skip = self._dec("cu_skip_flag", cond)
        if skip:
            mv = self._prediction_unit(x0, y0, n, skip=True)
            self._inter_pred(x0, y0, n, mv)
            self._mark(x0, y0, n, slice=self.slice_addr, intra=0, skip=1, depth=depth, ipm=1)
            self.cur["mv"][y0 >> 2:(y0 + n) >> 2, x0 >> 2:(x0 + n) >> 2] = mv
            return
        intra = 1 if self.slice_type == 2 else self._dec("pred_mode_flag")
        part = 0   # 0 2Nx2N, 1 2NxN, 2 Nx2N, 3 NxN (Table 7-10 order aside)
        if not intra or log2 == s.log2_min_cb:   # intra part_mode only at the minimum CB size
            part = part_mode_of_bins(lambda i: self._dec("part_mode", i), bool(intra), log2, s.log2_min_cb, s.amp)
        if intra:
            npu = 4 if part == 3 else 1
            h = n // 2 if part == 3 else n
            pus = [(x0 + (k & 1) * h, y0 + (k >> 1) * h) for k in range(npu)]
            prev = [self._dec("prev_intra_luma_pred_flag") for _ in pus]
            local = {}   # modes of this CU's PUs (z-scan available to the later ones, 6.4.1)
            modes = []
            for k, (xp, yp) in enumerate(pus):
                if prev[k]:
                    mpm_idx = 0
                    if self.cabac.bypass():
                        mpm_idx = 1 + self.cabac.bypass()
                else:
                    rem = self.cabac.bypass_bits(5)
                # candidate list (8.4.2)
                cands = []
                for (xn, yn) in ((xp - 1, yp), (xp, yp - 1)):
                    inside = x0 <= xn < x0 + n and y0 <= yn < y0 + n
                    if inside:
                        cands.append(local[(xn - x0) // h, (yn - y0) // h])
                    elif not self._avail(x0, y0, xn, yn) or not self.cur["intra"][yn >> 2, xn >> 2]:
                        cands.append(1)
                    elif yn == yp - 1 and yn < ((yp >> s.log2_ctb) << s.log2_ctb):
                        cands.append(1)
                    else:
                        cands.append(int(self.cur["ipm"][yn >> 2, xn >> 2]))
                lst = mpm_list(*cands)
                mode = lst[mpm_idx] if prev[k] else mode_from_rem(rem, lst)
                local[(xp - x0) // h, (yp - y0) // h] = mode
                modes.append(mode)
            c = self._dec("intra_chroma_pred_mode")
            chroma = 4 if c == 0 else self.cabac.bypass_bits(2)
            mode0 = modes[0]
            if chroma == 4:
                cmode = mode0
            else:
                cmode = [0, 26, 10, 1][chroma]
                if cmode == mode0:
                    cmode = 34
            # decoded-ness (the slice map) is set per transform unit by _intra_pred, so a TU's
            # not-yet-decoded neighbours inside this CU stay unavailable
            self._mark(x0, y0, n, intra=1, skip=0, depth=depth)
            for (xp, yp), mode in zip(pus, modes):
                self._mark(xp, yp, h, ipm=mode)
            self.cur["mv"][y0 >> 2:(y0 + n) >> 2, x0 >> 2:(x0 + n) >> 2] = 0
            self.cu_intra = (None, cmode)   # luma modes: per TU from the ipm map
            self._transform_tree(x0, y0, x0, y0, log2, 0, 0, True, s.max_th_intra + (1 if part == 3 else 0), (1, 1),
                                 intra_split=part == 3)
            return
        rects = {0: [(x0, y0, n, n)], 1: [(x0, y0, n, n // 2), (x0, y0 + n // 2, n, n // 2)],
                 2: [(x0, y0, n // 2, n), (x0 + n // 2, y0, n // 2, n)]}[part]
        merge0 = 0
        for pi, (xp, yp, pw, ph) in enumerate(rects):
            merge = self._dec("merge_flag")
            if pi == 0:
                merge0 = merge
            mv = self._prediction_unit(xp, yp, pw, skip=False, merge=merge, ph=ph, part=part, pidx=pi)
            self._inter_pred(xp, yp, pw, mv, ph)
            self._mark(xp, yp, 0, slice=self.slice_addr)
            sl = (slice(yp >> 2, (yp + ph) >> 2), slice(xp >> 2, (xp + pw) >> 2))
            self.cur["slice"][sl] = self.slice_addr
            self.cur["mv"][sl] = mv
            if pi == 1:   # prediction block edge (8.7.2.4)
                if part == 1:
                    self.cur["eh"][yp >> 2, xp >> 2:(xp + pw) >> 2] = True
                else:
                    self.cur["ev"][yp >> 2:(yp + ph) >> 2, xp >> 2] = True
        self._mark(x0, y0, n, slice=self.slice_addr, intra=0, skip=0, depth=depth, ipm=1)
        root = 1 if (merge0 and part == 0) else self._dec("rqt_root_cbf")
        if root:
            self.cu_intra = None
            self._transform_tree(x0, y0, x0, y0, log2, 0, 0, False, s.max_th_inter, (1, 1),
                                 inter_split=s.max_th_inter == 0 and part != 0)

    # ---------------- inter ----------------
    def _mvd(self):
        g0 = [self._dec("abs_mvd_greater0_flag"), self._dec("abs_mvd_greater0_flag")]
        g1 = [self._dec("abs_mvd_greater1_flag") if g0[0] else 0, self._dec("abs_mvd_greater1_flag") if g0[1] else 0]
        out = []
        for i in range(2):
            v = 0
            if g0[i]:
                v = 1
                if g1[i]:
                    # EG1
                    k = 1
                    absv = 0
                    while self.cabac.bypass():
                        absv += 1 << k
                        k += 1
                    absv += self.cabac.bypass_bits(k)
                    v = absv + 2
                if self.cabac.bypass():
                    v = -v
            out.append(v)
        return out

    def _nb_motion(self, x0, y0, xn, yn):
        if not self._avail(x0, y0, xn, yn) or self.cur["intra"][yn >> 2, xn >> 2]:
            return None
        return tuple(int(v) for v in self.cur["mv"][yn >> 2, xn >> 2])

    def _merge_cands(self, x0, y0, w, h, part=0, pidx=0):
        A1 = self._nb_motion(x0, y0, x0 - 1, y0 + h - 1)
        B1 = self._nb_motion(x0, y0, x0 + w - 1, y0 - 1)
        B0 = self._nb_motion(x0, y0, x0 + w, y0 - 1)
        A0 = self._nb_motion(x0, y0, x0 - 1, y0 + h)
        B2 = self._nb_motion(x0, y0, x0 - 1, y0 - 1)
        if pidx == 1 and part == 2:   # 8.5.3.2.3: PART_Nx2N / 2NxN part 1 ignore A1 / B1
            A1 = None
        if pidx == 1 and part == 1:
            B1 = None
        lst = []
        if A1 is not None:
            lst.append(A1)
        if B1 is not None and B1 != A1:
            lst.append(B1)
        if B0 is not None and B0 != B1:
            lst.append(B0)
        if A0 is not None and A0 != A1:
            lst.append(A0)
        cnt = sum(v is not None for v in (A1, B1 if (B1 is not None and B1 != A1) else None,
                                          B0 if (B0 is not None and B0 != B1) else None,
                                          A0 if (A0 is not None and A0 != A1) else None))
        if B2 is not None and B2 != A1 and B2 != B1 and cnt != 4:
            lst.append(B2)
        zero_idx = 0
        while len(lst) < self.max_merge:
            lst.append((0, 0))   # refIdx min(zeroIdx, numRef-1): same picture, zero vector
            zero_idx += 1
        return lst

    def _amvp_cands(self, x0, y0, w, h):
        A0 = self._nb_motion(x0, y0, x0 - 1, y0 + h)
        A1 = self._nb_motion(x0, y0, x0 - 1, y0 + h - 1)
        B0 = self._nb_motion(x0, y0, x0 + w, y0 - 1)
        B1 = self._nb_motion(x0, y0, x0 + w - 1, y0 - 1)
        B2 = self._nb_motion(x0, y0, x0 - 1, y0 - 1)
        # single reference picture: every inter neighbour refers to it (no scaling)
        is_scaled = A0 is not None or A1 is not None   # availableA0 || availableA1 (6.4.2: inter only)
        mvA = A0 if A0 is not None else A1
        mvB = B0 if B0 is not None else (B1 if B1 is not None else B2)
        if not is_scaled and mvB is not None:
            mvA = mvB
        if not is_scaled:
            mvB = B0 if B0 is not None else (B1 if B1 is not None else B2)
        lst = []
        if mvA is not None:
            lst.append(mvA)
        if mvB is not None and not (mvA is not None and mvA == mvB):
            lst.append(mvB)
        while len(lst) < 2:
            lst.append((0, 0))
        return lst[:2]

    def _prediction_unit(self, x0, y0, n, skip, merge=1, ph=None, part=0, pidx=0):
        h = n if ph is None else ph
        if skip or merge:
            idx = 0
            if self.max_merge > 1 and self._dec("merge_idx"):
                idx = 1
                while idx < self.max_merge - 1 and self.cabac.bypass():
                    idx += 1
            return self._merge_cands(x0, y0, n, h, part, pidx)[idx]
        if self.num_ref > 1:
            raise NotImplementedError("ref_idx")
        mvd = self._mvd()
        mvp = self._dec("mvp_flag")
        pred = self._amvp_cands(x0, y0, n, h)[mvp]
        mv = [(pred[i] + mvd[i] + (1 << 16)) % (1 << 16) for i in range(2)]
        return tuple(v - (1 << 16) if v >= (1 << 15) else v for v in mv)

    def _inter_pred(self, x0, y0, n, mv, ph=None):
        if self.ref is None:
            raise BitstreamError("P slice without a reference picture")
        s = self.sps
        hgt = n if ph is None else ph
        RY, RU, RV = (r.astype(np.int64) for r in self.ref)
        mvx, mvy = mv
        ys = np.arange(hgt)[:, None]
        xs = np.arange(n)[None, :]
        xi, yi, fx, fy = x0 + (mvx >> 2), y0 + (mvy >> 2), mvx & 3, mvy & 3

        def refl(xx, yy):
            return RY[np.clip(yy, 0, s.height - 1), np.clip(xx, 0, s.width - 1)]
        if fx == 0 and fy == 0:
            pred = refl(xi + xs, yi + ys) << 6
        elif fy == 0:
            pred = sum(LUMA_FILTER[fx][i] * refl(xi + xs + i - 3, yi + ys) for i in range(8))
        elif fx == 0:
            pred = sum(LUMA_FILTER[fy][i] * refl(xi + xs, yi + ys + i - 3) for i in range(8))
        else:
            tmp = [sum(LUMA_FILTER[fx][i] * refl(xi + xs + i - 3, yi + ys + k - 3) for i in range(8)) for k in range(8)]
            pred = sum(LUMA_FILTER[fy][k] * tmp[k] for k in range(8)) >> 6
        self.cur["Y"][y0:y0 + hgt, x0:x0 + n] = np.clip((pred + 32) >> 6, 0, 255)
        m, mh = n // 2, hgt // 2
        ys = np.arange(mh)[:, None]
        xs = np.arange(m)[None, :]
        xc0, yc0 = x0 // 2, y0 // 2
        xi, yi, fx, fy = xc0 + (mvx >> 3), yc0 + (mvy >> 3), mvx & 7, mvy & 7
        for plane, R in (("U", RU), ("V", RV)):
            def refc(xx, yy, R=R):
                return R[np.clip(yy, 0, s.height // 2 - 1), np.clip(xx, 0, s.width // 2 - 1)]
            if fx == 0 and fy == 0:
                pred = refc(xi + xs, yi + ys) << 6
            elif fy == 0:
                pred = sum(CHROMA_FILTER[fx][i] * refc(xi + xs + i - 1, yi + ys) for i in range(4))
            elif fx == 0:
                pred = sum(CHROMA_FILTER[fy][i] * refc(xi + xs, yi + ys + i - 1) for i in range(4))
            else:
                tmp = [sum(CHROMA_FILTER[fx][i] * refc(xi + xs + i - 1, yi + ys + k - 1) for i in range(4))
                       for k in range(4)]
                pred = sum(CHROMA_FILTER[fy][k] * tmp[k] for k in range(4)) >> 6
            self.cur[plane][yc0:yc0 + mh, xc0:xc0 + m] = np.clip((pred + 32) >> 6, 0, 255)

    # ---------------- transform tree ----------------
    def _transform_tree(self, x0, y0, xb, yb, log2, depth, blk, intra, max_depth, parent_cbf, intra_split=False,
                        inter_split=False):
        s = self.sps
        forced = (intra_split or inter_split) and depth == 0
        if log2 <= s.log2_max_tb and log2 > s.log2_min_tb and depth < max_depth and not forced:
            split = self._dec("split_transform_flag", 5 - log2)
        else:
            split = 1 if (log2 > s.log2_max_tb or forced) else 0
        cbf_cb = cbf_cr = 0
        if log2 > 2:
            if depth == 0 or parent_cbf[0]:
                cbf_cb = self._dec("cbf_chroma", depth)
            if depth == 0 or parent_cbf[1]:
                cbf_cr = self._dec("cbf_chroma", depth)
        else:
            cbf_cb, cbf_cr = parent_cbf
        if split:
            h = 1 << (log2 - 1)
            for k, (dx, dy) in enumerate(((0, 0), (h, 0), (0, h), (h, h))):
                self._transform_tree(x0 + dx, y0 + dy, x0, y0, log2 - 1, depth + 1, k, intra, max_depth,
                                     (cbf_cb, cbf_cr))
            return
        cbf_y = 1
        if intra or depth != 0 or cbf_cb or cbf_cr:
            cbf_y = self._dec("cbf_luma", 1 if depth == 0 else 0)
        self._transform_unit(x0, y0, xb, yb, log2, blk, cbf_y, cbf_cb, cbf_cr, intra)

    def _qp_c(self, off):
        qpi = min(max(self.qp + off, 0), 57)
        if qpi < 30:
            return qpi
        if qpi > 43:
            return qpi - 6
        return QPC_TABLE[qpi]

    def _block_edges(self, x0, y0, n):
        """Coding / transform block edges (left and top boundary of the block)."""
        c = self.cur
        for k in ("ev", "tev"):
            c[k][y0 >> 2:(y0 + n) >> 2, x0 >> 2] = True
        for k in ("eh", "teh"):
            c[k][y0 >> 2, x0 >> 2:(x0 + n) >> 2] = True

    def _transform_unit(self, x0, y0, xb, yb, log2, blk, cbf_y, cbf_cb, cbf_cr, intra):
        p = self.pps
        n = 1 << log2
        self._block_edges(x0, y0, n)
        self._mark(x0, y0, n, cbf=bool(cbf_y))
        mode, cmode = self.cu_intra if intra else (None, None)
        if intra:
            mode = int(self.cur["ipm"][y0 >> 2, x0 >> 2])   # the PU covering this TU
            self._intra_pred("Y", x0, y0, n, mode, 0)
        if cbf_y:
            self._residual(x0, y0, log2, 0, mode, self.qp)
        if log2 > 2:
            xc, yc, lc = x0 // 2, y0 // 2, log2 - 1
        elif blk == 3:
            xc, yc, lc = xb // 2, yb // 2, 2
        else:
            return
        for plane, cbf, off, ci in (("U", cbf_cb, p.cb_qp_offset, 1), ("V", cbf_cr, p.cr_qp_offset, 2)):
            if intra:
                self._intra_pred(plane, xc, yc, 1 << lc, cmode, ci)
            if cbf:
                self._residual(xc, yc, lc, ci, cmode, self._qp_c(off))

    # ---------------- residual ----------------
    def _residual(self, x0, y0, log2, cidx, intra_mode, qp):
        n = 1 << log2
        scan_idx = 0
        if intra_mode is not None and (log2 == 2 or (log2 == 3 and cidx == 0)):
            if 6 <= intra_mode <= 14:
                scan_idx = 2
            elif 22 <= intra_mode <= 30:
                scan_idx = 1
        # transform_skip_flag (7.3.8.11): 4x4 TUs when the PPS enables it
        ts = bool(self.pps.transform_skip and log2 == 2 and self._dec("transform_skip_flag", 0 if cidx == 0 else 1))
        # last significant coefficient
        if cidx == 0:
            off, sh = 3 * (log2 - 2) + ((log2 - 1) >> 2), (log2 + 1) >> 2
        else:
            off, sh = 15, log2 - 2
        cmax = (log2 << 1) - 1

        def prefix(name):
            v = 0
            while v < cmax and self._dec(name, off + (v >> sh)):
                v += 1
            return v
        px, py = prefix("last_x_prefix"), prefix("last_y_prefix")

        def fin(pre):
            if pre <= 3:
                return pre
            nb = (pre >> 1) - 1
            suf = self.cabac.bypass_bits(nb)
            return (1 << nb) * (2 + (pre & 1)) + suf
        lx = fin(px)
        ly = fin(py)
        if scan_idx == 2:
            lx, ly = ly, lx
        sb = scan_order(n >> 2, scan_idx) if log2 > 2 else [(0, 0)]
        sc4 = scan_order(4, scan_idx)
        levels = np.zeros((n, n), np.int64)
        # locate last sub-block / position
        last_sb, last_pos = None, None
        for i, (xs, ys) in enumerate(sb):
            for k, (xp, yp) in enumerate(sc4):
                if xs * 4 + xp == lx and ys * 4 + yp == ly:
                    last_sb, last_pos = i, k
        if last_sb is None:
            raise BitstreamError("last position outside the TU")
        csbf = {}
        greater1_ctx_prev = None
        nsb = n >> 2
        for i in range(last_sb, -1, -1):
            xs, ys = sb[i]
            infer_dc = False
            if i < last_sb and i > 0:
                c = 0
                if xs < nsb - 1:
                    c += csbf.get((xs + 1, ys), 0)
                if ys < nsb - 1:
                    c += csbf.get((xs, ys + 1), 0)
                flag = self._dec("coded_sub_block_flag", min(c, 1) + (2 if cidx else 0))
                infer_dc = True
            else:
                flag = 1
            csbf[(xs, ys)] = flag
            sig = [0] * 16
            start = last_pos - 1 if i == last_sb else 15
            if i == last_sb:
                sig[last_pos] = 1
            prev_csbf = 0
            if xs < nsb - 1:
                prev_csbf |= csbf.get((xs + 1, ys), 0)
            if ys < nsb - 1:
                prev_csbf |= csbf.get((xs, ys + 1), 0) << 1
            for k in range(start, -1, -1):
                if not flag:
                    break
                xp, yp = sc4[k]
                xc, yc = xs * 4 + xp, ys * 4 + yp
                if k == 0 and infer_dc:
                    sig[0] = 1
                    break
                if log2 == 2:
                    sctx = [0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8][(yc << 2) + xc]
                elif xc + yc == 0:
                    sctx = 0
                else:
                    if prev_csbf == 0:
                        sctx = 2 if xp + yp == 0 else (1 if xp + yp < 3 else 0)
                    elif prev_csbf == 1:
                        sctx = 2 if yp == 0 else (1 if yp == 1 else 0)
                    elif prev_csbf == 2:
                        sctx = 2 if xp == 0 else (1 if xp == 1 else 0)
                    else:
                        sctx = 2
                    if cidx == 0:
                        if xs or ys:
                            sctx += 3
                        sctx += (9 if scan_idx == 0 else 15) if log2 == 3 else 21
                    else:
                        sctx += 9 if log2 == 3 else 12
                v = self._dec("sig_coeff_flag", sctx if cidx == 0 else 27 + sctx)
                sig[k] = v
                if v:
                    infer_dc = False
            if not any(sig):
                continue
            # greater1
            ctx_set = 0 if (i == 0 or cidx > 0) else 2
            if greater1_ctx_prev is not None and greater1_ctx_prev == 0:
                ctx_set += 1
            g1ctx = 1
            g1 = [0] * 16
            g2 = [0] * 16
            first_g1 = -1
            n_g1 = 0
            for k in range(15, -1, -1):
                if sig[k]:
                    if n_g1 < 8:
                        f = self._dec("coeff_abs_level_greater1_flag", ctx_set * 4 + min(3, g1ctx) + (16 if cidx else 0))
                        g1[k] = f
                        n_g1 += 1
                        if f and first_g1 < 0:
                            first_g1 = k
                        if g1ctx > 0:
                            g1ctx = 0 if f else g1ctx + 1
            greater1_ctx_prev = g1ctx
            if first_g1 >= 0:
                g2[first_g1] = self._dec("coeff_abs_level_greater2_flag", ctx_set + (4 if cidx else 0))
            signs = [0] * 16
            for k in range(15, -1, -1):
                if sig[k]:
                    signs[k] = self.cabac.bypass()
            rice = 0
            nsig = 0
            for k in range(15, -1, -1):
                if not sig[k]:
                    continue
                base = 1 + g1[k] + g2[k]
                thr = (3 if k == first_g1 else 2) if nsig < 8 else 1
                absv = base
                if base == thr:
                    # coeff_abs_level_remaining (9.3.3.11): prefix unary, TR / EGk suffix
                    pre = 0
                    while self.cabac.bypass():
                        pre += 1
                    if pre <= 3:
                        rem = (pre << rice) + self.cabac.bypass_bits(rice)
                    else:
                        k2 = pre - 3 + rice
                        rem = (((1 << (pre - 3)) + 3 - 1) << rice) + self.cabac.bypass_bits(k2)
                    absv = base + rem
                    if absv > 3 * (1 << rice):
                        rice = min(rice + 1, 4)
                xp, yp = sc4[k]
                levels[ys * 4 + yp, xs * 4 + xp] = -absv if signs[k] else absv
                nsig += 1
        dst = cidx == 0 and log2 == 2 and intra_mode is not None
        r = residual_from_levels(levels, qp, log2, ts, dst)
        plane = "YUV"[cidx]
        blk = self.cur[plane][y0:y0 + n, x0:x0 + n].astype(np.int64)
        self.cur[plane][y0:y0 + n, x0:x0 + n] = np.clip(blk + r, 0, 255)

    # ---------------- intra ----------------
    def _intra_pred(self, plane, x0, y0, n, mode, cidx):
        """8.4.4.2: reference samples, substitution, filtering and the prediction."""
        s = self.sps
        P = self.cur[plane]
        sh = 0 if cidx == 0 else 1
        W = s.width >> sh
        H = s.height >> sh
        # p[-1][y] for y = -1 .. 2n-1 and p[x][-1] for x = 0 .. 2n-1
        left = np.zeros(2 * n + 1, np.int64)   # index y+1
        top = np.zeros(2 * n, np.int64)
        lav = np.zeros(2 * n + 1, bool)
        tav = np.zeros(2 * n, bool)

        def av(xs, ys):   # sample coords in this plane -> availability of the luma location
            if xs < 0 or ys < 0 or xs >= W or ys >= H:
                return False
            return self._avail(x0 << sh, y0 << sh, xs << sh, ys << sh)
        for y in range(-1, 2 * n):
            if av(x0 - 1, y0 + y):
                left[y + 1] = P[y0 + y, x0 - 1]
                lav[y + 1] = True
        for x in range(2 * n):
            if av(x0 + x, y0 - 1):
                top[x] = P[y0 - 1, x0 + x]
                tav[x] = True
        # linear order: p[-1][2n-1] .. p[-1][-1], p[0][-1] .. p[2n-1][-1]
        lin = [left[y + 1] for y in range(2 * n - 1, -2, -1)] + list(top)
        lav_ = [lav[y + 1] for y in range(2 * n - 1, -2, -1)] + list(tav)
        if not any(lav_):
            lin = [128] * len(lin)
        else:
            first = lav_.index(True)
            for i in range(first):
                lin[i] = lin[first]
            for i in range(first + 1, len(lin)):
                if not lav_[i]:
                    lin[i] = lin[i - 1]
        lin = np.array(lin, np.int64)
        log2 = n.bit_length() - 1
        if cidx == 0 and mode != 1 and n != 4:
            thres = {8: 7, 16: 1, 32: 0}[n]
            if min(abs(mode - 26), abs(mode - 10)) > thres:
                if s.strong_smoothing and n == 32:
                    raise NotImplementedError("strong intra smoothing")
                f = lin.copy()
                f[1:-1] = (lin[:-2] + 2 * lin[1:-1] + lin[2:] + 2) >> 2
                lin = f

        def L(y):
            return lin[2 * n - 1 - y]

        def T(x):
            return lin[2 * n + 1 + x]
        pred = np.zeros((n, n), np.int64)
        if mode == 0:
            for y in range(n):
                for x in range(n):
                    pred[y, x] = ((n - 1 - x) * L(y) + (x + 1) * T(n) + (n - 1 - y) * T(x) + (y + 1) * L(n) + n) >> (log2 + 1)
        elif mode == 1:
            dc = (sum(T(x) for x in range(n)) + sum(L(y) for y in range(n)) + n) >> (log2 + 1)
            pred[:] = dc
            if cidx == 0 and n < 32:
                pred[0, 0] = (L(0) + 2 * dc + T(0) + 2) >> 2
                for x in range(1, n):
                    pred[0, x] = (T(x) + 3 * dc + 2) >> 2
                for y in range(1, n):
                    pred[y, 0] = (L(y) + 3 * dc + 2) >> 2
        else:
            ang = INTRA_ANGLE[mode]
            ref = {}
            if mode >= 18:
                for x in range(0, 2 * n + 1):
                    ref[x] = T(x - 1)
                if ang < 0 and (n * ang) >> 5 < -1:
                    for x in range((n * ang) >> 5, 0):
                        ref[x] = L(-1 + ((x * INV_ANGLE[mode] + 128) >> 8))
                for y in range(n):
                    idx, fact = ((y + 1) * ang) >> 5, ((y + 1) * ang) & 31
                    for x in range(n):
                        if fact:
                            pred[y, x] = ((32 - fact) * ref[x + idx + 1] + fact * ref[x + idx + 2] + 16) >> 5
                        else:
                            pred[y, x] = ref[x + idx + 1]
                if mode == 26 and cidx == 0 and n < 32:
                    for y in range(n):
                        pred[y, 0] = min(max(T(0) + ((L(y) - L(-1)) >> 1), 0), 255)
            else:
                for x in range(0, 2 * n + 1):
                    ref[x] = L(x - 1)
                if ang < 0 and (n * ang) >> 5 < -1:
                    for x in range((n * ang) >> 5, 0):
                        ref[x] = T(-1 + ((x * INV_ANGLE[mode] + 128) >> 8))
                for x in range(n):
                    idx, fact = ((x + 1) * ang) >> 5, ((x + 1) * ang) & 31
                    for y in range(n):
                        if fact:
                            pred[y, x] = ((32 - fact) * ref[y + idx + 1] + fact * ref[y + idx + 2] + 16) >> 5
                        else:
                            pred[y, x] = ref[y + idx + 1]
                if mode == 10 and cidx == 0 and n < 32:
                    for x in range(n):
                        pred[0, x] = min(max(L(0) + ((T(x) - T(-1)) >> 1), 0), 255)
        P[y0:y0 + n, x0:x0 + n] = np.clip(pred, 0, 255)
        # mark the TU decoded for later intra neighbours (luma drives availability)
        if cidx == 0:
            self._mark(x0, y0, n, slice=self.slice_addr)


BETA_TABLE = [0] * 16 + [6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32, 34, 36, 38, 40,
                          42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64]                      # Table 8-11 (beta')
TC_TABLE = [0] * 18 + [1] * 9 + [2] * 4 + [3] * 4 + [4] * 3 + [5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24]


def split_cu_ctx_inc(avail_l: bool, depth_l: int, avail_a: bool, depth_a: int, cqt_depth: int) -> int:
    """ctxInc of split_cu_flag (9.3.4.2.2, Table 9-41 condTerm CtDepth[xNb][yNb] > cqtDepth)."""
    return int(avail_l and depth_l > cqt_depth) + int(avail_a and depth_a > cqt_depth)


def part_mode_of_bins(dec, intra: bool, log2_cb: int, log2_min_cb: int, amp: bool) -> int:
    """part_mode (7.4.9.5) from its bins (Table 9-43; AMP off), `dec(ctx_inc)` the next
    context-coded bin: 0 PART_2Nx2N, 1 PART_2NxN, 2 PART_Nx2N, 3 PART_NxN."""
    if dec(0):
        return 0
    if intra:
        return 3   # only coded at the minimum CB size: "0" = NxN
    if log2_cb > log2_min_cb and amp:
        raise NotImplementedError("AMP")
    if log2_cb == log2_min_cb and log2_cb > 3:
        raise NotImplementedError("inter NxN")
    return 1 if dec(1) else 2


def mpm_list(a: int, b: int) -> list:
    """candModeList (8.4.2) from candIntraPredModeA / B."""
    if a == b:
        return [0, 1, 26] if a < 2 else [a, 2 + ((a + 29) % 32), 2 + ((a - 2 + 1) % 32)]
    third = 0 if (a != 0 and b != 0) else (1 if (a != 1 and b != 1) else 26)
    return [a, b, third]


def mode_from_rem(rem: int, lst: list) -> int:
    """IntraPredModeY from rem_intra_luma_pred_mode (8.4.2: ascending candidates, increment)."""
    mode = rem
    for c in sorted(lst):
        if mode >= c:
            mode += 1
    return mode


def _qpc(qpi: int) -> int:
    qpi = min(max(qpi, 0), 57)
    return qpi if qpi < 30 else (qpi - 6 if qpi > 43 else QPC_TABLE[qpi])


def _deblock_pass(c: dict, planes: tuple, vertical: bool, slices: dict) -> None:
    """One direction of 8.7.2 over the whole picture (all edges of a direction are
    independent: 8 samples apart, at most 3 samples changed per side)."""
    Y, U, V = planes
    edge = c["ev"] if vertical else c["eh"]
    tedge = c["tev"] if vertical else c["teh"]
    sl, intra, cbf, mv, qp = c["slice"], c["intra"], c["cbf"], c["mv"], c["qp"]
    h4, w4 = edge.shape
    yq, xq = np.nonzero(edge)
    keep = (xq % 2 == 0) & (xq > 0) if vertical else (yq % 2 == 0) & (yq > 0)   # 8x8 grid, not the border
    yq, xq = yq[keep], xq[keep]
    yp, xp = (yq, xq - 1) if vertical else (yq - 1, xq)
    sq, sp = sl[yq, xq], sl[yp, xp]
    # filterEdgeFlag: slice boundaries only where the q slice allows filtering across
    ok = np.array([bool(slices.get(int(a), (True, 0, 0, False))[0]) for a in sq], bool)
    across = np.array([bool(slices.get(int(a), (True, 0, 0, False))[3]) for a in sq], bool)
    ok &= (sq == sp) | across
    bs = np.where(intra[yq, xq] | intra[yp, xp], 2,
                  np.where(tedge[yq, xq] & (cbf[yq, xq] | cbf[yp, xp]), 1,
                           np.where((np.abs(mv[yq, xq] - mv[yp, xp]) >= 4).any(axis=-1), 1, 0)))
    bs = np.where(ok, bs, 0)
    qpl = (qp[yq, xq] + qp[yp, xp] + 1) >> 1
    beta_off = np.array([slices.get(int(a), (True, 0, 0, False))[1] for a in sq], np.int64)
    tc_off = np.array([slices.get(int(a), (True, 0, 0, False))[2] for a in sq], np.int64)
    sel = bs > 0
    # ---- luma: 4-line segments
    if sel.any():
        yy, xx, b, q, bo, to = yq[sel], xq[sel], bs[sel], qpl[sel], beta_off[sel], tc_off[sel]
        beta = np.array(BETA_TABLE)[np.clip(q + bo, 0, 51)]
        tc = np.array(TC_TABLE)[np.clip(q + 2 * (b - 1) + to, 0, 53)]
        ln = np.arange(4)
        off = np.arange(-4, 4)
        if vertical:
            rows = (yy * 4)[:, None, None] + ln[None, :, None]
            cols = (xx * 4)[:, None, None] + off[None, None, :]
        else:
            rows = (yy * 4)[:, None, None] + off[None, None, :]
            cols = (xx * 4)[:, None, None] + ln[None, :, None]
        blk = Y[rows, cols].astype(np.int64)          # [seg, line, p3 p2 p1 p0 q0 q1 q2 q3]
        p3, p2, p1, p0, q0, q1, q2, q3 = (blk[:, :, k] for k in range(8))
        dp = np.abs(p2 - 2 * p1 + p0)
        dq = np.abs(q2 - 2 * q1 + q0)
        dpq0, dpq3 = dp[:, 0] + dq[:, 0], dp[:, 3] + dq[:, 3]
        on = (dpq0 + dpq3) < beta

        def strong(k, dpq):
            return ((2 * dpq < (beta >> 2)) & (np.abs(p3[:, k] - p0[:, k]) + np.abs(q0[:, k] - q3[:, k]) < (beta >> 3))
                    & (np.abs(p0[:, k] - q0[:, k]) < ((5 * tc + 1) >> 1)))
        de2 = strong(0, dpq0) & strong(3, dpq3)
        side = (beta + (beta >> 1)) >> 3
        dep = (dp[:, 0] + dp[:, 3]) < side
        deq = (dq[:, 0] + dq[:, 3]) < side
        t = tc[:, None]
        out = blk.copy()
        # strong filter
        s2 = (on & de2)[:, None]
        t2 = 2 * t
        new = {
            3: np.clip((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, p0 - t2, p0 + t2),
            2: np.clip((p2 + p1 + p0 + q0 + 2) >> 2, p1 - t2, p1 + t2),
            1: np.clip((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3, p2 - t2, p2 + t2),
            4: np.clip((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, q0 - t2, q0 + t2),
            5: np.clip((p0 + q0 + q1 + q2 + 2) >> 2, q1 - t2, q1 + t2),
            6: np.clip((p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3, q2 - t2, q2 + t2),
        }
        for k, v in new.items():
            out[:, :, k] = np.where(s2, v, out[:, :, k])
        # normal filter
        d = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4
        nrm = (on & ~de2)[:, None] & (np.abs(d) < t * 10)
        d = np.clip(d, -t, t)
        out[:, :, 3] = np.where(nrm, np.clip(p0 + d, 0, 255), out[:, :, 3])
        out[:, :, 4] = np.where(nrm, np.clip(q0 - d, 0, 255), out[:, :, 4])
        th = t >> 1
        dpv = np.clip((((p2 + p0 + 1) >> 1) - p1 + d) >> 1, -th, th)
        dqv = np.clip((((q2 + q0 + 1) >> 1) - q1 - d) >> 1, -th, th)
        out[:, :, 2] = np.where(nrm & dep[:, None], np.clip(p1 + dpv, 0, 255), out[:, :, 2])
        out[:, :, 5] = np.where(nrm & deq[:, None], np.clip(q1 + dqv, 0, 255), out[:, :, 5])
        Y[rows, cols] = out.astype(np.uint8)
    # ---- chroma (4:2:0): bS 2 edges on the 8x8 chroma grid, i.e. every 16 luma samples
    csel = (bs == 2) & (((xq if vertical else yq) % 4) == 0)
    if csel.any():
        yy, xx, q, to = yq[csel], xq[csel], qpl[csel], tc_off[csel]
        ln = np.arange(2)                            # a 4-sample luma segment = 2 chroma lines
        off = np.arange(-2, 2)
        for P, cqoff in ((U, c["cb_off"]), (V, c["cr_off"])):
            tc = np.array(TC_TABLE)[np.clip(np.array([_qpc(int(v) + cqoff) for v in q]) + 2 + to, 0, 53)]
            if vertical:
                rows = (yy * 2)[:, None, None] + ln[None, :, None]
                cols = (xx * 2)[:, None, None] + off[None, None, :]
            else:
                rows = (yy * 2)[:, None, None] + off[None, None, :]
                cols = (xx * 2)[:, None, None] + ln[None, :, None]
            blk = P[rows, cols].astype(np.int64)
            p1, p0, q0, q1 = (blk[:, :, k] for k in range(4))
            t = tc[:, None]
            d = np.clip((((q0 - p0) * 4) + p1 - q1 + 4) >> 3, -t, t)
            blk[:, :, 1] = np.clip(p0 + d, 0, 255)
            blk[:, :, 2] = np.clip(q0 - d, 0, 255)
            P[rows, cols] = blk.astype(np.uint8)


def psnr(a: np.ndarray, b: np.ndarray) -> float:
    d = a.astype(np.float64) - b.astype(np.float64)
    mse = float(np.mean(d * d))
    return 99.0 if mse == 0 else 10 * np.log10(255.0 * 255.0 / mse)
