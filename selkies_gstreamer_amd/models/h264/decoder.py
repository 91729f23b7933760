"""Minimal H.264 Constrained-Baseline (CAVLC) decoder used to verify the encoder.

There is no ffmpeg/PyAV/browser in the build environment, so
bitstream conformance is checked against this independent implementation of
the decoding process of ITU-T H.264 clauses 7 (syntax), 8 (decoding) and 9.2
(CAVLC). It supports exactly what a Baseline stream from our encoder may contain
plus a little more (I_PCM, quarter-pel luma MC), and raises NotImplementedError
for the rest (CABAC, interlace, FMO/ASO, B slices, in-loop deblocking).

Pure Python + numpy; intended for test-sized pictures.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import tables as T


class BitstreamError(ValueError):
    pass


# ---------------------------------------------------------------------------
def split_annexb(data: bytes) -> list[bytes]:
    """Splits an Annex-B byte stream into NAL units (start codes removed)."""
    out = []
    i, n = 0, len(data)
    starts = []
    while i + 2 < n:
        if data[i] == 0 and data[i + 1] == 0 and data[i + 2] == 1:
            starts.append(i + 3)
            i += 3
        else:
            i += 1
    for k, s in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else n
        nal = data[s:e]
        # strip trailing zero bytes (they belong to the next start code / trailing_zero_8bits)
        j = len(nal)
        while j > 0 and nal[j - 1] == 0:
            j -= 1
        out.append(bytes(nal[:j]))
    return out


def unescape(nal_payload: bytes) -> bytes:
    out = bytearray()
    zeros = 0
    for b in nal_payload:
        if zeros >= 2 and b == 3:
            zeros = 0
            continue
        out.append(b)
        zeros = zeros + 1 if b == 0 else 0
    return bytes(out)


class BitReader:
    def __init__(self, data: bytes):
        self.data = data
        self.pos = 0
        self.nbits = len(data) * 8
        # position of the rbsp_stop_one_bit (last 1 bit)
        last = -1
        for i in range(len(data) - 1, -1, -1):
            if data[i]:
                b = data[i]
                k = 0
                while not (b >> k) & 1:
                    k += 1
                last = i * 8 + (7 - k)
                break
        self.stop_bit = last

    def u1(self) -> int:
        if self.pos >= self.nbits:
            raise BitstreamError("read past end of RBSP")
        b = (self.data[self.pos >> 3] >> (7 - (self.pos & 7))) & 1
        self.pos += 1
        return b

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | self.u1()
        return v

    def ue(self) -> int:
        lz = 0
        while self.u1() == 0:
            lz += 1
            if lz > 31:
                raise BitstreamError("invalid exp-golomb code")
        return (1 << lz) - 1 + (self.u(lz) if lz else 0)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)

    def vlc(self, mapping: dict, maxlen: int = 16):
        code = 0
        for length in range(1, maxlen + 1):
            code = (code << 1) | self.u1()
            if (length, code) in mapping:
                return mapping[(length, code)]
        raise BitstreamError("invalid VLC code")

    def more_rbsp_data(self) -> bool:
        return self.pos < self.stop_bit

    def byte_aligned(self) -> bool:
        return (self.pos & 7) == 0


# ---------------------------------------------------------------------------
@dataclass
class SPS:
    profile_idc: int
    constraint_flags: int
    level_idc: int
    log2_max_frame_num: int
    poc_type: int
    log2_max_poc_lsb: int
    max_num_ref_frames: int
    mb_w: int
    mb_h: int
    crop: tuple
    full_range: int = 0
    matrix: int = 2
    max_num_reorder_frames: int = -1

    @property
    def width(self):
        return self.mb_w * 16 - 2 * (self.crop[0] + self.crop[1])

    @property
    def height(self):
        return self.mb_h * 16 - 2 * (self.crop[2] + self.crop[3])


@dataclass
class PPS:
    sps_id: int
    entropy_coding_mode: int
    num_ref_idx_l0: int
    pic_init_qp: int
    chroma_qp_index_offset: int
    deblocking_filter_control_present: int
    constrained_intra_pred: int
    redundant_pic_cnt_present: int


def parse_sps(br: BitReader) -> tuple[int, SPS]:
    profile = br.u(8)
    cflags = br.u(8)
    level = br.u(8)
    sps_id = br.ue()
    if profile in (100, 110, 122, 244, 44, 83, 86, 118, 128, 138, 139, 134, 135):
        raise NotImplementedError("High profiles are not supported by the test decoder")
    log2_mfn = br.ue() + 4
    poc_type = br.ue()
    log2_poc = 0
    if poc_type == 0:
        log2_poc = br.ue() + 4
    elif poc_type == 1:
        br.u1()
        br.se()
        br.se()
        for _ in range(br.ue()):
            br.se()
    max_refs = br.ue()
    br.u1()  # gaps_in_frame_num_value_allowed_flag
    mb_w = br.ue() + 1
    mb_h = br.ue() + 1
    if not br.u1():
        raise NotImplementedError("interlaced streams")
    br.u1()  # direct_8x8_inference_flag
    crop = (0, 0, 0, 0)
    if br.u1():
        crop = (br.ue(), br.ue(), br.ue(), br.ue())
    sps = SPS(profile, cflags, level, log2_mfn, poc_type, log2_poc, max_refs, mb_w, mb_h, crop)
    if br.u1():  # vui
        if br.u1():
            idc = br.u(8)
            if idc == 255:
                br.u(16)
                br.u(16)
        if br.u1():
            br.u1()
        if br.u1():
            br.u(3)
            sps.full_range = br.u1()
            if br.u1():
                br.u(8)
                br.u(8)
                sps.matrix = br.u(8)
        if br.u1():
            br.ue()
            br.ue()
        if br.u1():
            br.u(32)
            br.u(32)
            br.u1()
        nal_hrd = br.u1()
        if nal_hrd:
            raise NotImplementedError("HRD parameters")
        vcl_hrd = br.u1()
        if vcl_hrd:
            raise NotImplementedError("HRD parameters")
        br.u1()  # pic_struct_present_flag
        if br.u1():
            br.u1()
            br.ue()
            br.ue()
            br.ue()
            br.ue()
            sps.max_num_reorder_frames = br.ue()
            br.ue()
    return sps_id, sps


def parse_pps(br: BitReader) -> tuple[int, PPS]:
    pps_id = br.ue()
    sps_id = br.ue()
    entropy = br.u1()
    if entropy:
        raise NotImplementedError("CABAC")
    br.u1()  # bottom_field_pic_order_in_frame_present_flag
    if br.ue() != 0:
        raise NotImplementedError("slice groups (FMO)")
    nref0 = br.ue() + 1
    br.ue()
    if br.u1() or br.u(2):
        raise NotImplementedError("weighted prediction")
    qp = 26 + br.se()
    br.se()
    cqo = br.se()
    dfc = br.u1()
    cip = br.u1()
    rpc = br.u1()
    return pps_id, PPS(sps_id, entropy, nref0, qp, cqo, dfc, cip, rpc)


# ---------------------------------------------------------------------------
def _idct4(d: np.ndarray) -> np.ndarray:
    """Inverse core transform of a 4x4 int array (rows, then columns), (x+32)>>6."""
    d = d.astype(np.int64)
    e0 = d[:, 0] + d[:, 2]
    e1 = d[:, 0] - d[:, 2]
    e2 = (d[:, 1] >> 1) - d[:, 3]
    e3 = d[:, 1] + (d[:, 3] >> 1)
    f = np.stack([e0 + e3, e1 + e2, e1 - e2, e0 - e3], axis=1)
    g0 = f[0] + f[2]
    g1 = f[0] - f[2]
    g2 = (f[1] >> 1) - f[3]
    g3 = f[1] + (f[3] >> 1)
    h = np.stack([g0 + g3, g1 + g2, g1 - g2, g0 - g3], axis=0)
    return (h + 32) >> 6


_H4 = np.array([[1, 1, 1, 1], [1, 1, -1, -1], [1, -1, -1, 1], [1, -1, 1, -1]], dtype=np.int64)


def _levelscale(qp_mod: int, r: int) -> int:
    return 16 * T.DEQUANT_V[qp_mod][T.POS_CLASS[r]]


def _scale_4x4(c: np.ndarray, qp: int, skip_dc: bool) -> np.ndarray:
    """8.5.12.1 with flat weight matrices; c is a 4x4 raster array of levels."""
    d = np.zeros((4, 4), dtype=np.int64)
    for i in range(4):
        for j in range(4):
            if skip_dc and i == 0 and j == 0:
                continue
            ls = _levelscale(qp % 6, i * 4 + j)
            if qp >= 24:
                d[i, j] = (int(c[i, j]) * ls) << (qp // 6 - 4)
            else:
                d[i, j] = (int(c[i, j]) * ls + (1 << (3 - qp // 6))) >> (4 - qp // 6)
    return d


def _unzigzag(levels) -> np.ndarray:
    c = np.zeros(16, dtype=np.int64)
    for k, v in enumerate(levels):
        c[T.ZIGZAG[k]] = v
    return c.reshape(4, 4)


def _clip1(x):
    return np.clip(x, 0, 255)


# ---------------------------------------------------------------------------
# deblocking tables (8.7.2.2: Tables 8-16, 8-17)
_DB_ALPHA = np.array([0] * 16 + [4, 4, 5, 6, 7, 8, 9, 10, 12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63,
                                 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255])
_DB_BETA = np.array([0] * 16 + [2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13,
                                13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18])
_DB_TC0 = np.array([[0, 0, 0]] * 17 + [[0, 0, 1]] * 4 + [[0, 1, 1]] * 2 + [[1, 1, 1]] * 4 + [[1, 1, 2]] * 4 +
                   [[1, 2, 3]] * 2 + [[2, 2, 3], [2, 2, 4], [2, 3, 4], [2, 3, 4], [3, 3, 5], [3, 4, 6], [3, 4, 6],
                                      [4, 5, 7], [4, 5, 8], [4, 6, 9], [5, 7, 10], [6, 8, 11], [6, 8, 13],
                                      [7, 10, 14], [8, 11, 16], [9, 12, 18], [10, 13, 20], [11, 15, 23],
                                      [13, 17, 25]])


def _db_qp(m) -> int:
    return 0 if m.pcm else m.qp


def _db_bs(p, q, e: int, j: int, vertical: bool) -> int:
    """bS (8.7.2.1) of segment j of luma edge e between MB p (left/top, or q itself for e > 0) and q."""
    pe = 3 if e == 0 else e - 1
    pb, qb = (j * 4 + pe, j * 4 + e) if vertical else (pe * 4 + j, e * 4 + j)
    if p.intra or q.intra:
        return 4 if e == 0 else 3
    if p.tc_luma[pb] or q.tc_luma[qb]:
        return 2
    if p.ref[pb] != q.ref[qb] or abs(int(p.mvx[pb]) - int(q.mvx[qb])) >= 4 or abs(int(p.mvy[pb]) - int(q.mvy[qb])) >= 4:
        return 1
    return 0


def _db_filter(L: np.ndarray, bs: np.ndarray, qpav: int, fa: int, fb: int, chroma: bool) -> np.ndarray:
    """Filters the lines of one edge. L: (n, 8) = p3..q3 (luma) or (n, 4) = p1 p0 q0 q1 (chroma)."""
    ia, ib = min(51, max(0, qpav + fa)), min(51, max(0, qpav + fb))
    alpha, beta = int(_DB_ALPHA[ia]), int(_DB_BETA[ib])
    out = L.copy()
    o = 2 if chroma else 0
    p1, p0, q0, q1 = L[:, 2 - o], L[:, 3 - o], L[:, 4 - o], L[:, 5 - o]
    on = (bs > 0) & (np.abs(p0 - q0) < alpha) & (np.abs(p1 - p0) < beta) & (np.abs(q1 - q0) < beta)
    tc0 = _DB_TC0[ia][np.clip(bs - 1, 0, 2)]
    weak, strong4 = on & (bs < 4), on & (bs == 4)
    if chroma:
        tc = tc0 + 1
        d = np.clip((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc)
        out[weak, 1] = np.clip(p0 + d, 0, 255)[weak]
        out[weak, 2] = np.clip(q0 - d, 0, 255)[weak]
        out[strong4, 1] = ((2 * p1 + p0 + q1 + 2) >> 2)[strong4]
        out[strong4, 2] = ((2 * q1 + q0 + p1 + 2) >> 2)[strong4]
        return out
    p3, p2, q2, q3 = L[:, 0], L[:, 1], L[:, 6], L[:, 7]
    ap, aq = np.abs(p2 - p0) < beta, np.abs(q2 - q0) < beta
    tc = tc0 + ap + aq
    d = np.clip((((q0 - p0) << 2) + (p1 - q1) + 4) >> 3, -tc, tc)
    out[weak, 3] = np.clip(p0 + d, 0, 255)[weak]
    out[weak, 4] = np.clip(q0 - d, 0, 255)[weak]
    m = weak & ap
    out[m, 2] = (p1 + np.clip((p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1, -tc0, tc0))[m]
    m = weak & aq
    out[m, 5] = (q1 + np.clip((q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1, -tc0, tc0))[m]
    small = np.abs(p0 - q0) < ((alpha >> 2) + 2)
    sp, sq = strong4 & ap & small, strong4 & aq & small
    out[sp, 3] = ((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3)[sp]
    out[sp, 2] = ((p2 + p1 + p0 + q0 + 2) >> 2)[sp]
    out[sp, 1] = ((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3)[sp]
    wp = strong4 & ~(ap & small)
    out[wp, 3] = ((2 * p1 + p0 + q1 + 2) >> 2)[wp]
    out[sq, 4] = ((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3)[sq]
    out[sq, 5] = ((p0 + q0 + q1 + q2 + 2) >> 2)[sq]
    out[sq, 6] = ((2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3)[sq]
    wq = strong4 & ~(aq & small)
    out[wq, 4] = ((2 * q1 + q0 + p1 + 2) >> 2)[wq]
    return out


# ---------------------------------------------------------------------------
@dataclass
class MbState:
    avail: bool = False
    slice_id: int = -1
    intra: bool = False
    skip: bool = False
    pcm: bool = False
    qp: int = 0
    mvx: np.ndarray = field(default_factory=lambda: np.zeros(16, dtype=np.int64))  # per 4x4 (blkIdx raster y*4+x)
    mvy: np.ndarray = field(default_factory=lambda: np.zeros(16, dtype=np.int64))
    ref: np.ndarray = field(default_factory=lambda: np.full(16, -1, dtype=np.int64))
    tc_luma: np.ndarray = field(default_factory=lambda: np.zeros(16, dtype=np.int64))  # raster y*4+x
    tc_chroma: np.ndarray = field(default_factory=lambda: np.zeros((2, 4), dtype=np.int64))  # raster 2x2
    i4: bool = False         # coded as Intra_4x4 (I_NxN)
    i4_modes: np.ndarray = field(default_factory=lambda: np.full(16, 2, dtype=np.int64))  # raster y*4+x
    db: tuple = (1, 0, 0)  # (disable_deblocking_filter_idc, FilterOffsetA, FilterOffsetB) of its slice


class H264Decoder:
    """Decodes an Annex-B stream; `decode(data)` returns a list of decoded frames
    as (Y, U, V) uint8 arrays cropped to the SPS display size."""

    def __init__(self):
        self.sps: dict[int, SPS] = {}
        self.pps: dict[int, PPS] = {}
        self.dpb: list = []      # short-term reference pictures (Y, U, V), most recent first (8.2.4.2.1)
        self.cur_ref_idc = 0
        self.cur_idr = False
        self.cur = None
        self.mbs: list[MbState] = []
        self.cur_sps: SPS | None = None
        self.cur_frame_num = None
        self.frames: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []
        self.slice_counter = 0
        self.stats = {"slices": 0, "idr": 0, "skip": 0, "i16": 0, "p16": 0, "pcm": 0, "i4": 0}

    # -------------------------------------------------------------------
    def decode(self, data: bytes):
        out_start = len(self.frames)
        for nal in split_annexb(data):
            self.decode_nal(nal)
        self.flush()
        return self.frames[out_start:]

    def decode_nal(self, nal: bytes):
        if not nal:
            return
        hdr = nal[0]
        if hdr & 0x80:
            raise BitstreamError("forbidden_zero_bit set")
        ref_idc = (hdr >> 5) & 3
        ntype = hdr & 31
        br = BitReader(unescape(nal[1:]))
        if ntype == 7:
            i, s = parse_sps(br)
            self.sps[i] = s
        elif ntype == 8:
            i, p = parse_pps(br)
            self.pps[i] = p
        elif ntype in (1, 5):
            self.decode_slice(br, ntype == 5, ref_idc)
        elif ntype in (6, 9, 10, 11, 12):
            pass  # SEI, AUD, end of seq/stream, filler
        else:
            raise NotImplementedError(f"nal_unit_type {ntype}")

    def flush(self):
        if self.cur is not None:
            self._finish_picture()

    def _finish_picture(self):
        self._deblock_picture()
        sps = self.cur_sps
        y, u, v = self.cur
        cl, cr, ct, cb = sps.crop
        W, H = sps.width, sps.height
        x0, y0 = 2 * cl, 2 * ct
        self.frames.append((y[y0:y0 + H, x0:x0 + W].copy(), u[y0 // 2:(y0 + H) // 2, x0 // 2:(x0 + W) // 2].copy(),
                            v[y0 // 2:(y0 + H) // 2, x0 // 2:(x0 + W) // 2].copy()))
        if self.cur_ref_idc:   # sliding-window marking (8.2.5.3); IDR empties the DPB first
            pic = (y.copy(), u.copy(), v.copy())
            self.dpb = [pic] if self.cur_idr else [pic] + self.dpb
            del self.dpb[max(1, sps.max_num_ref_frames):]
        self.cur = None

    # -------------------------------------------------------------------
    def decode_slice(self, br: BitReader, idr: bool, ref_idc: int):
        first_mb = br.ue()
        slice_type = br.ue() % 5
        pps = self.pps[br.ue()]
        sps = self.sps[pps.sps_id]
        frame_num = br.u(sps.log2_max_frame_num)
        if idr:
            br.ue()  # idr_pic_id
        if sps.poc_type == 0:
            br.u(sps.log2_max_poc_lsb)
        if pps.redundant_pic_cnt_present:
            br.ue()
        if slice_type not in (0, 2):
            raise NotImplementedError(f"slice_type {slice_type}")
        num_ref = pps.num_ref_idx_l0
        if slice_type == 0:
            if br.u1():
                num_ref = br.ue() + 1
            if br.u1():
                raise NotImplementedError("ref_pic_list_modification")
        if ref_idc:
            if idr:
                br.u1()
                br.u1()
            elif br.u1():
                raise NotImplementedError("adaptive_ref_pic_marking")
        qp = pps.pic_init_qp + br.se()
        db = (0, 0, 0)
        if pps.deblocking_filter_control_present:
            dis = br.ue()
            if dis > 2:
                raise BitstreamError("disable_deblocking_filter_idc out of range")
            db = (dis, 0, 0) if dis == 1 else (dis, 2 * br.se(), 2 * br.se())
        self._db_params = db

        new_picture = self.cur is None or first_mb == 0 or frame_num != self.cur_frame_num
        if new_picture and self.cur is not None:
            self._finish_picture()
        if self.cur is None:
            self.cur_sps = sps
            self.cur_frame_num = frame_num
            self.cur_ref_idc = ref_idc
            self.cur_idr = idr
            self.cur = (np.zeros((sps.mb_h * 16, sps.mb_w * 16), np.uint8),
                        np.zeros((sps.mb_h * 8, sps.mb_w * 8), np.uint8),
                        np.zeros((sps.mb_h * 8, sps.mb_w * 8), np.uint8))
            self.mbs = [MbState() for _ in range(sps.mb_w * sps.mb_h)]
            if idr:
                self.stats["idr"] += 1
        if slice_type == 0 and not self.dpb:
            raise BitstreamError("P slice without a reference picture")
        self.slice_counter += 1
        self.stats["slices"] += 1
        self.cur_pps = pps
        self._slice_data(br, sps, pps, first_mb, slice_type, qp, num_ref)

    # -------------------------------------------------------------------
    def _slice_data(self, br, sps, pps, first_mb, slice_type, qp, num_ref):
        sid = self.slice_counter
        mb_addr = first_mb
        nmb = sps.mb_w * sps.mb_h
        more = True
        self.qp = qp
        while more:
            if slice_type == 0:
                run = br.ue()
                for _ in range(run):
                    if mb_addr >= nmb:
                        raise BitstreamError("mb_skip_run past end of picture")
                    self._decode_skip(sps, mb_addr, sid)
                    self.mbs[mb_addr].db = self._db_params
                    mb_addr += 1
                if run > 0:
                    more = br.more_rbsp_data()
                    if not more:
                        break
            if mb_addr >= nmb:
                raise BitstreamError("macroblock address past end of picture")
            self._macroblock(br, sps, pps, mb_addr, sid, slice_type, num_ref)
            self.mbs[mb_addr].db = self._db_params
            mb_addr += 1
            more = br.more_rbsp_data()

    # ---- in-loop deblocking (8.7) ----------------------------------------------
    def _deblock_picture(self):
        """Filters the finished picture in macroblock raster order: per MB the luma vertical
        edges left to right, the luma horizontal edges top to bottom, then the same for Cb
        and Cr. Each edge is filtered for all its lines at once (lines are independent)."""
        sps, pps = self.cur_sps, getattr(self, "cur_pps", None)
        if pps is None:
            return
        Y, U, V = self.cur
        mbw = sps.mb_w
        coff = pps.chroma_qp_index_offset
        for addr, cur in enumerate(self.mbs):
            if not cur.avail or cur.db[0] == 1:
                continue
            mbx, mby = addr % mbw, addr // mbw
            left = self._db_neighbour(cur, addr - 1) if mbx > 0 else None
            top = self._db_neighbour(cur, addr - mbw) if mby > 0 else None
            _, fa, fb = cur.db
            for vertical, nb in ((True, left), (False, top)):
                for e in range(4):
                    p = nb if e == 0 else cur
                    if p is None:
                        continue
                    bs = np.repeat([_db_bs(p, cur, e, j, vertical) for j in range(4)], 4)
                    if not bs.any():
                        continue
                    qpav = (_db_qp(p) + _db_qp(cur) + 1) >> 1
                    x0, y0 = mbx * 16, mby * 16
                    seg = (Y[y0:y0 + 16, x0 + 4 * e - 4:x0 + 4 * e + 4] if vertical
                           else Y[y0 + 4 * e - 4:y0 + 4 * e + 4, x0:x0 + 16].T)
                    seg[...] = _db_filter(seg.astype(np.int64), bs, qpav, fa, fb, chroma=False)
            for P in (U, V):
                for vertical, nb in ((True, left), (False, top)):
                    for e in range(2):
                        p = nb if e == 0 else cur
                        if p is None:
                            continue
                        bs = np.repeat([_db_bs(p, cur, 2 * e, j, vertical) for j in range(4)], 2)
                        if not bs.any():
                            continue
                        qpc = lambda m: T.CHROMA_QP[min(51, max(0, _db_qp(m) + coff))]  # noqa: E731
                        qpav = (qpc(p) + qpc(cur) + 1) >> 1
                        x0, y0 = mbx * 8, mby * 8
                        seg = (P[y0:y0 + 8, x0 + 4 * e - 2:x0 + 4 * e + 2] if vertical
                               else P[y0 + 4 * e - 2:y0 + 4 * e + 2, x0:x0 + 8].T)
                        seg[...] = _db_filter(seg.astype(np.int64), bs, qpav, fa, fb, chroma=True)

    def _db_neighbour(self, cur, addr):
        m = self.mbs[addr]
        if not m.avail or (cur.db[0] == 2 and m.slice_id != cur.slice_id):
            return None
        return m

    # ---- neighbour helpers ----------------------------------------------
    def _mb(self, sps, mbx, mby, sid):
        if mbx < 0 or mby < 0 or mbx >= sps.mb_w or mby >= sps.mb_h:
            return None
        m = self.mbs[mby * sps.mb_w + mbx]
        if not m.avail or m.slice_id != sid:
            return None
        return m

    def _nb4(self, sps, mbx, mby, x4, y4, sid):
        """Neighbouring 4x4 luma position (x4,y4 relative to the MB, may be -1 or 4)."""
        ox = mbx + (x4 >> 2) if x4 >= 0 else mbx - 1
        oy = mby + (y4 >> 2) if y4 >= 0 else mby - 1
        m = self._mb(sps, ox, oy, sid)
        return m, (x4 & 3), (y4 & 3)

    def _total_coeff_luma(self, cur, sps, mbx, mby, bx, by, sid):
        def get(x, y):
            if 0 <= x < 4 and 0 <= y < 4:
                return True, int(cur.tc_luma[y * 4 + x])
            m, xx, yy = self._nb4(sps, mbx, mby, x, y, sid)
            if m is None:
                return False, 0
            if m.pcm:
                return True, 16
            return True, int(m.tc_luma[yy * 4 + xx])
        aA, nA = get(bx - 1, by)
        aB, nB = get(bx, by - 1)
        return self._nc(aA, nA, aB, nB)

    def _total_coeff_chroma(self, cur, sps, mbx, mby, comp, bx, by, sid):
        def get(x, y):
            if 0 <= x < 2 and 0 <= y < 2:
                return True, int(cur.tc_chroma[comp, y * 2 + x])
            ox = mbx - 1 if x < 0 else mbx
            oy = mby - 1 if y < 0 else mby
            m = self._mb(sps, ox, oy, sid)
            if m is None:
                return False, 0
            if m.pcm:
                return True, 16
            return True, int(m.tc_chroma[comp, (y & 1) * 2 + (x & 1)])
        aA, nA = get(bx - 1, by)
        aB, nB = get(bx, by - 1)
        return self._nc(aA, nA, aB, nB)

    @staticmethod
    def _nc(aA, nA, aB, nB):
        if aA and aB:
            return (nA + nB + 1) >> 1
        if aA:
            return nA
        if aB:
            return nB
        return 0

    # ---- CAVLC residual_block (9.2) ---------------------------------------
    @staticmethod
    def residual_block(br: BitReader, nC: int, max_num: int):
        if nC == -1:
            tc, t1 = br.vlc(T.coeff_token_map(-1))
        else:
            vlc = 0 if nC < 2 else 1 if nC < 4 else 2 if nC < 8 else 3
            if vlc == 3:
                code = br.u(6)
                mp = T.coeff_token_map(3)
                if (6, code) not in mp:
                    raise BitstreamError("invalid FLC coeff_token")
                tc, t1 = mp[(6, code)]
            else:
                tc, t1 = br.vlc(T.coeff_token_map(vlc))
        coeff = [0] * max_num
        if tc == 0:
            return coeff, 0
        if tc > max_num:
            raise BitstreamError("TotalCoeff exceeds maxNumCoeff")
        suffix_len = 1 if (tc > 10 and t1 < 3) else 0
        levels = []
        for i in range(tc):
            if i < t1:
                levels.append(-1 if br.u1() else 1)
                continue
            prefix = 0
            while br.u1() == 0:
                prefix += 1
                if prefix > 32:
                    raise BitstreamError("level_prefix too long")
            if prefix == 14 and suffix_len == 0:
                ssize = 4
            elif prefix >= 15:
                ssize = prefix - 3
            else:
                ssize = suffix_len
            level_code = (min(15, prefix) << suffix_len) + (br.u(ssize) if ssize > 0 else 0)
            if prefix >= 15 and suffix_len == 0:
                level_code += 15
            if prefix >= 16:
                level_code += (1 << (prefix - 3)) - 4096
            if i == t1 and t1 < 3:
                level_code += 2
            lv = (level_code + 2) >> 1 if level_code % 2 == 0 else (-level_code - 1) >> 1
            levels.append(lv)
            if suffix_len == 0:
                suffix_len = 1
            if abs(lv) > (3 << (suffix_len - 1)) and suffix_len < 6:
                suffix_len += 1
        if tc < max_num:
            total_zeros = br.vlc(T.total_zeros_map(tc, max_num == 4))
        else:
            total_zeros = 0
        zeros_left = total_zeros
        runs = []
        for i in range(tc - 1):
            if zeros_left > 0:
                r = br.vlc(T.run_before_map(zeros_left))
            else:
                r = 0
            runs.append(r)
            zeros_left -= r
        if zeros_left < 0:
            raise BitstreamError("run_before exceeds total_zeros")
        runs.append(zeros_left)
        pos = -1
        for i in range(tc - 1, -1, -1):
            pos += runs[i] + 1
            if pos >= max_num:
                raise BitstreamError("coefficient index overflow")
            coeff[pos] = levels[i]
        return coeff, tc

    # ---- macroblock layer ---------------------------------------------------
    def _macroblock(self, br, sps, pps, addr, sid, slice_type, num_ref):
        mbx, mby = addr % sps.mb_w, addr // sps.mb_w
        cur = self.mbs[addr]
        cur.__init__()
        cur.slice_id = sid
        mb_type = br.ue()
        if slice_type == 0:
            if mb_type < 5:
                if mb_type != 0:
                    raise NotImplementedError("P partitions other than 16x16")
                self._decode_p16(br, sps, pps, cur, mbx, mby, sid, num_ref)
                cur.avail = True
                return
            mb_type -= 5
        if mb_type == 25:
            self._decode_pcm(br, sps, cur, mbx, mby)
        elif mb_type == 0:
            self._decode_i4(br, sps, pps, cur, mbx, mby, sid)
        elif 1 <= mb_type <= 24:
            self._decode_i16(br, sps, pps, cur, mbx, mby, sid, mb_type)
        else:
            raise BitstreamError(f"mb_type {mb_type}")
        cur.avail = True

    def _read_qp_delta(self, br):
        dq = br.se()
        if dq < -26 or dq > 25:
            raise BitstreamError("mb_qp_delta out of range")
        self.qp = (self.qp + dq + 52) % 52

    def _chroma_residual(self, br, sps, pps, cur, mbx, mby, sid, cbp_c):
        dc = [[0] * 4, [0] * 4]
        ac = [[[0] * 15 for _ in range(4)] for _ in range(2)]
        if cbp_c & 3:
            for c in range(2):
                dc[c], _ = self.residual_block(br, -1, 4)
        if cbp_c & 2:
            for c in range(2):
                for b in range(4):
                    nc = self._total_coeff_chroma(cur, sps, mbx, mby, c, b & 1, b >> 1, sid)
                    ac[c][b], tc = self.residual_block(br, nc, 15)
                    cur.tc_chroma[c, b] = tc
        return dc, ac

    def _recon_chroma(self, sps, pps, cur, mbx, mby, dc, ac, pred_u, pred_v):
        qpc = T.CHROMA_QP[min(51, max(0, cur.qp + pps.chroma_qp_index_offset))]
        for c, pred in enumerate((pred_u, pred_v)):
            cm = np.array(dc[c], dtype=np.int64).reshape(2, 2)
            f = np.array([[1, 1], [1, -1]]) @ cm @ np.array([[1, 1], [1, -1]])
            ls = 16 * T.DEQUANT_V[qpc % 6][0]
            dcc = ((f * ls) << (qpc // 6)) >> 5
            plane = self.cur[1 + c]
            for b in range(4):
                bx, by = b & 1, b >> 1
                c4 = _unzigzag([0] + list(ac[c][b]))
                d = _scale_4x4(c4, qpc, skip_dc=True)
                d[0, 0] = dcc[by, bx]
                r = _idct4(d)
                p = pred[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4].astype(np.int64)
                plane[mby * 8 + by * 4:mby * 8 + by * 4 + 4, mbx * 8 + bx * 4:mbx * 8 + bx * 4 + 4] = _clip1(p + r)

    # ---- intra ----------------------------------------------------------------
    def _intra_neighbours(self, sps, pps, plane, mbx, mby, sid, size):
        A = self._mb(sps, mbx - 1, mby, sid)
        B = self._mb(sps, mbx, mby - 1, sid)
        D = self._mb(sps, mbx - 1, mby - 1, sid)
        if pps.constrained_intra_pred:
            A = A if (A and A.intra) else None
            B = B if (B and B.intra) else None
            D = D if (D and D.intra) else None
        x0, y0 = mbx * size, mby * size
        top = plane[y0 - 1, x0:x0 + size].astype(np.int64) if B else None
        left = plane[y0:y0 + size, x0 - 1].astype(np.int64) if A else None
        tl = int(plane[y0 - 1, x0 - 1]) if D else None
        return top, left, tl

    def _pred_i16(self, mode, top, left, tl):
        if mode == 0:
            if top is None:
                raise BitstreamError("I16 vertical without top")
            return np.tile(top, (16, 1))
        if mode == 1:
            if left is None:
                raise BitstreamError("I16 horizontal without left")
            return np.tile(left[:, None], (1, 16))
        if mode == 2:
            if top is not None and left is not None:
                v = (int(top.sum()) + int(left.sum()) + 16) >> 5
            elif left is not None:
                v = (int(left.sum()) + 8) >> 4
            elif top is not None:
                v = (int(top.sum()) + 8) >> 4
            else:
                v = 128
            return np.full((16, 16), v, dtype=np.int64)
        if mode == 3:
            if top is None or left is None or tl is None:
                raise BitstreamError("I16 plane without neighbours")
            H = sum((x + 1) * (int(top[8 + x]) - (int(top[6 - x]) if 6 - x >= 0 else tl)) for x in range(8))
            V = sum((y + 1) * (int(left[8 + y]) - (int(left[6 - y]) if 6 - y >= 0 else tl)) for y in range(8))
            a = 16 * (int(left[15]) + int(top[15]))
            b = (5 * H + 32) >> 6
            c = (5 * V + 32) >> 6
            yy, xx = np.mgrid[0:16, 0:16]
            return _clip1((a + b * (xx - 7) + c * (yy - 7) + 16) >> 5)
        raise BitstreamError("bad I16 mode")

    def _pred_chroma(self, mode, top, left, tl):
        if mode == 0:
            out = np.zeros((8, 8), dtype=np.int64)
            for by in range(2):
                for bx in range(2):
                    st = int(top[bx * 4:bx * 4 + 4].sum()) if top is not None else None
                    sl = int(left[by * 4:by * 4 + 4].sum()) if left is not None else None
                    if (bx, by) in ((0, 0), (1, 1)):
                        if st is not None and sl is not None:
                            v = (st + sl + 4) >> 3
                        elif sl is not None:
                            v = (sl + 2) >> 2
                        elif st is not None:
                            v = (st + 2) >> 2
                        else:
                            v = 128
                    elif (bx, by) == (1, 0):
                        v = (st + 2) >> 2 if st is not None else ((sl + 2) >> 2 if sl is not None else 128)
                    else:
                        v = (sl + 2) >> 2 if sl is not None else ((st + 2) >> 2 if st is not None else 128)
                    out[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4] = v
            return out
        if mode == 1:
            if left is None:
                raise BitstreamError("chroma horizontal without left")
            return np.tile(left[:, None], (1, 8))
        if mode == 2:
            if top is None:
                raise BitstreamError("chroma vertical without top")
            return np.tile(top, (8, 1))
        if mode == 3:
            if top is None or left is None or tl is None:
                raise BitstreamError("chroma plane without neighbours")
            H = sum((x + 1) * (int(top[4 + x]) - (int(top[2 - x]) if 2 - x >= 0 else tl)) for x in range(4))
            V = sum((y + 1) * (int(left[4 + y]) - (int(left[2 - y]) if 2 - y >= 0 else tl)) for y in range(4))
            a = 16 * (int(left[7]) + int(top[7]))
            b = (34 * H + 32) >> 6
            c = (34 * V + 32) >> 6
            yy, xx = np.mgrid[0:8, 0:8]
            return _clip1((a + b * (xx - 3) + c * (yy - 3) + 16) >> 5)
        raise BitstreamError("bad chroma mode")

    def _decode_i16(self, br, sps, pps, cur, mbx, mby, sid, mb_type):
        self.stats["i16"] += 1
        t = mb_type - 1
        pred_mode = t % 4
        cbp_c = (t // 4) % 3
        cbp_l = 15 if t >= 12 else 0
        cur.intra = True
        chroma_mode = br.ue()
        self._read_qp_delta(br)
        cur.qp = self.qp
        # residual
        nc0 = self._total_coeff_luma(cur, sps, mbx, mby, 0, 0, sid)
        dc_levels, _ = self.residual_block(br, nc0, 16)
        ac = [[0] * 15 for _ in range(16)]
        if cbp_l:
            for blk in range(16):
                bx, by = T.BLK_X[blk], T.BLK_Y[blk]
                nc = self._total_coeff_luma(cur, sps, mbx, mby, bx, by, sid)
                ac[blk], tc = self.residual_block(br, nc, 15)
                cur.tc_luma[by * 4 + bx] = tc
        dc, acc = self._chroma_residual(br, sps, pps, cur, mbx, mby, sid, cbp_c)
        # reconstruction
        Y = self.cur[0]
        top, left, tl = self._intra_neighbours(sps, pps, Y, mbx, mby, sid, 16)
        pred = self._pred_i16(pred_mode, top, left, tl)
        qp = cur.qp
        c = _unzigzag(dc_levels)
        f = _H4 @ c @ _H4
        ls = 16 * T.DEQUANT_V[qp % 6][0]
        if qp >= 36:
            dcy = (f * ls) << (qp // 6 - 6)
        else:
            dcy = (f * ls + (1 << (5 - qp // 6))) >> (6 - qp // 6)
        for blk in range(16):
            bx, by = T.BLK_X[blk], T.BLK_Y[blk]
            c4 = _unzigzag([0] + list(ac[blk]))
            d = _scale_4x4(c4, qp, skip_dc=True)
            d[0, 0] = dcy[by, bx]
            r = _idct4(d)
            p = pred[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4]
            Y[mby * 16 + by * 4:mby * 16 + by * 4 + 4, mbx * 16 + bx * 4:mbx * 16 + bx * 4 + 4] = _clip1(p + r)
        pu = self._pred_chroma(chroma_mode, *self._intra_neighbours(sps, pps, self.cur[1], mbx, mby, sid, 8))
        pv = self._pred_chroma(chroma_mode, *self._intra_neighbours(sps, pps, self.cur[2], mbx, mby, sid, 8))
        self._recon_chroma(sps, pps, cur, mbx, mby, dc, acc, pu, pv)

    # ---- Intra_4x4 (8.3.1) ------------------------------------------------------
    def _i4_nb_mode(self, sps, cur, mbx, mby, x4, y4, sid):
        """intraMxMPredModeN of the 4x4 block at MB-relative (x4, y4); None if unavailable."""
        if 0 <= x4 < 4 and 0 <= y4 < 4:
            return int(cur.i4_modes[y4 * 4 + x4])
        m, xx, yy = self._nb4(sps, mbx, mby, x4, y4, sid)
        if m is None:
            return None
        return int(m.i4_modes[yy * 4 + xx]) if m.i4 else 2

    def _i4_samples(self, sps, Y, mbx, mby, bx, by, sid):
        """p[x, -1] for x = -1..7 and p[-1, y] for y = 0..3 of block (bx, by) (None where
        not available for Intra_4x4 prediction, p[4..7, -1] already substituted)."""
        x0, y0 = mbx * 16 + bx * 4, mby * 16 + by * 4

        def decoded(x4, y4):   # neighbouring 4x4 block (MB-relative, may be outside) already decoded?
            if 0 <= x4 < 4 and 0 <= y4 < 4:
                order = [(T.BLK_X[k], T.BLK_Y[k]) for k in range(16)]
                return order.index((x4, y4)) < order.index((bx, by))
            if x4 >= 4 and y4 >= 0:
                return False   # macroblock to the right: not decoded yet
            m, _, _ = self._nb4(sps, mbx, mby, x4, y4, sid)
            return m is not None
        top = [None] * 9   # index x + 1, x = -1..7
        left = [None] * 4
        if decoded(bx, by - 1):
            for x in range(4):
                top[x + 1] = int(Y[y0 - 1, x0 + x])
            if decoded(bx + 1, by - 1):
                for x in range(4, 8):
                    top[x + 1] = int(Y[y0 - 1, x0 + x])
            else:
                for x in range(4, 8):
                    top[x + 1] = top[4]
        if decoded(bx - 1, by):
            for y in range(4):
                left[y] = int(Y[y0 + y, x0 - 1])
        if decoded(bx - 1, by - 1):
            top[0] = int(Y[y0 - 1, x0 - 1])
        return top, left

    def _pred_i4(self, mode, top, left):
        P = np.zeros((4, 4), np.int64)
        t = lambda x: top[x + 1]           # p[x, -1], x = -1..7
        l = lambda y: top[0] if y < 0 else left[y]   # p[-1, y], y = -1..3
        need_t = mode in (0, 3, 4, 5, 6, 7)
        need_l = mode in (1, 4, 5, 6, 8)
        if (need_t and top[1] is None) or (need_l and left[0] is None) or (mode in (4, 5, 6) and top[0] is None):
            raise BitstreamError(f"Intra4x4 mode {mode} without its neighbours")
        for y in range(4):
            for x in range(4):
                if mode == 0:
                    v = t(x)
                elif mode == 1:
                    v = l(y)
                elif mode == 2:
                    ht, hl = top[1] is not None, left[0] is not None
                    if ht and hl:
                        v = (sum(t(i) for i in range(4)) + sum(l(i) for i in range(4)) + 4) >> 3
                    elif hl:
                        v = (sum(l(i) for i in range(4)) + 2) >> 2
                    elif ht:
                        v = (sum(t(i) for i in range(4)) + 2) >> 2
                    else:
                        v = 128
                elif mode == 3:   # Diagonal_Down_Left
                    v = (t(6) + 3 * t(7) + 2) >> 2 if x == 3 and y == 3 else (t(x + y) + 2 * t(x + y + 1) + t(x + y + 2) + 2) >> 2
                elif mode == 4:   # Diagonal_Down_Right
                    if x > y:
                        v = (t(x - y - 2) + 2 * t(x - y - 1) + t(x - y) + 2) >> 2
                    elif x < y:
                        v = (l(y - x - 2) + 2 * l(y - x - 1) + l(y - x) + 2) >> 2
                    else:
                        v = (t(0) + 2 * t(-1) + l(0) + 2) >> 2
                elif mode == 5:   # Vertical_Right
                    z = 2 * x - y
                    if z in (0, 2, 4, 6):
                        v = (t(x - (y >> 1) - 1) + t(x - (y >> 1)) + 1) >> 1
                    elif z in (1, 3, 5):
                        v = (t(x - (y >> 1) - 2) + 2 * t(x - (y >> 1) - 1) + t(x - (y >> 1)) + 2) >> 2
                    elif z == -1:
                        v = (l(0) + 2 * l(-1) + t(0) + 2) >> 2
                    else:
                        v = (l(y - 1) + 2 * l(y - 2) + l(y - 3) + 2) >> 2
                elif mode == 6:   # Horizontal_Down
                    z = 2 * y - x
                    if z in (0, 2, 4, 6):
                        v = (l(y - (x >> 1) - 1) + l(y - (x >> 1)) + 1) >> 1
                    elif z in (1, 3, 5):
                        v = (l(y - (x >> 1) - 2) + 2 * l(y - (x >> 1) - 1) + l(y - (x >> 1)) + 2) >> 2
                    elif z == -1:
                        v = (l(0) + 2 * l(-1) + t(0) + 2) >> 2
                    else:
                        v = (t(x - 1) + 2 * t(x - 2) + t(x - 3) + 2) >> 2
                elif mode == 7:   # Vertical_Left
                    if y in (0, 2):
                        v = (t(x + (y >> 1)) + t(x + (y >> 1) + 1) + 1) >> 1
                    else:
                        v = (t(x + (y >> 1)) + 2 * t(x + (y >> 1) + 1) + t(x + (y >> 1) + 2) + 2) >> 2
                elif mode == 8:   # Horizontal_Up
                    z = x + 2 * y
                    if z in (0, 2, 4):
                        v = (l(y + (x >> 1)) + l(y + (x >> 1) + 1) + 1) >> 1
                    elif z in (1, 3):
                        v = (l(y + (x >> 1)) + 2 * l(y + (x >> 1) + 1) + l(y + (x >> 1) + 2) + 2) >> 2
                    elif z == 5:
                        v = (l(2) + 3 * l(3) + 2) >> 2
                    else:
                        v = l(3)
                else:
                    raise BitstreamError(f"Intra4x4 mode {mode}")
                P[y, x] = v
        return P

    def _decode_i4(self, br, sps, pps, cur, mbx, mby, sid):
        self.stats["i4"] += 1
        cur.intra = True
        cur.i4 = True
        for blk in range(16):
            bx, by = T.BLK_X[blk], T.BLK_Y[blk]
            a = self._i4_nb_mode(sps, cur, mbx, mby, bx - 1, by, sid)
            b = self._i4_nb_mode(sps, cur, mbx, mby, bx, by - 1, sid)
            pred = 2 if a is None or b is None else min(a, b)
            if br.u1():
                mode = pred
            else:
                rem = br.u(3)
                mode = rem if rem < pred else rem + 1
            cur.i4_modes[by * 4 + bx] = mode
        chroma_mode = br.ue()
        code = br.ue()
        if code > 47:
            raise BitstreamError("coded_block_pattern out of range")
        cbp = T.CODE_TO_CBP_INTRA[code]
        cbp_l, cbp_c = cbp & 15, cbp >> 4
        if cbp:
            self._read_qp_delta(br)
        cur.qp = self.qp
        levels = [[0] * 16 for _ in range(16)]
        for b8 in range(4):
            if not cbp_l & (1 << b8):
                continue
            for i in range(4):
                blk = b8 * 4 + i
                bx, by = T.BLK_X[blk], T.BLK_Y[blk]
                nc = self._total_coeff_luma(cur, sps, mbx, mby, bx, by, sid)
                levels[blk], tc = self.residual_block(br, nc, 16)
                cur.tc_luma[by * 4 + bx] = tc
        dc, ac = self._chroma_residual(br, sps, pps, cur, mbx, mby, sid, cbp_c)
        Y = self.cur[0]
        qp = cur.qp
        for blk in range(16):   # decoding order: each block predicts from the ones before it
            bx, by = T.BLK_X[blk], T.BLK_Y[blk]
            top, left = self._i4_samples(sps, Y, mbx, mby, bx, by, sid)
            p = self._pred_i4(int(cur.i4_modes[by * 4 + bx]), top, left)
            r = _idct4(_scale_4x4(_unzigzag(levels[blk]), qp, skip_dc=False))
            Y[mby * 16 + by * 4:mby * 16 + by * 4 + 4, mbx * 16 + bx * 4:mbx * 16 + bx * 4 + 4] = _clip1(p + r)
        pu = self._pred_chroma(chroma_mode, *self._intra_neighbours(sps, pps, self.cur[1], mbx, mby, sid, 8))
        pv = self._pred_chroma(chroma_mode, *self._intra_neighbours(sps, pps, self.cur[2], mbx, mby, sid, 8))
        self._recon_chroma(sps, pps, cur, mbx, mby, dc, ac, pu, pv)

    def _decode_pcm(self, br, sps, cur, mbx, mby):
        self.stats["pcm"] += 1
        while not br.byte_aligned():
            if br.u1():
                raise BitstreamError("pcm_alignment_zero_bit is 1")
        Y, U, V = self.cur
        for y in range(16):
            for x in range(16):
                Y[mby * 16 + y, mbx * 16 + x] = br.u(8)
        for P in (U, V):
            for y in range(8):
                for x in range(8):
                    P[mby * 8 + y, mbx * 8 + x] = br.u(8)
        cur.intra = True
        cur.pcm = True
        cur.qp = self.qp  # QP'Y unchanged for later prediction; deblocking would use 0
        cur.tc_luma[:] = 16
        cur.tc_chroma[:] = 16

    # ---- inter ----------------------------------------------------------------
    def _mv_neighbour(self, sps, mbx, mby, x4, y4, sid):
        """(available, refIdx, mvx, mvy) for the 4x4 neighbour at relative (x4,y4)."""
        m, xx, yy = self._nb4(sps, mbx, mby, x4, y4, sid)
        if m is None:
            return False, -1, 0, 0
        if m.intra:
            return True, -1, 0, 0
        k = yy * 4 + xx
        return True, int(m.ref[k]), int(m.mvx[k]), int(m.mvy[k])

    def _mvp16(self, sps, mbx, mby, sid):
        aA, rA, ax, ay = self._mv_neighbour(sps, mbx, mby, -1, 0, sid)
        aB, rB, bx, by = self._mv_neighbour(sps, mbx, mby, 0, -1, sid)
        aC, rC, cx, cy = self._mv_neighbour(sps, mbx, mby, 4, -1, sid)
        if not aC:
            aC, rC, cx, cy = self._mv_neighbour(sps, mbx, mby, -1, -1, sid)
        return (aA, rA, ax, ay), (aB, rB, bx, by), (aC, rC, cx, cy)

    @staticmethod
    def _median_pred(A, B, C, ref=0):
        aA, rA, ax, ay = A
        aB, rB, bx, by = B
        aC, rC, cx, cy = C
        if not aB and not aC and aA:
            bx, by, rB = ax, ay, rA
            cx, cy, rC = ax, ay, rA
        m = [r == ref for r in (rA, rB, rC)]
        if sum(m) == 1:
            if m[0]:
                return ax, ay
            if m[1]:
                return bx, by
            return cx, cy
        return sorted([ax, bx, cx])[1], sorted([ay, by, cy])[1]

    def _decode_skip(self, sps, addr, sid):
        self.stats["skip"] += 1
        mbx, mby = addr % sps.mb_w, addr // sps.mb_w
        cur = self.mbs[addr]
        cur.__init__()
        cur.slice_id = sid
        cur.skip = True
        cur.qp = self.qp
        A, B, C = self._mvp16(sps, mbx, mby, sid)
        if not A[0] or not B[0]:
            mvx, mvy = 0, 0
        elif (A[1] == 0 and A[2] == 0 and A[3] == 0) or (B[1] == 0 and B[2] == 0 and B[3] == 0):
            mvx, mvy = 0, 0
        else:
            mvx, mvy = self._median_pred(A, B, C)
        cur.mvx[:] = mvx
        cur.mvy[:] = mvy
        cur.ref[:] = 0
        self._mc(sps, mbx, mby, mvx, mvy)
        cur.avail = True

    def _decode_p16(self, br, sps, pps, cur, mbx, mby, sid, num_ref):
        self.stats["p16"] += 1
        ref_idx = 0
        if num_ref == 2:
            ref_idx = 1 - br.u1()          # te(v) with range 1
        elif num_ref > 2:
            ref_idx = br.ue()
        if ref_idx >= num_ref:
            raise BitstreamError("ref_idx_l0 out of range")
        mvdx, mvdy = br.se(), br.se()
        A, B, C = self._mvp16(sps, mbx, mby, sid)
        px, py = self._median_pred(A, B, C, ref_idx)
        mvx, mvy = px + mvdx, py + mvdy
        cur.mvx[:] = mvx
        cur.mvy[:] = mvy
        cur.ref[:] = ref_idx
        code = br.ue()
        if code > 47:
            raise BitstreamError("coded_block_pattern out of range")
        cbp = T.CODE_TO_CBP_INTER[code]
        cbp_l, cbp_c = cbp & 15, cbp >> 4
        if cbp:
            self._read_qp_delta(br)
        cur.qp = self.qp
        levels = [[0] * 16 for _ in range(16)]
        for b8 in range(4):
            if not cbp_l & (1 << b8):
                continue
            for i in range(4):
                blk = b8 * 4 + i
                bx, by = T.BLK_X[blk], T.BLK_Y[blk]
                nc = self._total_coeff_luma(cur, sps, mbx, mby, bx, by, sid)
                levels[blk], tc = self.residual_block(br, nc, 16)
                cur.tc_luma[by * 4 + bx] = tc
        dc, ac = self._chroma_residual(br, sps, pps, cur, mbx, mby, sid, cbp_c)
        py_, pu, pv = self._mc(sps, mbx, mby, mvx, mvy, write=False, ref_idx=ref_idx)
        Y = self.cur[0]
        qp = cur.qp
        for blk in range(16):
            bx, by = T.BLK_X[blk], T.BLK_Y[blk]
            d = _scale_4x4(_unzigzag(levels[blk]), qp, skip_dc=False)
            r = _idct4(d)
            p = py_[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4].astype(np.int64)
            Y[mby * 16 + by * 4:mby * 16 + by * 4 + 4, mbx * 16 + bx * 4:mbx * 16 + bx * 4 + 4] = _clip1(p + r)
        self._recon_chroma(sps, pps, cur, mbx, mby, dc, ac, pu, pv)

    # ---- motion compensation (8.4.2.2) ------------------------------------------
    def _mc(self, sps, mbx, mby, mvx, mvy, write=True, ref_idx=0):
        if ref_idx >= len(self.dpb):
            raise BitstreamError(f"ref_idx {ref_idx} with {len(self.dpb)} reference pictures")
        rY, rU, rV = self.dpb[ref_idx]
        H, W = rY.shape
        x0, y0 = mbx * 16, mby * 16
        xi, yi = x0 + (mvx >> 2), y0 + (mvy >> 2)
        xf, yf = mvx & 3, mvy & 3

        def L(x, y):
            return rY[np.clip(y, 0, H - 1)][:, np.clip(x, 0, W - 1)].astype(np.int64)

        ys = np.arange(yi - 2, yi + 16 + 3)
        xs = np.arange(xi - 2, xi + 16 + 3)
        win = L(xs, ys)  # 21x21 window, origin at (xi-2, yi-2)
        G = win[2:18, 2:18]
        if xf == 0 and yf == 0:
            pred = G
        else:
            def tap(a, b, c, d, e, f):
                return a - 5 * b + 20 * c + 20 * d - 5 * e + f
            # horizontal half-pel b (between G and H) at all 21 rows
            b1 = tap(win[:, 0:16], win[:, 1:17], win[:, 2:18], win[:, 3:19], win[:, 4:20], win[:, 5:21])
            b = _clip1((b1 + 16) >> 5)
            # vertical half-pel h at all 21 columns
            h1 = tap(win[0:16, :], win[1:17, :], win[2:18, :], win[3:19, :], win[4:20, :], win[5:21, :])
            hh = _clip1((h1 + 16) >> 5)
            # centre j from the intermediate horizontal values b1
            j1 = tap(b1[0:16], b1[1:17], b1[2:18], b1[3:19], b1[4:20], b1[5:21])
            j = _clip1((j1 + 512) >> 10)
            bb = b[2:18]             # b at rows of G
            hh_ = hh[:, 2:18]        # h at columns of G
            s = b[3:19]              # half-pel one row below (b of G+1 row)
            m = hh[:, 3:19]          # vertical half-pel one column right
            Gr = win[2:18, 3:19]     # G shifted right
            Gd = win[3:19, 2:18]     # G shifted down
            table = {
                (1, 0): (G + bb + 1) >> 1, (2, 0): bb, (3, 0): (bb + Gr + 1) >> 1,
                (0, 1): (G + hh_ + 1) >> 1, (0, 2): hh_, (0, 3): (hh_ + Gd + 1) >> 1,
                (1, 1): (bb + hh_ + 1) >> 1, (3, 1): (bb + m + 1) >> 1,
                (1, 3): (hh_ + s + 1) >> 1, (3, 3): (s + m + 1) >> 1,
                (2, 1): (bb + j + 1) >> 1, (2, 3): (j + s + 1) >> 1,
                (1, 2): (hh_ + j + 1) >> 1, (3, 2): (j + m + 1) >> 1, (2, 2): j,
            }
            pred = table[(xf, yf)]
        # chroma (8.4.2.2.2)
        Hc, Wc = rU.shape
        cx, cy = mbx * 8, mby * 8
        preds = []
        for P in (rU, rV):
            yy, xx = np.mgrid[0:8, 0:8]
            xa = cx + xx + (mvx >> 3)
            ya = cy + yy + (mvy >> 3)
            fx, fy = mvx & 7, mvy & 7
            x0c, x1c = np.clip(xa, 0, Wc - 1), np.clip(xa + 1, 0, Wc - 1)
            y0c, y1c = np.clip(ya, 0, Hc - 1), np.clip(ya + 1, 0, Hc - 1)
            A = P[y0c, x0c].astype(np.int64)
            B = P[y0c, x1c].astype(np.int64)
            C = P[y1c, x0c].astype(np.int64)
            D = P[y1c, x1c].astype(np.int64)
            preds.append(((8 - fx) * (8 - fy) * A + fx * (8 - fy) * B + (8 - fx) * fy * C + fx * fy * D + 32) >> 6)
        if write:
            self.cur[0][y0:y0 + 16, x0:x0 + 16] = pred
            self.cur[1][cy:cy + 8, cx:cx + 8] = preds[0]
            self.cur[2][cy:cy + 8, cx:cx + 8] = preds[1]
        return pred, preds[0], preds[1]


def decode_stream(data: bytes):
    """Convenience: decode an Annex-B byte string, return list of (Y,U,V) frames."""
    return H264Decoder().decode(data)
