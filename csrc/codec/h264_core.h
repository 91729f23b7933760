// H.264 Constrained-Baseline primitives shared by the CPU reference encoder and
// the gfx950 kernels: integer transforms, (de)quantisation, intra prediction,
// motion-vector prediction and the CAVLC residual coder.
//
// The decoder-side operations (dequant, inverse transforms, prediction) follow
// the normative process of H.264 clause 8 exactly, so the encoder's
// reconstruction equals what any conforming decoder (browser WebCodecs) builds.
// The forward/quant side is encoder choice (JM/x264-style dead-zone quant).
#pragma once
#include "sk_common.h"
#include "h264_tables.h"

namespace sk {
namespace h264 {

enum MbType : uint8_t { MB_P_SKIP = 0, MB_P_16x16 = 1, MB_I16x16 = 2, MB_I4x4 = 3 };
enum SliceKind : uint8_t { SLICE_NONE = 0, SLICE_P = 1, SLICE_I = 2 };

constexpr int kMaxLevel = 2063;       // keeps every level inside the Baseline escape range
constexpr int kMaxMbBits = 3200;      // 128 + RawMbBits (A.3.1) for 8-bit 4:2:0
constexpr int kMbBitBudget = 3000;    // conservative target used for QP escalation

// Coefficient storage per macroblock (int16, scan order inside each block).
constexpr int kCoefLuma = 0;          // 16 blocks x 16 (luma4x4BlkIdx order)
constexpr int kCoefLumaDC = 256;      // 16 (Intra16x16 DC, scan order)
constexpr int kCoefChromaDC = 272;    // 2 x 4 (Cb, Cr)
constexpr int kCoefChromaAC = 280;    // 8 x 16 (Cb blk0..3, Cr blk0..3); index 0 unused
constexpr int kCoefPerMb = 408;

// Per-macroblock side information written by the mode-decision stage and read
// by the entropy stage. Layout is shared by CPU and GPU (tests diff it).
struct MbInfo {
    int16_t mvx, mvy;        // final motion vector, quarter-pel
    int16_t mvdx, mvdy;      // mvd written to the bitstream (P_L0_16x16)
    uint8_t type;            // MbType
    uint8_t i16_mode;        // Intra16x16PredMode
    uint8_t chroma_mode;     // intra_chroma_pred_mode
    uint8_t cbp;             // bits 0..3 luma 8x8, bits 4..5 chroma (0,1,2)
    uint8_t qp;              // QP used for quantisation
    uint8_t nnz[24];         // TotalCoeff per block: 16 luma (blkIdx), 4 Cb, 4 Cr
    uint8_t ref;             // ref_idx_l0 (P_L0_16x16)
    uint8_t pad[2];
    uint32_t i4lo, i4hi;     // Intra4x4PredMode per luma4x4BlkIdx, 4 bits each (blocks 0-7, 8-15; I_NxN)
};
static_assert(sizeof(MbInfo) == 48, "MbInfo layout");
// (two scalar words rather than an array: a GPU loop over blocks then needs no scratch)
SK_HD int i4_mode(const MbInfo& mb, int blk) { return (int)(((blk < 8 ? mb.i4lo : mb.i4hi) >> (4 * (blk & 7))) & 15u); }
SK_HD void set_i4_mode(MbInfo& mb, int blk, int mode) {
    const uint32_t sh = 4 * (blk & 7), v = (uint32_t)mode << sh, msk = 15u << sh;
    if (blk < 8) mb.i4lo = (mb.i4lo & ~msk) | v;
    else mb.i4hi = (mb.i4hi & ~msk) | v;
}

// K4a exhaustive integer search (MFMA on the GPU): candidates dx, dy in
// [-kFsR, kFsR), reference window (2*kFsR + 16)^2 clamped like every ME read.
// Candidates are ranked by the SSD proxy |r_d|^2 - 2<s, r_d> (|s|^2 is common to
// all of them) on 128-offset samples, ties to the lower raster index (dy, dx).
constexpr int kFsR = 16;
constexpr int kFsWin = 2 * kFsR + 16;
SK_HD uint64_t fs_key(int cost, int dyw, int dxw) {
    return ((uint64_t)(uint32_t)(cost + (1 << 24)) << 10) | (uint64_t)(dyw * (2 * kFsR) + dxw);
}
SK_HD int fs_key_dx(uint64_t k) { return (int)(k & (2 * kFsR - 1)) - kFsR; }
SK_HD int fs_key_dy(uint64_t k) { return (int)((k >> 5) & (2 * kFsR - 1)) - kFsR; }

// ---------------------------------------------------------------------------
// Bit writers. `put` appends the `len` low bits of `code`, MSB first.
struct BitCounter {
    int n = 0;
    SK_HD void put(uint32_t, int len) { n += len; }
};

struct BitWriter {  // sequential writer into a zeroed byte buffer
    uint8_t* buf;
    uint32_t pos;   // in bits
    SK_HD BitWriter(uint8_t* b, uint32_t p = 0) : buf(b), pos(p) {}
    SK_HD void put1(int bit) {
        if (bit) buf[pos >> 3] |= (uint8_t)(0x80u >> (pos & 7));
        pos++;
    }
    SK_HD void put(uint32_t code, int len) {
        for (int i = len - 1; i >= 0; --i) put1((code >> i) & 1);
    }
};

template <class W>
SK_HD void put_ue(W& w, uint32_t v) {
    uint32_t x = v + 1;
    int n = 0;
    while (x >> n) n++;
    // (n-1) zeros then the n-bit value of x
    if (n - 1 > 0) w.put(0, n - 1);
    w.put(x, n);
}
template <class W>
SK_HD void put_se(W& w, int v) { put_ue(w, sk_se_to_ue(v)); }

// ---------------------------------------------------------------------------
// Forward 4x4 core transform: W = Cf * X * Cf^T, X raster (row*4 + col).
SK_HD void fdct4x4(const int* x, int* w) {
    int t[16];
    for (int i = 0; i < 4; i++) {  // rows: horizontal transform
        int a = x[i * 4 + 0], b = x[i * 4 + 1], c = x[i * 4 + 2], d = x[i * 4 + 3];
        int s03 = a + d, d03 = a - d, s12 = b + c, d12 = b - c;
        t[i * 4 + 0] = s03 + s12;
        t[i * 4 + 1] = 2 * d03 + d12;
        t[i * 4 + 2] = s03 - s12;
        t[i * 4 + 3] = d03 - 2 * d12;
    }
    for (int j = 0; j < 4; j++) {  // columns: vertical transform
        int a = t[0 + j], b = t[4 + j], c = t[8 + j], d = t[12 + j];
        int s03 = a + d, d03 = a - d, s12 = b + c, d12 = b - c;
        w[0 + j] = s03 + s12;
        w[4 + j] = 2 * d03 + d12;
        w[8 + j] = s03 - s12;
        w[12 + j] = d03 - 2 * d12;
    }
}

// Inverse 4x4 transform (8.5.12.2): rows first, then columns, (x + 32) >> 6.
SK_HD void idct4x4(const int* d, int* r) {
    int f[16];
    for (int i = 0; i < 4; i++) {
        int d0 = d[i * 4 + 0], d1 = d[i * 4 + 1], d2 = d[i * 4 + 2], d3 = d[i * 4 + 3];
        int e0 = d0 + d2, e1 = d0 - d2, e2 = (d1 >> 1) - d3, e3 = d1 + (d3 >> 1);
        f[i * 4 + 0] = e0 + e3;
        f[i * 4 + 1] = e1 + e2;
        f[i * 4 + 2] = e1 - e2;
        f[i * 4 + 3] = e0 - e3;
    }
    for (int j = 0; j < 4; j++) {
        int f0 = f[0 + j], f1 = f[4 + j], f2 = f[8 + j], f3 = f[12 + j];
        int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        r[0 + j] = (g0 + g3 + 32) >> 6;
        r[4 + j] = (g1 + g2 + 32) >> 6;
        r[8 + j] = (g1 - g2 + 32) >> 6;
        r[12 + j] = (g0 - g3 + 32) >> 6;
    }
}

// 4x4 Hadamard (symmetric, unnormalised): out = H * in * H.
SK_HD void hadamard4x4(const int* in, int* out) {
    int t[16];
    for (int i = 0; i < 4; i++) {
        int a = in[i * 4 + 0], b = in[i * 4 + 1], c = in[i * 4 + 2], d = in[i * 4 + 3];
        int s01 = a + b, d01 = a - b, s23 = c + d, d23 = c - d;
        t[i * 4 + 0] = s01 + s23;
        t[i * 4 + 1] = s01 - s23;
        t[i * 4 + 2] = d01 - d23;
        t[i * 4 + 3] = d01 + d23;
    }
    for (int j = 0; j < 4; j++) {
        int a = t[0 + j], b = t[4 + j], c = t[8 + j], d = t[12 + j];
        int s01 = a + b, d01 = a - b, s23 = c + d, d23 = c - d;
        out[0 + j] = s01 + s23;
        out[4 + j] = s01 - s23;
        out[8 + j] = d01 - d23;
        out[12 + j] = d01 + d23;
    }
}

// ---------------------------------------------------------------------------
// Quantisation helpers.
SK_HD int quant_coef(int w, int mf, int f, int qbits) {
    int a = sk_abs(w);
    int l = (int)(((int64_t)a * mf + f) >> qbits);
    l = sk_min(l, kMaxLevel);
    return w < 0 ? -l : l;
}
SK_HD int quant_f(int qbits, bool intra) { return intra ? (1 << qbits) / 3 : (1 << qbits) / 6; }

// Position class of raster index r: 0 = (even,even), 1 = (odd,odd), 2 = mixed.
SK_HD int pos_class(int r) {
    int i = r >> 2, j = r & 3;
    return ((i | j) & 1) == 0 ? 0 : (((i & j) & 1) ? 1 : 2);
}
SK_HD int sel3(int c, int a0, int a1, int a2) { return c == 0 ? a0 : (c == 1 ? a1 : a2); }

// Dequantise a non-DC coefficient at raster position `r` (flat scaling lists).
SK_HD int dequant_coef(int l, int qp, int r) {
    const int32_t* v = H264_DEQUANT_V[qp % 6];
    return l * sel3(pos_class(r), v[0], v[1], v[2]) * (1 << (qp / 6));   // l may be negative: no <<
}

// Intra16x16 DC: inverse Hadamard of the 4x4 DC level matrix and scaling (8.5.10).
SK_HD void i16_dc_dequant(const int* c, int* dcy, int qp) {
    int f[16];
    hadamard4x4(c, f);
    int ls = 16 * H264_DEQUANT_V[qp % 6][0];
    int q6 = qp / 6;
    for (int i = 0; i < 16; i++) {
        if (qp >= 36) dcy[i] = f[i] * ls * (1 << (q6 - 6));
        else dcy[i] = (f[i] * ls + (1 << (5 - q6))) >> (6 - q6);
    }
}

// Chroma DC 2x2 (8.5.11): c raster [c00 c01 c10 c11].
SK_HD void chroma_dc_dequant(const int* c, int* dcc, int qpc) {
    int f0 = c[0] + c[1] + c[2] + c[3];
    int f1 = c[0] - c[1] + c[2] - c[3];
    int f2 = c[0] + c[1] - c[2] - c[3];
    int f3 = c[0] - c[1] - c[2] + c[3];
    int ls = 16 * H264_DEQUANT_V[qpc % 6][0];
    int q6 = qpc / 6;
    dcc[0] = (f0 * ls * (1 << q6)) >> 5;   // multiply: f may be negative
    dcc[1] = (f1 * ls * (1 << q6)) >> 5;   // multiply: f may be negative
    dcc[2] = (f2 * ls * (1 << q6)) >> 5;   // multiply: f may be negative
    dcc[3] = (f3 * ls * (1 << q6)) >> 5;   // multiply: f may be negative
}

// QPc (Table 8-15) without a memory table: on the GPU a table lookup is a vector load
// that would wait behind the coding kernels' outstanding stores.
SK_HD int chroma_qp(int qp) {
    qp = sk_clip(qp, 0, 51);
    if (qp < 30) return qp;
    const int i = qp - 30;
    const uint64_t d = i < 16 ? (0x9888776655433210ULL >> (4 * i)) : (0xaaaa99ULL >> (4 * (i - 16)));
    return 29 + (int)(d & 15);
}

// Lagrangian multiplier for motion-vector / mode bits (x264-like 0.85*2^((qp-12)/3)).
SK_TABLE uint8_t H264_LAMBDA[52] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2,
                                    2, 2, 3, 3, 3, 4, 4, 4, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14,
                                    16, 18, 20, 23, 25, 29, 32, 36, 40, 45, 51, 57, 64, 72, 81, 91};
SK_HD int lambda_for_qp(int qp) { return H264_LAMBDA[sk_clip(qp, 0, 51)]; }

// Decimation score of a 4x4 block (scan order, `n` coeffs): x264-style; a block
// with any |level| > 1 is never decimated.
SK_TABLE uint8_t H264_DECIMATE_RUN[16] = {3, 2, 2, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
SK_HD int decimate_score(const int16_t* c, int n) {
    int idx = n - 1;
    while (idx >= 0 && c[idx] == 0) idx--;
    int score = 0;
    while (idx >= 0) {
        if (sk_abs(c[idx]) > 1) return 9;
        int run = 0;
        idx--;
        while (idx >= 0 && c[idx] == 0) { idx--; run++; }
        score += run == 0 ? 3 : (run <= 2 ? 2 : (run <= 5 ? 1 : 0));
    }
    return score;
}

// ---------------------------------------------------------------------------
// CAVLC residual block coder (9.2). `c` holds `maxNum` levels in scan order.
// vlc selection: nC >= 0 -> luma/chroma-AC tables, nC == -1 -> chroma DC.
// Streaming formulation (no per-coefficient arrays) so the GPU build keeps
// everything in registers. Returns the TotalCoeff of the block.
template <class W>
SK_HD int cavlc_block(W& w, const int16_t* c, int maxNum, int nC, const CavlcTables& T) {
    // pass 1: TotalCoeff, TrailingOnes, position of the last non-zero
    int total = 0, t1 = 0, last = -1;
    bool in_t1 = true;
    for (int i = maxNum - 1; i >= 0; i--) {
        int v = c[i];
        if (v == 0) continue;
        if (last < 0) last = i;
        total++;
        if (in_t1 && t1 < 3 && (v == 1 || v == -1)) t1++;
        else in_t1 = false;
    }
    int tok = total * 4 + t1;
    if (nC == -1) {
        w.put(T.cdc_code[tok], T.cdc_len[tok]);
    } else {
        int vlc = nC < 2 ? 0 : (nC < 4 ? 1 : (nC < 8 ? 2 : 3));
        w.put(T.ct_code[vlc][tok], T.ct_len[vlc][tok]);
    }
    if (total == 0) return 0;
    const int total_zeros = (last + 1) - total;
    // pass 2: trailing-one signs and levels, highest frequency first
    int k = 0;
    int suffix_len = (total > 10 && t1 < 3) ? 1 : 0;
    for (int i = last; i >= 0; i--) {
        int lv = c[i];
        if (lv == 0) continue;
        if (k < t1) {
            w.put(lv < 0 ? 1 : 0, 1);
        } else {
            int lc = lv > 0 ? 2 * lv - 2 : -2 * lv - 1;
            if (k == t1 && t1 < 3) lc -= 2;
            if (suffix_len == 0) {
                if (lc < 14) {
                    w.put(1, lc + 1);
                } else if (lc < 30) {
                    w.put(1, 15);  // level_prefix 14
                    w.put(lc - 14, 4);
                } else {
                    w.put(1, 16);  // level_prefix 15
                    w.put(lc - 30, 12);
                }
            } else {
                if (lc < (15 << suffix_len)) {
                    w.put(1, (lc >> suffix_len) + 1);
                    w.put(lc & ((1 << suffix_len) - 1), suffix_len);
                } else {
                    w.put(1, 16);
                    w.put(lc - (15 << suffix_len), 12);
                }
            }
            if (suffix_len == 0) suffix_len = 1;
            if (sk_abs(lv) > (3 << (suffix_len - 1)) && suffix_len < 6) suffix_len++;
        }
        k++;
    }
    if (total < maxNum) {
        if (maxNum == 4) w.put(T.cdc_tz_code[total - 1][total_zeros], T.cdc_tz_len[total - 1][total_zeros]);
        else w.put(T.tz_code[total - 1][total_zeros], T.tz_len[total - 1][total_zeros]);
    }
    // pass 3: run_before of each coefficient but the lowest-frequency one
    int zeros_left = total_zeros;
    k = 0;
    for (int i = last; i >= 0 && zeros_left > 0 && k < total - 1;) {
        int run = 0;
        int j = i - 1;
        while (j >= 0 && c[j] == 0) { run++; j--; }
        int tbl = sk_min(zeros_left, 7) - 1;
        w.put(T.rb_code[tbl][run], T.rb_len[tbl][run]);
        zeros_left -= run;
        k++;
        i = j;
    }
    return total;
}

SK_HD void cavlc_token_stats(const int16_t* c, int maxNum, int* total, int* t1) {
    int n = 0, t = 0;
    bool in_t1 = true;
    for (int i = maxNum - 1; i >= 0; i--) {
        if (c[i] == 0) continue;
        n++;
        if (in_t1 && t < 3 && (c[i] == 1 || c[i] == -1)) t++;
        else in_t1 = false;
    }
    *total = n;
    *t1 = t;
}
SK_HD int cavlc_block_bits_bound(const int16_t* c, int maxNum, const CavlcTables& T) {
    BitCounter bc;
    cavlc_block(bc, c, maxNum, 0, T);
    int total, t1;
    cavlc_token_stats(c, maxNum, &total, &t1);
    int tok = total * 4 + t1;
    return bc.n - T.ct_len[0][tok] + T.ct_maxlen[tok];
}

// Host-side table instance (the GPU kernels keep theirs in LDS).
inline const CavlcTables& host_cavlc_tables() {
    static CavlcTables t = [] {
        CavlcTables x;
        cavlc_tables_copy_range(x, 0, 1);
        return x;
    }();
    return t;
}

SK_HD int count_nonzero(const int16_t* c, int n) {
    int k = 0;
    for (int i = 0; i < n; i++) k += c[i] != 0;
    return k;
}

// nC from neighbour availability and counts (9.2.1).
SK_HD int nc_from(bool availA, int nA, bool availB, int nB) {
    if (availA && availB) return (nA + nB + 1) >> 1;
    if (availA) return nA;
    if (availB) return nB;
    return 0;
}

// ---------------------------------------------------------------------------
// Motion-vector prediction for a 16x16 partition with one reference (8.4.1.3).
struct MvNb {
    bool avail;   // neighbour macroblock exists in this slice (already coded)
    int ref;      // its refIdxL0; -1 when unavailable or intra
    int mvx, mvy;
};

// mvpLX of a 16x16 partition with refIdx `ref` (8.4.1.3, 8.4.1.3.1).
SK_HD void mv_pred16x16(MvNb A, MvNb B, MvNb C, int ref, int* px, int* py) {
    int rA = A.avail ? A.ref : -1, rB = B.avail ? B.ref : -1, rC = C.avail ? C.ref : -1;
    int ax = rA >= 0 ? A.mvx : 0, ay = rA >= 0 ? A.mvy : 0;
    int bx = rB >= 0 ? B.mvx : 0, by = rB >= 0 ? B.mvy : 0;
    int cx = rC >= 0 ? C.mvx : 0, cy = rC >= 0 ? C.mvy : 0;
    if (!B.avail && !C.avail && A.avail) {
        bx = cx = ax;
        by = cy = ay;
        rB = rC = rA;
    }
    int matches = (rA == ref) + (rB == ref) + (rC == ref);
    if (matches == 1) {
        if (rA == ref) { *px = ax; *py = ay; }
        else if (rB == ref) { *px = bx; *py = by; }
        else { *px = cx; *py = cy; }
        return;
    }
    *px = sk_median(ax, bx, cx);
    *py = sk_median(ay, by, cy);
}

// P_Skip motion vector (8.4.1.1): refIdx 0.
SK_HD void mv_pskip(MvNb A, MvNb B, MvNb C, int* px, int* py) {
    if (!A.avail || !B.avail) { *px = 0; *py = 0; return; }
    if (A.ref == 0 && A.mvx == 0 && A.mvy == 0) { *px = 0; *py = 0; return; }
    if (B.ref == 0 && B.mvx == 0 && B.mvy == 0) { *px = 0; *py = 0; return; }
    mv_pred16x16(A, B, C, 0, px, py);
}

// ---------------------------------------------------------------------------
// Intra 16x16 prediction (8.3.3). top[16], left[16], tl = p[-1,-1].
// Modes: 0 vertical, 1 horizontal, 2 DC, 3 plane.
SK_HD int i16_pred_pixel(int mode, int x, int y, const uint8_t* top, const uint8_t* left,
                         int tl, bool availT, bool availL, int dc, int pa, int pb, int pc) {
    switch (mode) {
        case 0: return top[x];
        case 1: return left[y];
        case 2: return dc;
        default: return sk_clip255((pa + pb * (x - 7) + pc * (y - 7) + 16) >> 5);
    }
}
SK_HD int i16_dc(const uint8_t* top, const uint8_t* left, bool availT, bool availL) {
    int s = 0;
    if (availT && availL) {
        for (int i = 0; i < 16; i++) s += top[i] + left[i];
        return (s + 16) >> 5;
    }
    if (availL) {
        for (int i = 0; i < 16; i++) s += left[i];
        return (s + 8) >> 4;
    }
    if (availT) {
        for (int i = 0; i < 16; i++) s += top[i];
        return (s + 8) >> 4;
    }
    return 128;
}
SK_HD void i16_plane_params(const uint8_t* top, const uint8_t* left, int tl, int* pa, int* pb,
                            int* pc) {
    int H = 0, V = 0;
    for (int i = 0; i < 8; i++) {
        int tpos = 8 + i, tneg = 6 - i;
        int t1 = top[tpos], t0 = tneg >= 0 ? top[tneg] : tl;
        int l1 = left[tpos], l0 = tneg >= 0 ? left[tneg] : tl;
        H += (i + 1) * (t1 - t0);
        V += (i + 1) * (l1 - l0);
    }
    *pa = 16 * (left[15] + top[15]);
    *pb = (5 * H + 32) >> 6;
    *pc = (5 * V + 32) >> 6;
}

// Intra chroma 8x8 prediction (8.3.4). Modes: 0 DC, 1 horizontal, 2 vertical, 3 plane.
SK_HD int chroma_dc_block(int bx, int by, const uint8_t* top, const uint8_t* left, bool availT,
                          bool availL) {
    int st = 0, sl = 0;
    for (int i = 0; i < 4; i++) {
        st += top[bx * 4 + i];
        sl += left[by * 4 + i];
    }
    bool diag = (bx == by);
    if (diag) {
        if (availT && availL) return (st + sl + 4) >> 3;
        if (availL) return (sl + 2) >> 2;
        if (availT) return (st + 2) >> 2;
        return 128;
    }
    if (bx == 1 && by == 0) {  // top-right block prefers top
        if (availT) return (st + 2) >> 2;
        if (availL) return (sl + 2) >> 2;
        return 128;
    }
    // bottom-left block prefers left
    if (availL) return (sl + 2) >> 2;
    if (availT) return (st + 2) >> 2;
    return 128;
}
SK_HD void chroma_plane_params(const uint8_t* top, const uint8_t* left, int tl, int* pa, int* pb,
                               int* pc) {
    int H = 0, V = 0;
    for (int i = 0; i < 4; i++) {
        int tpos = 4 + i, tneg = 2 - i;
        int t0 = tneg >= 0 ? top[tneg] : tl;
        int l0 = tneg >= 0 ? left[tneg] : tl;
        H += (i + 1) * (top[tpos] - t0);
        V += (i + 1) * (left[tpos] - l0);
    }
    *pa = 16 * (left[7] + top[7]);
    *pb = (34 * H + 32) >> 6;
    *pc = (34 * V + 32) >> 6;
}

// Full 8x8 chroma prediction of one component for mode m (0 DC, 1 H, 2 V, 3 plane).
SK_HD void intra_chroma_pred(int m, const uint8_t* top, const uint8_t* left, int tl, bool aT, bool aL,
                             uint8_t* out) {
    int qa = 0, qb = 0, qc = 0;
    if (m == 3) chroma_plane_params(top, left, tl, &qa, &qb, &qc);
    for (int y = 0; y < 8; y++)
        for (int x = 0; x < 8; x++) {
            int v;
            if (m == 0) v = chroma_dc_block(x >> 2, y >> 2, top, left, aT, aL);
            else if (m == 1) v = left[y];
            else if (m == 2) v = top[x];
            else v = sk_clip255((qa + qb * (x - 3) + qc * (y - 3) + 16) >> 5);
            out[y * 8 + x] = (uint8_t)v;
        }
}

// mb_type ue(v) code number for an I16x16 macroblock in an I slice (add 5 in P slices).
SK_HD int i16_mb_type(int pred_mode, int cbp_luma15, int cbp_chroma) {
    return 1 + pred_mode + 4 * cbp_chroma + 12 * (cbp_luma15 ? 1 : 0);
}

// Chroma motion compensation sample (8.4.2.2.2), mv in 1/8 chroma pel.
// ---- quarter-pel luma interpolation (8.4.2.2.1) -----------------------------------
// Reference samples at clamped coordinates: x in [0, w - 1], y in [ylo, yhi] (the picture
// a stripe is: rows of its own slice only). Computed on the fly, identically on host
// and device (no half-pel planes to keep in sync with per-stripe reference commits).
SK_HD int qp_ref(const uint8_t* ref, int stride, int w, int ylo, int yhi, int x, int y) {
    return ref[(size_t)sk_clip(y, ylo, yhi) * stride + sk_clip(x, 0, w - 1)];
}
SK_HD int qp_tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }
// unclipped horizontal half-sample intermediate b1 at (x + 1/2, y)
SK_HD int qp_b1(const uint8_t* r, int st, int w, int ylo, int yhi, int x, int y) {
    return qp_tap6(qp_ref(r, st, w, ylo, yhi, x - 2, y), qp_ref(r, st, w, ylo, yhi, x - 1, y),
                   qp_ref(r, st, w, ylo, yhi, x, y), qp_ref(r, st, w, ylo, yhi, x + 1, y),
                   qp_ref(r, st, w, ylo, yhi, x + 2, y), qp_ref(r, st, w, ylo, yhi, x + 3, y));
}
SK_HD int qp_h1(const uint8_t* r, int st, int w, int ylo, int yhi, int x, int y) {
    return qp_tap6(qp_ref(r, st, w, ylo, yhi, x, y - 2), qp_ref(r, st, w, ylo, yhi, x, y - 1),
                   qp_ref(r, st, w, ylo, yhi, x, y), qp_ref(r, st, w, ylo, yhi, x, y + 1),
                   qp_ref(r, st, w, ylo, yhi, x, y + 2), qp_ref(r, st, w, ylo, yhi, x, y + 3));
}
SK_HD int qp_b(const uint8_t* r, int st, int w, int ylo, int yhi, int x, int y) {
    return sk_clip255((qp_b1(r, st, w, ylo, yhi, x, y) + 16) >> 5);
}
SK_HD int qp_h(const uint8_t* r, int st, int w, int ylo, int yhi, int x, int y) {
    return sk_clip255((qp_h1(r, st, w, ylo, yhi, x, y) + 16) >> 5);
}
SK_HD int qp_j(const uint8_t* r, int st, int w, int ylo, int yhi, int x, int y) {
    return sk_clip255((qp_tap6(qp_b1(r, st, w, ylo, yhi, x, y - 2), qp_b1(r, st, w, ylo, yhi, x, y - 1),
                               qp_b1(r, st, w, ylo, yhi, x, y), qp_b1(r, st, w, ylo, yhi, x, y + 1),
                               qp_b1(r, st, w, ylo, yhi, x, y + 2), qp_b1(r, st, w, ylo, yhi, x, y + 3)) +
                       512) >> 10);
}
// Luma prediction sample at full-sample position (x, y) displaced by the quarter-pel
// vector (mvx, mvy): Table 8-12 (G, a..s).
SK_HD int luma_qpel_sample(const uint8_t* r, int st, int w, int ylo, int yhi, int x, int y, int mvx, int mvy) {
    const int xi = x + (mvx >> 2), yi = y + (mvy >> 2), fx = mvx & 3, fy = mvy & 3;
    if (!(fx | fy)) return qp_ref(r, st, w, ylo, yhi, xi, yi);
    if (fy == 0) {
        const int b = qp_b(r, st, w, ylo, yhi, xi, yi);
        if (fx == 2) return b;
        return (qp_ref(r, st, w, ylo, yhi, xi + (fx >> 1), yi) + b + 1) >> 1;   // a (fx 1) / c (fx 3)
    }
    if (fx == 0) {
        const int h = qp_h(r, st, w, ylo, yhi, xi, yi);
        if (fy == 2) return h;
        return (qp_ref(r, st, w, ylo, yhi, xi, yi + (fy >> 1)) + h + 1) >> 1;   // d (fy 1) / n (fy 3)
    }
    if (fx == 2 && fy == 2) return qp_j(r, st, w, ylo, yhi, xi, yi);
    if (fx == 2) {   // f (fy 1) / q (fy 3): j with b of the row above / below the half row
        const int j = qp_j(r, st, w, ylo, yhi, xi, yi);
        return (qp_b(r, st, w, ylo, yhi, xi, yi + (fy >> 1)) + j + 1) >> 1;
    }
    if (fy == 2) {   // i (fx 1) / k (fx 3)
        const int j = qp_j(r, st, w, ylo, yhi, xi, yi);
        return (qp_h(r, st, w, ylo, yhi, xi + (fx >> 1), yi) + j + 1) >> 1;
    }
    // e, g, p, r: diagonal averages of a horizontal and a vertical half sample
    return (qp_b(r, st, w, ylo, yhi, xi, yi + (fy >> 1)) + qp_h(r, st, w, ylo, yhi, xi + (fx >> 1), yi) + 1) >> 1;
}

SK_HD int chroma_mc_sample(const uint8_t* ref, int stride, int w, int h, int x, int y, int mvx,
                           int mvy) {
    int xi = x + (mvx >> 3), yi = y + (mvy >> 3);
    int xf = mvx & 7, yf = mvy & 7;
    int x0 = sk_clip(xi, 0, w - 1), x1 = sk_clip(xi + 1, 0, w - 1);
    int y0 = sk_clip(yi, 0, h - 1), y1 = sk_clip(yi + 1, 0, h - 1);
    int A = ref[y0 * stride + x0], B = ref[y0 * stride + x1];
    int C = ref[y1 * stride + x0], D = ref[y1 * stride + x1];
    return ((8 - xf) * (8 - yf) * A + xf * (8 - yf) * B + (8 - xf) * yf * C + xf * yf * D + 32) >> 6;
}

}  // namespace h264
}  // namespace sk
