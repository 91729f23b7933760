// H.264 in-loop deblocking filter (clause 8.7) for the macroblock types this
// encoder emits: I16x16, P_L0_16x16 and P_Skip frame macroblocks, 4x4
// transforms, 4:2:0, one reference picture. Slices are coded with
// disable_deblocking_filter_idc = 2 (filter inside a slice only), so every
// stripe/slice deblocks independently — the unit of GPU parallelism.
//
// The per-line filters and the boundary-strength rule are SK_HD and shared by
// the CPU reference (deblock_slice_cpu, raster MB order as in 8.7) and the
// gfx950 wavefront kernel (k_deblock in csrc/kernels/h264_kernels.hip), which
// reorders the MBs along anti-diagonals without changing any sample: the result
// is bit-identical and equals what a conforming decoder (WebCodecs) produces.
#pragma once
#include <stddef.h>
#include "h264_core.h"

namespace sk {
namespace h264 {

// Table 8-16 (alpha', beta') and 8-17 (tC0 for bS = 1, 2, 3), indexed by indexA/indexB.
SK_TABLE uint8_t H264_DB_ALPHA[52] = {
    0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  4,   4,   5,   6,   7,   8,   9,   10,  12,  13,
    15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90, 101, 113, 127, 144, 162, 182, 203, 226, 255, 255};
SK_TABLE uint8_t H264_DB_BETA[52] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  2,  2,  2,  3,  3,  3,  3,  4,  4,  4,
    6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15, 15, 16, 16, 17, 17, 18, 18};
SK_TABLE uint8_t H264_DB_TC0[52][3] = {
    {0, 0, 0},    {0, 0, 0},    {0, 0, 0},    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},    {0, 0, 0},
    {0, 0, 0},    {0, 0, 0},    {0, 0, 0},    {0, 0, 0},   {0, 0, 0},   {0, 0, 0},    {0, 0, 0},
    {0, 0, 0},    {0, 0, 0},    {0, 0, 0},    {0, 0, 1},   {0, 0, 1},   {0, 0, 1},    {0, 0, 1},
    {0, 1, 1},    {0, 1, 1},    {1, 1, 1},    {1, 1, 1},   {1, 1, 1},   {1, 1, 1},    {1, 1, 2},
    {1, 1, 2},    {1, 1, 2},    {1, 1, 2},    {1, 2, 3},   {1, 2, 3},   {2, 2, 3},    {2, 2, 4},
    {2, 3, 4},    {2, 3, 4},    {3, 3, 5},    {3, 4, 6},   {3, 4, 6},   {4, 5, 7},    {4, 5, 8},
    {4, 6, 9},    {5, 7, 10},   {6, 8, 11},   {6, 8, 13},  {7, 10, 14}, {8, 11, 16},  {9, 12, 18},
    {10, 13, 20}, {11, 15, 23}, {13, 17, 25}};

// Filter tables as one POD: the GPU kernel copies it to LDS once per workgroup (a
// __constant__ lookup per edge would be a global-memory round trip on every edge).
struct DbTables {
    uint8_t alpha[52], beta[52], tc0[52][3], cqp[52];
};
SK_HD void db_tables_init(DbTables& t, int begin = 0, int step = 1) {
    for (int i = begin; i < 52; i += step) {
        t.alpha[i] = H264_DB_ALPHA[i];
        t.beta[i] = H264_DB_BETA[i];
        t.tc0[i][0] = H264_DB_TC0[i][0];
        t.tc0[i][1] = H264_DB_TC0[i][1];
        t.tc0[i][2] = H264_DB_TC0[i][2];
        t.cqp[i] = H264_CHROMA_QP[i];
    }
}
inline const DbTables& host_db_tables() {
    static const DbTables t = [] {
        DbTables x;
        db_tables_init(x);
        return x;
    }();
    return t;
}

// What the filter needs to know about one macroblock (8 bytes, shared CPU/GPU layout).
struct DbInfo {
    uint8_t intra;     // bit 0: intra MB (I16x16 / I4x4); bits 1+: ref_idx (bS 1 across different reference pictures)
    uint8_t qpy;       // QP_Y as the decoder derives it (mb_qp_delta chain, 7.4.5)
    uint16_t nz;       // bit (by*4+bx): luma 4x4 block at raster (bx,by) has coded coefficients
    int16_t mvx, mvy;  // quarter-pel
};
static_assert(sizeof(DbInfo) == 8, "DbInfo layout");

SK_HD DbInfo db_info(const MbInfo& mb, int qpy) {
    DbInfo d;
    const bool intra = mb.type == MB_I16x16 || mb.type == MB_I4x4;
    d.intra = (uint8_t)(intra ? 1 : mb.ref << 1);
    d.qpy = (uint8_t)qpy;
    uint32_t nz = 0;
    for (int b = 0; b < 16; b++)
        if (mb.nnz[b]) nz |= 1u << (blk_y(b) * 4 + blk_x(b));
    d.nz = (uint16_t)nz;
    d.mvx = mb.mvx;
    d.mvy = mb.mvy;
    return d;
}

// Boundary strength (8.7.2.1) between blocks pb (in MB p) and qb (in MB q), raster 4x4 indices.
SK_HD int db_bs(const DbInfo& p, const DbInfo& q, bool mb_edge, int pb, int qb) {
    if ((p.intra & 1) || (q.intra & 1)) return mb_edge ? 4 : 3;
    if (((p.nz >> pb) & 1) || ((q.nz >> qb) & 1)) return 2;
    if ((p.intra >> 1) != (q.intra >> 1)) return 1;   // different reference pictures
    if (sk_abs(p.mvx - q.mvx) >= 4 || sk_abs(p.mvy - q.mvy) >= 4) return 1;
    return 0;
}

// Luma line filter (8.7.2.3/8.7.2.4). v = {p3, p2, p1, p0, q0, q1, q2, q3}, updated in place.
// Written select-style (every candidate value computed, one final choice) so a
// wavefront running many lines executes one short straight-line sequence.
SK_HD void db_filter_luma(int* v, int bs, int qpav, const DbTables& T) {
    const int alpha = T.alpha[qpav], beta = T.beta[qpav];
    const int tc0 = T.tc0[qpav][sk_clip(bs - 1, 0, 2)];
    const int p3 = v[0], p2 = v[1], p1 = v[2], p0 = v[3], q0 = v[4], q1 = v[5], q2 = v[6], q3 = v[7];
    const bool on = bs != 0 && sk_abs(p0 - q0) < alpha && sk_abs(p1 - p0) < beta && sk_abs(q1 - q0) < beta;
    const bool ap = sk_abs(p2 - p0) < beta, aq = sk_abs(q2 - q0) < beta;
    // bS < 4
    const int tc = tc0 + (ap ? 1 : 0) + (aq ? 1 : 0);
    const int d = sk_clip((((q0 - p0) * 4) + (p1 - q1) + 4) >> 3, -tc, tc);
    const int avg = (p0 + q0 + 1) >> 1;
    int np0 = sk_clip255(p0 + d), nq0 = sk_clip255(q0 - d);
    int np1 = ap ? p1 + sk_clip((p2 + avg - (p1 * 2)) >> 1, -tc0, tc0) : p1;
    int nq1 = aq ? q1 + sk_clip((q2 + avg - (q1 * 2)) >> 1, -tc0, tc0) : q1;
    int np2 = p2, nq2 = q2;
    if (bs == 4) {
        const bool sm = sk_abs(p0 - q0) < ((alpha >> 2) + 2);
        const bool ps = ap && sm, qs = aq && sm;
        np0 = ps ? (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3 : (2 * p1 + p0 + q1 + 2) >> 2;
        np1 = ps ? (p2 + p1 + p0 + q0 + 2) >> 2 : p1;
        np2 = ps ? (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3 : p2;
        nq0 = qs ? (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3 : (2 * q1 + q0 + p1 + 2) >> 2;
        nq1 = qs ? (p0 + q0 + q1 + q2 + 2) >> 2 : q1;
        nq2 = qs ? (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3 : q2;
    }
    if (on) {
        v[1] = np2;
        v[2] = np1;
        v[3] = np0;
        v[4] = nq0;
        v[5] = nq1;
        v[6] = nq2;
    }
}

// Chroma line filter. v = {p1, p0, q0, q1}; qpav is the average of the two MBs' QP_C.
SK_HD void db_filter_chroma(int* v, int bs, int qpav, const DbTables& T) {
    const int alpha = T.alpha[qpav], beta = T.beta[qpav];
    const int p1 = v[0], p0 = v[1], q0 = v[2], q1 = v[3];
    const bool on = bs != 0 && sk_abs(p0 - q0) < alpha && sk_abs(p1 - p0) < beta && sk_abs(q1 - q0) < beta;
    const int tc = T.tc0[qpav][sk_clip(bs - 1, 0, 2)] + 1;
    const int d = sk_clip((((q0 - p0) * 4) + (p1 - q1) + 4) >> 3, -tc, tc);
    const int np0 = bs == 4 ? (2 * p1 + p0 + q1 + 2) >> 2 : sk_clip255(p0 + d);
    const int nq0 = bs == 4 ? (2 * q1 + q0 + p1 + 2) >> 2 : sk_clip255(q0 - d);
    if (on) {
        v[1] = np0;
        v[2] = nq0;
    }
}

SK_HD int db_qpav_luma(const DbInfo& p, const DbInfo& q) { return (p.qpy + q.qpy + 1) >> 1; }
SK_HD int db_qpav_chroma(const DbInfo& p, const DbInfo& q, const DbTables& T) {
    return (T.cqp[p.qpy] + T.cqp[q.qpy] + 1) >> 1;
}

// One luma row (lane-parallel on the GPU): `row` holds the 4 samples left of the MB
// (cols -4..-1) followed by its 16 samples; vertical edges 0..3 in order. i = row in MB.
SK_HD void db_luma_row(int* row, const DbInfo& cur, const DbInfo& left, bool has_left, int i, const DbTables& T) {
    const int by = i >> 2;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        if (e == 0 && !has_left) continue;
        const DbInfo& p = e == 0 ? left : cur;
        const int bs = db_bs(p, cur, e == 0, by * 4 + (e == 0 ? 3 : e - 1), by * 4 + e);
        db_filter_luma(row + 4 * e, bs, db_qpav_luma(p, cur), T);
    }
}

// One luma column: 4 samples above the MB then its 16; horizontal edges 0..3. j = column.
SK_HD void db_luma_col(int* col, const DbInfo& cur, const DbInfo& top, bool has_top, int j, const DbTables& T) {
    const int bx = j >> 2;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        if (e == 0 && !has_top) continue;
        const DbInfo& p = e == 0 ? top : cur;
        const int bs = db_bs(p, cur, e == 0, (e == 0 ? 3 : e - 1) * 4 + bx, e * 4 + bx);
        db_filter_luma(col + 4 * e, bs, db_qpav_luma(p, cur), T);
    }
}

// One chroma row/column of one component: 2 samples before the MB then its 8
// (p1 p0 | q0..q7); edges at chroma 0 and 4 use the bS of luma edges 0 and 2 at
// luma line 2*i (8.7.2: chroma bS is taken from the co-sited luma sample).
SK_HD void db_chroma_line(int* line, const DbInfo& cur, const DbInfo& nb, bool has_nb, int i, bool vertical,
                          const DbTables& T) {
    const int b = (2 * i) >> 2;  // luma 4x4 block row (vertical edges) / column (horizontal)
#pragma unroll
    for (int e = 0; e < 2; e++) {
        if (e == 0 && !has_nb) continue;
        const DbInfo& p = e == 0 ? nb : cur;
        const int le = 2 * e;  // luma edge index
        int pb, qb;
        if (vertical) {
            pb = b * 4 + (le == 0 ? 3 : le - 1);
            qb = b * 4 + le;
        } else {
            pb = (le == 0 ? 3 : le - 1) * 4 + b;
            qb = le * 4 + b;
        }
        const int bs = db_bs(p, cur, e == 0, pb, qb);
        db_filter_chroma(line + 4 * e, bs, db_qpav_chroma(p, cur, T), T);
    }
}

// Host-only helpers of the CPU reference (never called from device code).
// QP_Y of every MB of a slice in raster order (skip / cbp-0 MBs inherit, 7.4.5).
// sub_len > 0: the slice is coded as sub-slices of sub_len MBs (h264_encoder.h
// intra_split): QP_Y,PRED restarts at the slice QP at every sub-slice start.
inline void db_slice_info(const MbInfo* mbs, int mb_w, int first_row, int num_rows, int slice_qp,
                          DbInfo* out, int sub_len = 0) {
    int qp = slice_qp;
    const int first = first_row * mb_w;
    for (int r = first_row; r < first_row + num_rows; r++)
        for (int x = 0; x < mb_w; x++) {
            const int idx = r * mb_w + x;
            if (sub_len > 0 && (idx - first) % sub_len == 0) qp = slice_qp;
            const MbInfo& mb = mbs[idx];
            if (mb_has_qp_delta(mb)) qp = mb.qp;
            out[idx] = db_info(mb, qp);
        }
}

// Reference deblocking of one slice in place, raster macroblock order (8.7).
// sub_len > 0: sub-slices of sub_len MBs; with disable_deblocking_filter_idc 2 no edge
// between two of them is filtered (the left / top MB must lie in the MB's sub-slice).
inline void deblock_slice_cpu(uint8_t* y, uint8_t* u, uint8_t* v, int stride_y, int stride_c, const DbInfo* info,
                              int mb_w, int first_row, int num_rows, int sub_len = 0) {
    const int first = first_row * mb_w;
    for (int r = first_row; r < first_row + num_rows; r++)
        for (int x = 0; x < mb_w; x++) {
            const DbTables& T = host_db_tables();
            const DbInfo& cur = info[r * mb_w + x];
            const int idx = r * mb_w + x, sub0 = sub_len > 0 ? first + ((idx - first) / sub_len) * sub_len : first;
            const bool hl = x > 0 && idx - 1 >= sub0, ht = r > first_row && idx - mb_w >= sub0;
            const DbInfo& left = info[r * mb_w + x - (hl ? 1 : 0)];
            const DbInfo& top = info[(r - (ht ? 1 : 0)) * mb_w + x];
            int buf[20];
            for (int i = 0; i < 16; i++) {  // vertical edges
                uint8_t* p = y + (size_t)(r * 16 + i) * stride_y + x * 16;
                for (int k = 0; k < 20; k++) buf[k] = (k < 4 && !hl) ? 0 : p[k - 4];
                db_luma_row(buf, cur, left, hl, i, T);
                for (int k = hl ? 0 : 4; k < 20; k++) p[k - 4] = (uint8_t)buf[k];
            }
            for (int j = 0; j < 16; j++) {  // horizontal edges
                uint8_t* p = y + (size_t)(r * 16) * stride_y + x * 16 + j;
                for (int k = 0; k < 20; k++) buf[k] = (k < 4 && !ht) ? 0 : p[(ptrdiff_t)(k - 4) * stride_y];
                db_luma_col(buf, cur, top, ht, j, T);
                for (int k = ht ? 0 : 4; k < 20; k++) p[(ptrdiff_t)(k - 4) * stride_y] = (uint8_t)buf[k];
            }
            for (int c = 0; c < 2; c++) {
                uint8_t* pl = c ? v : u;
                for (int i = 0; i < 8; i++) {  // chroma vertical edges: buf = p1 p0 | q0..q7
                    uint8_t* p = pl + (size_t)(r * 8 + i) * stride_c + x * 8;
                    for (int k = 0; k < 10; k++) buf[k] = (k < 2 && !hl) ? 0 : p[k - 2];
                    db_chroma_line(buf, cur, left, hl, i, true, T);
                    for (int k = hl ? 0 : 2; k < 10; k++) p[k - 2] = (uint8_t)buf[k];
                }
                for (int j = 0; j < 8; j++) {
                    uint8_t* p = pl + (size_t)(r * 8) * stride_c + x * 8 + j;
                    for (int k = 0; k < 10; k++) buf[k] = (k < 2 && !ht) ? 0 : p[(ptrdiff_t)(k - 2) * stride_c];
                    db_chroma_line(buf, cur, top, ht, j, false, T);
                    for (int k = ht ? 0 : 2; k < 10; k++) p[(ptrdiff_t)(k - 2) * stride_c] = (uint8_t)buf[k];
                }
            }
        }
}

}  // namespace h264
}  // namespace sk
