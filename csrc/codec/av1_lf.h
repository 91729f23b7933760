// AV1 in-loop deblocking filter (spec 7.14) shared by the CPU reference (av1_cpu.cpp)
// and the gfx950 kernel k_av1_lf (av1_kernels.hip): edge decisions, filter masks, the
// narrow (4-tap) and wide (6 / 8 / 14-tap) filters, and the encoder's level choice.
//
// The encoder's structure makes the edge set simple: TX_MODE_LARGEST with square blocks
// means every transform edge is a block edge (and vice versa), so applyFilter is "on a
// block edge"; sharpness is 0, no segmentation. The frame header enables the level
// deltas with ref delta INTRA = 0 and mode delta[0] = -63: GLOBALMV inter blocks (the
// static desktop, zero global motion) get level 0, so unchanged content is not filtered
// again every frame (AV1 filters skip-block edges too; HEVC's bS 0 has no counterpart).
// Within one pass two edges never touch the same samples (a filter reaches at most half the smaller transform on each
// side), so all edges of a pass can run in parallel and equal the raster order.
#pragma once
#include "av1_core.h"

namespace sk {
namespace av1 {

// Encoder choice: libaom's 8-bit LPF_PICK_FROM_Q fit from the AC quantiser step.
SK_HD int lf_level_for(int ac_q, bool key) {
    const long long v = key ? (long long)ac_q * 17563 - 421574 : (long long)ac_q * 6017 + 650707;
    return sk_clip((int)((v + (1 << 17)) >> 18), 0, 63);
}

SK_HD int lf_clamp8(int v) { return sk_clip(v, -128, 127); }

// Wide filter (7.14.6.4) over the samples read: N taps a side (6 for the 14-tap luma
// filter, 3 for 8-tap luma, 2 for 6-tap chroma), centre weight 2 for |j| <= N2.
template <int N, int N2, int LOG2>
SK_HD void lf_wide(const int* P, const int* Q, uint8_t* q0p, int step) {
    int out[2 * N];
#pragma unroll
    for (int i = -N; i < N; i++) {
        int t = 0;
#pragma unroll
        for (int j = -N; j <= N; j++) {
            const int p = sk_clip(i + j, -(N + 1), N);
            t += (p >= 0 ? Q[p] : P[-p - 1]) * (sk_abs(j) <= N2 ? 2 : 1);
        }
        out[i + N] = (t + (1 << (LOG2 - 1))) >> LOG2;
    }
#pragma unroll
    for (int i = -N; i < N; i++) q0p[i * step] = (uint8_t)out[i + N];
}

// One line across an edge: q0 at `q0p`, p_i = q0p[-(i + 1) * step], q_i = q0p[i * step]
// (7.14.6: filter mask, narrow / wide filter). LEN = filterLen (4, 6 chroma, 8, 16); the
// template keeps every sample in registers (compile-time indices) on the GPU.
template <int LEN>
SK_HD void lf_line_t(uint8_t* q0p, int step, int lvl) {
    constexpr int RD = LEN == 4 ? 2 : (LEN == 6 ? 3 : (LEN == 8 ? 4 : 7));   // samples read per side
    int P[7], Q[7];
#pragma unroll
    for (int i = 0; i < 7; i++) {
        P[i] = i < RD ? q0p[-(i + 1) * step] : 0;
        Q[i] = i < RD ? q0p[i * step] : 0;
    }
    const int limit = lvl > 1 ? lvl : 1;   // sharpness 0
    const int blimit = 2 * (lvl + 2) + limit, thresh = lvl >> 4;
    const bool hev = sk_abs(P[1] - P[0]) > thresh || sk_abs(Q[1] - Q[0]) > thresh;
    bool mask = sk_abs(P[1] - P[0]) <= limit && sk_abs(Q[1] - Q[0]) <= limit &&
                sk_abs(P[0] - Q[0]) * 2 + (sk_abs(P[1] - Q[1]) >> 1) <= blimit;
    if (LEN >= 6) mask = mask && sk_abs(P[2] - P[1]) <= limit && sk_abs(Q[2] - Q[1]) <= limit;
    if (LEN >= 8) mask = mask && sk_abs(P[3] - P[2]) <= limit && sk_abs(Q[3] - Q[2]) <= limit;
    if (!mask) return;
    bool flat = false, flat2 = false;
    if (LEN >= 6) {
        flat = sk_abs(P[1] - P[0]) <= 1 && sk_abs(Q[1] - Q[0]) <= 1 && sk_abs(P[2] - P[0]) <= 1 && sk_abs(Q[2] - Q[0]) <= 1;
        if (LEN >= 8) flat = flat && sk_abs(P[3] - P[0]) <= 1 && sk_abs(Q[3] - Q[0]) <= 1;
    }
    if (LEN == 16)
        flat2 = sk_abs(P[6] - P[0]) <= 1 && sk_abs(Q[6] - Q[0]) <= 1 && sk_abs(P[5] - P[0]) <= 1 &&
                sk_abs(Q[5] - Q[0]) <= 1 && sk_abs(P[4] - P[0]) <= 1 && sk_abs(Q[4] - Q[0]) <= 1;
    if (LEN == 4 || !flat) {   // narrow filter (7.14.6.3)
        const int ps1 = P[1] - 128, ps0 = P[0] - 128, qs0 = Q[0] - 128, qs1 = Q[1] - 128;
        int f = hev ? lf_clamp8(ps1 - qs1) : 0;
        f = lf_clamp8(f + 3 * (qs0 - ps0));
        const int f1 = lf_clamp8(f + 4) >> 3, f2 = lf_clamp8(f + 3) >> 3;
        q0p[0] = (uint8_t)(lf_clamp8(qs0 - f1) + 128);
        q0p[-step] = (uint8_t)(lf_clamp8(ps0 + f2) + 128);
        if (!hev) {
            const int g = (f1 + 1) >> 1;   // Round2(filter1, 1)
            q0p[step] = (uint8_t)(lf_clamp8(qs1 - g) + 128);
            q0p[-2 * step] = (uint8_t)(lf_clamp8(ps1 + g) + 128);
        }
        return;
    }
    if (LEN == 6) lf_wide<2, 1, 3>(P, Q, q0p, step);              // 6-tap chroma
    else if (LEN == 8 || !flat2) lf_wide<3, 0, 3>(P, Q, q0p, step);   // 8-tap luma
    else lf_wide<6, 1, 4>(P, Q, q0p, step);                        // 14-tap luma
}
SK_HD void lf_line(uint8_t* q0p, int step, int filter_size, int plane, int lvl) {
    if (filter_size == 4) lf_line_t<4>(q0p, step, lvl);
    else if (plane) lf_line_t<6>(q0p, step, lvl);
    else if (filter_size == 8) lf_line_t<8>(q0p, step, lvl);
    else lf_line_t<16>(q0p, step, lvl);
}

// Filter geometry of the frame: the 8x8 block map (bsl = Mi_Width_Log2 of the block
// covering the cell) and the frame size in luma samples.
struct LfFrame {
    const BlkInfo* blk;
    int c8, mi_rows, mi_cols, W, H;
    int lvl[4];   // loop_filter_level[0..3]: luma vertical, luma horizontal, U, V
};

// Filter level of a block (7.14.4 with the deltas above): 0 for GLOBALMV inter blocks.
SK_HD int lf_block_level(const LfFrame& f, const BlkInfo& b, int plane, int pass) {
    if (blk_inter(b) && b.mode == GLOBALMV) return 0;
    // selected, not indexed: a run-time index into lvl[] keeps the LfFrame in GPU scratch
    const int k = plane == 0 ? pass : plane + 1;
    return k == 0 ? f.lvl[0] : (k == 1 ? f.lvl[1] : (k == 2 ? f.lvl[2] : f.lvl[3]));
}

// edge_loop_filter (7.14.2) of MI (row, col) for one plane / pass: the four lines of the
// edge on the MI's left (pass 0) or top (pass 1) boundary.
SK_HD void lf_edge(const LfFrame& f, int plane, int pass, int row, int col, uint8_t* buf, int stride) {
    const int ss = plane ? 1 : 0;
    const int x = col * 4, y = row * 4;
    if (x >= f.W || y >= f.H || (pass == 0 ? x == 0 : y == 0)) return;
    row |= ss;
    col |= ss;
    const int prow = row - (pass == 1 ? (1 << ss) : 0), pcol = col - (pass == 0 ? (1 << ss) : 0);
    const BlkInfo& b = f.blk[(size_t)(row >> 1) * f.c8 + (col >> 1)];
    const BlkInfo& pb = f.blk[(size_t)(prow >> 1) * f.c8 + (pcol >> 1)];
    int lvl = lf_block_level(f, b, plane, pass);
    if (lvl == 0) lvl = lf_block_level(f, pb, plane, pass);   // the previous block's level
    if (lvl == 0) return;
    const int bw = (4 << b.bsl) >> ss;    // = transform size
    const int pbw = (4 << pb.bsl) >> ss;
    const int xp = x >> ss, yp = y >> ss;
    if ((pass == 0 ? xp : yp) % bw) return;   // not a transform (= block) edge
    const int base = sk_min(bw, pbw);
    const int fs = plane ? sk_min(8, base) : sk_min(16, base);
    for (int i = 0; i < 4; i++) {
        uint8_t* q0 = pass == 0 ? buf + (size_t)(yp + i) * stride + xp : buf + (size_t)yp * stride + xp + i;
        lf_line(q0, pass == 0 ? 1 : stride, fs, plane, lvl);
    }
}

}  // namespace av1
}  // namespace sk
