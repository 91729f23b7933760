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

// One line across an edge: q0 at `q0p`, p_i = q0p[-(i + 1) * step], q_i = q0p[i * step]
// (7.14.6: filter mask, narrow / wide filter).
SK_HD void lf_line(uint8_t* q0p, int step, int filter_size, int plane, int lvl) {
    const int len = filter_size == 4 ? 4 : (plane ? 6 : (filter_size == 8 ? 8 : 16));
    const int rd = len == 4 ? 2 : (len == 6 ? 3 : (len == 8 ? 4 : 7));   // samples read per side
    int P[7] = {0, 0, 0, 0, 0, 0, 0}, Q[7] = {0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < rd; i++) {
        P[i] = q0p[-(i + 1) * step];
        Q[i] = q0p[i * step];
    }
    const int limit = lvl > 1 ? lvl : 1;   // sharpness 0
    const int blimit = 2 * (lvl + 2) + limit, thresh = lvl >> 4;
    const bool hev = sk_abs(P[1] - P[0]) > thresh || sk_abs(Q[1] - Q[0]) > thresh;
    bool mask = sk_abs(P[1] - P[0]) <= limit && sk_abs(Q[1] - Q[0]) <= limit &&
                sk_abs(P[0] - Q[0]) * 2 + (sk_abs(P[1] - Q[1]) >> 1) <= blimit;
    if (len >= 6) mask = mask && sk_abs(P[2] - P[1]) <= limit && sk_abs(Q[2] - Q[1]) <= limit;
    if (len >= 8) mask = mask && sk_abs(P[3] - P[2]) <= limit && sk_abs(Q[3] - Q[2]) <= limit;
    if (!mask) return;
    bool flat = false, flat2 = false;
    if (len >= 6) {
        flat = sk_abs(P[1] - P[0]) <= 1 && sk_abs(Q[1] - Q[0]) <= 1 && sk_abs(P[2] - P[0]) <= 1 && sk_abs(Q[2] - Q[0]) <= 1;
        if (len >= 8) flat = flat && sk_abs(P[3] - P[0]) <= 1 && sk_abs(Q[3] - Q[0]) <= 1;
    }
    if (len == 16)
        flat2 = sk_abs(P[6] - P[0]) <= 1 && sk_abs(Q[6] - Q[0]) <= 1 && sk_abs(P[5] - P[0]) <= 1 &&
                sk_abs(Q[5] - Q[0]) <= 1 && sk_abs(P[4] - P[0]) <= 1 && sk_abs(Q[4] - Q[0]) <= 1;
    if (len == 4 || !flat) {   // narrow filter (7.14.6.3)
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
    // wide filter (7.14.6.4): log2Size 3 (6-tap chroma, 8-tap luma) or 4 (14-tap luma)
    const int log2 = (len == 16 && flat2) ? 4 : 3;
    const int n = log2 == 4 ? 6 : (plane == 0 ? 3 : 2);
    const int n2 = (log2 == 3 && plane == 0) ? 0 : 1;
    auto smp = [&](int k) { return k >= 0 ? Q[k] : P[-k - 1]; };
    int out[12];
    for (int i = -n; i < n; i++) {
        int t = 0;
        for (int j = -n; j <= n; j++) {
            const int p = sk_clip(i + j, -(n + 1), n);
            t += smp(p) * (sk_abs(j) <= n2 ? 2 : 1);
        }
        out[i + n] = (t + (1 << (log2 - 1))) >> log2;
    }
    for (int i = -n; i < n; i++) q0p[i * step] = (uint8_t)out[i + n];
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
    return f.lvl[plane == 0 ? pass : plane + 1];
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
