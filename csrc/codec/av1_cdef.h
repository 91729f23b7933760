// AV1 constrained directional enhancement filter (CDEF, spec 7.15) shared by the CPU
// reference (av1_cpu.cpp) and the gfx950 kernel k_av1_cdef (av1_kernels.hip).
//
// One strength set per frame (cdef_bits = 0), so no per-superblock syntax is coded: a
// 64x64 superblock is filtered when any of its blocks is not skipped (cdef_idx 0, else
// -1), and within it every 8x8 block that is not entirely skipped. The filter reads the
// deblocked picture and writes the output picture; its taps reach 2 samples (luma) /
// 2 samples (chroma) around each block, unavailable only outside the MiRows x MiCols
// area (CDEF crosses tile and slice boundaries).
#pragma once
#include "av1_core.h"

namespace sk {
namespace av1 {

struct CdefParams {
    int damping;              // CdefDamping = cdef_damping_minus_3 + 3
    int y_pri, y_sec;         // strengths (sec 0, 1, 2 or 4)
    int uv_pri, uv_sec;
};

// Encoder choice, from the AC quantiser step (a coarse fit of libaom's CDEF_PICK_FROM_Q).
SK_HD CdefParams cdef_choose(int qidx, int ac_q) {
    CdefParams p;
    p.damping = 3 + (qidx >> 6);
    p.y_pri = sk_clip((ac_q + 75) / 150, 0, 15);
    const int ys = sk_clip(ac_q / 400, 0, 3);
    p.y_sec = ys == 3 ? 4 : ys;
    p.uv_pri = sk_clip((ac_q + 150) / 300, 0, 15);
    p.uv_sec = 0;
    return p;
}
SK_HD bool cdef_on(const CdefParams& p) { return (p.y_pri | p.y_sec | p.uv_pri | p.uv_sec) != 0; }

SK_HD int floor_log2(int v) {
    int n = 0;
    while (v > 1) { v >>= 1; n++; }
    return n;
}

// Direction search (7.15.2) in two steps: the line sums `partial` of the 8x8 luma block
// (cdef_partial_index: where pixel (i, j) adds in line set d; order-independent, so the GPU
// accumulates them lane-parallel), then the costs and the best direction.
SK_HD int cdef_partial_index(int d, int i, int j) {
    switch (d) {
        case 0: return i + j;
        case 1: return i + j / 2;
        case 2: return i;
        case 3: return 3 + i - j / 2;
        case 4: return 7 + i - j;
        case 5: return 3 - i / 2 + j;
        case 6: return j;
        default: return i / 2 + j;
    }
}
// Div_Table and Cdef_Directions[dir][k] = (row, col) offsets of the k-th primary tap, in
// constant memory on the GPU (a function-local table would live in scratch).
SK_TABLE int32_t CDEF_DIV[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};
SK_TABLE int8_t CDEF_DIRS[8][2][2] = {{{-1, 1}, {-2, 2}}, {{0, 1}, {-1, 2}}, {{0, 1}, {0, 2}}, {{0, 1}, {1, 2}},
                                      {{1, 1}, {2, 2}},   {{1, 0}, {2, 1}},  {{1, 0}, {2, 0}}, {{1, 0}, {2, -1}}};

// Cost of direction d from the line sums (the spec's cost[d]).
SK_HD long long cdef_dir_cost(const int (*partial)[15], int d) {
    const int32_t* div_table = CDEF_DIV;
    long long c = 0;
    if (d == 2 || d == 6) {
        for (int i = 0; i < 8; i++) c += (long long)partial[d][i] * partial[d][i];
        c *= div_table[8];
    } else if (d == 0 || d == 4) {
        for (int i = 0; i < 7; i++)
            c += ((long long)partial[d][i] * partial[d][i] + (long long)partial[d][14 - i] * partial[d][14 - i]) *
                 div_table[i + 1];
        c += (long long)partial[d][7] * partial[d][7] * div_table[8];
    } else {
        for (int j = 0; j < 5; j++) c += (long long)partial[d][3 + j] * partial[d][3 + j];
        c *= div_table[8];
        for (int j = 0; j < 3; j++)
            c += ((long long)partial[d][j] * partial[d][j] + (long long)partial[d][10 - j] * partial[d][10 - j]) *
                 div_table[2 * j + 2];
    }
    return c;
}
// Best direction (first maximum) and var from the eight costs.
SK_HD int cdef_pick_dir(const long long* cost, int* var) {
    long long best = 0;
    int dir = 0;
    for (int i = 0; i < 8; i++)
        if (cost[i] > best) { best = cost[i]; dir = i; }
    *var = (int)((best - cost[(dir + 4) & 7]) >> 10);
    return dir;
}
SK_HD int cdef_dir_from_partials(const int (*partial)[15], int* var) {
    long long cost[8];
    for (int d = 0; d < 8; d++) cost[d] = cdef_dir_cost(partial, d);
    return cdef_pick_dir(cost, var);
}
// Direction of the luma 8x8 block at `src`: returns yDir, writes var.
SK_HD int cdef_find_dir(const uint8_t* src, int stride, int* var) {
    int partial[8][15];
    for (int d = 0; d < 8; d++)
        for (int k = 0; k < 15; k++) partial[d][k] = 0;
    for (int i = 0; i < 8; i++)
        for (int j = 0; j < 8; j++) {
            const int x = (int)src[(size_t)i * stride + j] - 128;
            for (int d = 0; d < 8; d++) partial[d][cdef_partial_index(d, i, j)] += x;
        }
    return cdef_dir_from_partials(partial, var);
}

SK_HD int cdef_constrain(int diff, int threshold, int damping) {
    if (!threshold) return 0;
    const int adj = sk_max(0, damping - floor_log2(threshold));
    const int a = sk_abs(diff);
    const int v = sk_min(a, sk_max(0, threshold - (a >> adj)));
    return diff < 0 ? -v : v;
}

SK_HD int cdef_dir_off(int dir, int k, int rc) { return CDEF_DIRS[dir][k][rc]; }

// cdef_filter (7.15.3) of sample (i, j) of the 8x8 (luma) / 4x4 (chroma) block at plane
// position (x0, y0): reads `in` (the deblocked plane), returns the output sample.
// mi_rows / mi_cols bound availability.
SK_HD int cdef_filter_px(const uint8_t* in, int in_stride, int ss, int x0, int y0, int i, int j, int pri, int sec,
                         int damping, int dir, int mi_rows, int mi_cols) {
    const int pt0 = (pri & 1) ? 3 : 4, pt1 = (pri & 1) ? 3 : 2;   // Cdef_Pri_Taps[(priStr >> 0) & 1]
    {
        {
            const int x = in[(size_t)(y0 + i) * in_stride + x0 + j];
            int sum = 0, mx = x, mn = x;
            auto tap = [&](int d, int k, int sign, int* v) {
                const int yy = y0 + i + sign * cdef_dir_off(d, k, 0), xx = x0 + j + sign * cdef_dir_off(d, k, 1);
                const int cr = (yy << ss) >> 2, cc = (xx << ss) >> 2;
                if (yy < 0 || xx < 0 || cr >= mi_rows || cc >= mi_cols) return false;   // CdefAvailable = 0
                *v = in[(size_t)yy * in_stride + xx];
                return true;
            };
            for (int k = 0; k < 2; k++)
                for (int sign = -1; sign <= 1; sign += 2) {
                    int p;
                    if (tap(dir, k, sign, &p)) {
                        sum += (k ? pt1 : pt0) * cdef_constrain(p - x, pri, damping);
                        mx = sk_max(p, mx);
                        mn = sk_min(p, mn);
                    }
                    for (int off = -2; off <= 2; off += 4) {
                        int s;
                        if (tap((dir + off) & 7, k, sign, &s)) {
                            sum += (k ? 1 : 2) * cdef_constrain(s - x, sec, damping);   // Cdef_Sec_Taps
                            mx = sk_max(s, mx);
                            mn = sk_min(s, mn);
                        }
                    }
                }
            return sk_clip(x + ((8 + sum - (sum < 0)) >> 4), mn, mx);
        }
    }
}
SK_HD void cdef_filter_block(const uint8_t* in, int in_stride, uint8_t* out, int out_stride, int ss, int x0, int y0,
                             int pri, int sec, int damping, int dir, int mi_rows, int mi_cols) {
    const int n = 8 >> ss;
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            out[(size_t)(y0 + i) * out_stride + x0 + j] =
                (uint8_t)cdef_filter_px(in, in_stride, ss, x0, y0, i, j, pri, sec, damping, dir, mi_rows, mi_cols);
}
// Luma strength and direction of the block from the search (7.15.1): the primary
// strength is scaled by the block's variance; dir is 0 when the frame's strength is 0.
SK_HD void cdef_luma_setup(const CdefParams& p, int ydir, int var, int* pri, int* dir) {
    *dir = p.y_pri == 0 ? 0 : ydir;
    const int vs = (var >> 6) ? sk_min(floor_log2(var >> 6), 12) : 0;
    *pri = var ? (p.y_pri * (4 + vs) + 8) >> 4 : 0;
}

// Whether the 64x64 superblock at MI (sr, sc) has a block that is not skipped (read_cdef
// then sets cdef_idx to 0; otherwise it stays -1 and the superblock is not filtered).
SK_HD bool cdef_sb_on(const BlkInfo* blk, const Av1Geo& g, int sr, int sc) {
    for (int r = sr; r < sr + 16 && r < g.mi_rows; r += 2)
        for (int c = sc; c < sc + 16 && c < g.mi_cols; c += 2)
            if (!blk_skip(blk[(size_t)(r >> 1) * g.c8 + (c >> 1)])) return true;
    return false;
}

// CDEF of the 8x8 luma block at MI (r, c) (its 4:2:0 chroma too) given the superblock
// decision (sb_on: some block of the 64x64 is not skipped) and the four MIs' skip flags.
SK_HD void cdef_block(const uint8_t* const* in, const int* in_stride, uint8_t* const* out, const int* out_stride,
                      const CdefParams& p, int r, int c, bool all_skip, int mi_rows, int mi_cols) {
    if (all_skip) return;
    int var = 0;
    const int ydir = cdef_find_dir(in[0] + (size_t)(r * 4) * in_stride[0] + c * 4, in_stride[0], &var);
    int pri, dir;
    cdef_luma_setup(p, ydir, var, &pri, &dir);
    cdef_filter_block(in[0], in_stride[0], out[0], out_stride[0], 0, c * 4, r * 4, pri, p.y_sec, p.damping, dir,
                      mi_rows, mi_cols);
    const int udir = p.uv_pri == 0 ? 0 : ydir;   // Cdef_Uv_Dir for 4:2:0 is the identity
    for (int pl = 1; pl < 3; pl++)
        cdef_filter_block(in[pl], in_stride[pl], out[pl], out_stride[pl], 1, c * 2, r * 2, p.uv_pri, p.uv_sec,
                          p.damping - 1, udir, mi_rows, mi_cols);
}

}  // namespace av1
}  // namespace sk
