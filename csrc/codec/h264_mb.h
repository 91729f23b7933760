// Macroblock-level residual coding (transform, quant, decimation, QP
// escalation, reconstruction) shared by the CPU reference and, block by block,
// mirrored by the GPU kernels (see csrc/kernels/h264_kernels.hip).
#pragma once
#include "h264_syntax.h"

namespace sk {
namespace h264 {

// Forward-transformed residual of one macroblock, kept so that QP escalation can
// requantise without recomputing prediction/transform.
struct MbTransform {
    int wl[16][16];      // luma, blkIdx order, raster coefficients
    int wc[2][4][16];    // chroma [comp][blk]
};

SK_HD void residual_transform(const uint8_t* src_y, const uint8_t* pred_y, const uint8_t* src_u,
                              const uint8_t* pred_u, const uint8_t* src_v, const uint8_t* pred_v,
                              MbTransform& t) {
    for (int blk = 0; blk < 16; blk++) {
        int x0 = blk_x(blk) * 4, y0 = blk_y(blk) * 4;
        int r[16];
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++)
                r[y * 4 + x] = (int)src_y[(y0 + y) * 16 + x0 + x] - (int)pred_y[(y0 + y) * 16 + x0 + x];
        fdct4x4(r, t.wl[blk]);
    }
    for (int c = 0; c < 2; c++) {
        const uint8_t* s = c ? src_v : src_u;
        const uint8_t* p = c ? pred_v : pred_u;
        for (int b = 0; b < 4; b++) {
            int x0 = (b & 1) * 4, y0 = (b >> 1) * 4;
            int r[16];
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++)
                    r[y * 4 + x] = (int)s[(y0 + y) * 8 + x0 + x] - (int)p[(y0 + y) * 8 + x0 + x];
            fdct4x4(r, t.wc[c][b]);
        }
    }
}

SK_HD int i16_dc_fwd_round(int v) { return v >= 0 ? (v + 1) >> 1 : -((-v + 1) >> 1); }

// Quantise luma. intra16: Intra16x16 (DC separated), else inter 4x4 with decimation.
// Fills coef (kCoefLuma.., kCoefLumaDC..) and returns cbp luma bits (0..15).
SK_HD int quant_luma(const MbTransform& t, int qp, bool intra16, int16_t* coef, uint8_t* nnz) {
    int qbits = 15 + qp / 6;
    int f = quant_f(qbits, intra16);
    const int* mf = H264_QUANT_MF[qp % 6];
    if (intra16) {
        int dc[16], hd[16];
        for (int blk = 0; blk < 16; blk++) dc[blk_y(blk) * 4 + blk_x(blk)] = t.wl[blk][0];
        hadamard4x4(dc, hd);
        for (int k = 0; k < 16; k++)
            coef[kCoefLumaDC + k] =
                (int16_t)quant_coef(i16_dc_fwd_round(hd[zigzag4x4(k)]), mf[0], 2 * f, qbits + 1);
        bool any = false;
        for (int blk = 0; blk < 16; blk++) {
            int16_t* c = coef + kCoefLuma + blk * 16;
            c[0] = 0;
            for (int k = 1; k < 16; k++) {
                int pos = zigzag4x4(k);
                c[k] = (int16_t)quant_coef(t.wl[blk][pos], sel3(pos_class(pos), mf[0], mf[1], mf[2]), f, qbits);
                any |= c[k] != 0;
            }
        }
        for (int blk = 0; blk < 16; blk++)
            nnz[blk] = any ? (uint8_t)count_nonzero(coef + kCoefLuma + blk * 16 + 1, 15) : 0;
        return any ? 15 : 0;
    }
    int cbp = 0;
    int mb_score = 0;
    for (int k = 0; k < 16; k++) coef[kCoefLumaDC + k] = 0;
    for (int b8 = 0; b8 < 4; b8++) {
        int score8 = 0;
        for (int i = 0; i < 4; i++) {
            int blk = b8 * 4 + i;
            int16_t* c = coef + kCoefLuma + blk * 16;
            for (int k = 0; k < 16; k++) {
                int pos = zigzag4x4(k);
                c[k] = (int16_t)quant_coef(t.wl[blk][pos], sel3(pos_class(pos), mf[0], mf[1], mf[2]), f, qbits);
            }
            score8 += decimate_score(c, 16);
        }
        mb_score += score8;
        if (score8 >= 4) cbp |= 1 << b8;
    }
    if (mb_score < 6) cbp = 0;
    for (int blk = 0; blk < 16; blk++) {
        int16_t* c = coef + kCoefLuma + blk * 16;
        if (!(cbp & (1 << (blk >> 2)))) {
            for (int k = 0; k < 16; k++) c[k] = 0;
            nnz[blk] = 0;
        } else {
            nnz[blk] = (uint8_t)count_nonzero(c, 16);
        }
    }
    // an 8x8 whose four blocks quantised to zero is not coded
    for (int b8 = 0; b8 < 4; b8++) {
        if (!(cbp & (1 << b8))) continue;
        int n = nnz[b8 * 4] + nnz[b8 * 4 + 1] + nnz[b8 * 4 + 2] + nnz[b8 * 4 + 3];
        if (n == 0) cbp &= ~(1 << b8);
    }
    return cbp;
}

// Quantise chroma; returns cbp chroma (0, 1, 2).
SK_HD int quant_chroma(const MbTransform& t, int qp, bool intra, int16_t* coef, uint8_t* nnz) {
    int qpc = chroma_qp(qp);
    int qbits = 15 + qpc / 6;
    int f = quant_f(qbits, intra);
    const int* mf = H264_QUANT_MF[qpc % 6];
    bool any_dc = false, any_ac = false;
    for (int c = 0; c < 2; c++) {
        int d0 = t.wc[c][0][0], d1 = t.wc[c][1][0], d2 = t.wc[c][2][0], d3 = t.wc[c][3][0];
        int f2[4] = {d0 + d1 + d2 + d3, d0 - d1 + d2 - d3, d0 + d1 - d2 - d3, d0 - d1 - d2 + d3};
        for (int i = 0; i < 4; i++) {
            int l = quant_coef(f2[i], mf[0], 2 * f, qbits + 1);
            coef[kCoefChromaDC + c * 4 + i] = (int16_t)l;
            any_dc |= l != 0;
        }
        int score = 0;
        bool comp_ac = false;
        for (int b = 0; b < 4; b++) {
            int16_t* cc = coef + kCoefChromaAC + (c * 4 + b) * 16;
            cc[0] = 0;
            for (int k = 1; k < 16; k++) {
                int pos = zigzag4x4(k);
                cc[k] = (int16_t)quant_coef(t.wc[c][b][pos], sel3(pos_class(pos), mf[0], mf[1], mf[2]), f, qbits);
                comp_ac |= cc[k] != 0;
            }
            if (!intra) score += decimate_score(cc + 1, 15);
        }
        if (!intra && comp_ac && score < 7) {
            for (int b = 0; b < 4; b++)
                for (int k = 0; k < 16; k++) coef[kCoefChromaAC + (c * 4 + b) * 16 + k] = 0;
            comp_ac = false;
        }
        any_ac |= comp_ac;
    }
    int cbp_c = any_ac ? 2 : (any_dc ? 1 : 0);
    for (int b = 0; b < 8; b++)
        nnz[16 + b] = cbp_c == 2 ? (uint8_t)count_nonzero(coef + kCoefChromaAC + b * 16 + 1, 15) : 0;
    return cbp_c;
}

// Reconstruct the luma of a macroblock (16x16 raster) from its levels.
SK_HD void recon_luma(const int16_t* coef, int qp, bool intra16, int cbp_l, const uint8_t* pred,
                      uint8_t* rec) {
    int dcy[16];
    if (intra16) {
        int c[16];
        for (int k = 0; k < 16; k++) c[zigzag4x4(k)] = coef[kCoefLumaDC + k];
        i16_dc_dequant(c, dcy, qp);
    }
    for (int blk = 0; blk < 16; blk++) {
        int bx = blk_x(blk), by = blk_y(blk);
        int d[16];
        for (int i = 0; i < 16; i++) d[i] = 0;
        const int16_t* c = coef + kCoefLuma + blk * 16;
        bool coded = intra16 ? (cbp_l != 0) : ((cbp_l >> (blk >> 2)) & 1);
        if (coded)
            for (int k = intra16 ? 1 : 0; k < 16; k++) {
                int pos = zigzag4x4(k);
                d[pos] = dequant_coef(c[k], qp, pos);
            }
        if (intra16) d[0] = dcy[by * 4 + bx];
        int r[16];
        idct4x4(d, r);
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                int o = (by * 4 + y) * 16 + bx * 4 + x;
                rec[o] = (uint8_t)sk_clip255(pred[o] + r[y * 4 + x]);
            }
    }
}

SK_HD void recon_chroma(const int16_t* coef, int qp, int cbp_c, const uint8_t* pred_u,
                        const uint8_t* pred_v, uint8_t* rec_u, uint8_t* rec_v) {
    int qpc = chroma_qp(qp);
    for (int c = 0; c < 2; c++) {
        int lv[4], dcc[4];
        for (int i = 0; i < 4; i++) lv[i] = cbp_c ? coef[kCoefChromaDC + c * 4 + i] : 0;
        chroma_dc_dequant(lv, dcc, qpc);
        const uint8_t* p = c ? pred_v : pred_u;
        uint8_t* o = c ? rec_v : rec_u;
        for (int b = 0; b < 4; b++) {
            int d[16];
            for (int i = 0; i < 16; i++) d[i] = 0;
            if (cbp_c == 2) {
                const int16_t* cc = coef + kCoefChromaAC + (c * 4 + b) * 16;
                for (int k = 1; k < 16; k++) {
                    int pos = zigzag4x4(k);
                    d[pos] = dequant_coef(cc[k], qpc, pos);
                }
            }
            d[0] = dcc[b];
            int r[16];
            idct4x4(d, r);
            int x0 = (b & 1) * 4, y0 = (b >> 1) * 4;
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++) {
                    int idx = (y0 + y) * 8 + x0 + x;
                    o[idx] = (uint8_t)sk_clip255(p[idx] + r[y * 4 + x]);
                }
        }
    }
}

// Variance-based adaptive quantisation (MB-level AQ, the x264 aq-mode 1 idea in
// integer form, bit-identical on host and device): the QP offset of a macroblock is
// strength * (log2(E) - log2(E_ref)), E = luma AC energy sum(x^2) - sum(x)^2 / 256 of
// the 16x16 source block. Flat areas (gradients, backgrounds) get a lower QP, busy
// texture a higher one. log2 in Q2 from the leading bit and the next two; strength in
// Q4 (16 = 1.0); the result is clamped to [kAqMin, kAqMax].
constexpr int kAqRefQ2 = 58;     // log2(E_ref) = 14.5 (x264's 14.427)
constexpr int kAqMin = -6, kAqMax = 4;
SK_HD int aq_log2_q2(uint32_t v) {
    v += 1;
    const int e = 31 - __builtin_clz(v);
    const int frac = e >= 2 ? (int)((v >> (e - 2)) & 3u) : (int)((v << (2 - e)) & 3u);
    return 4 * e + frac;
}
SK_HD int aq_offset(uint32_t energy, int strength_q4) {
    const int d = ((aq_log2_q2(energy) - kAqRefQ2) * strength_q4 + 32) >> 6;   // Q2 * Q4 = Q6
    return d < kAqMin ? kAqMin : (d > kAqMax ? kAqMax : d);
}
// AC energy of a 16x16 luma block from its pixel sum and sum of squares.
SK_HD uint32_t aq_energy(uint32_t sum, uint32_t ssq) { return ssq - ((sum * sum) >> 8); }
// Start QP of a coded macroblock: slice QP + its AQ offset.
SK_HD int aq_start_qp(int slice_qp, int offset) {
    const int q = slice_qp + offset;
    return q < 0 ? 0 : (q > 51 ? 51 : q);
}

// Upper bound of the CAVLC bits of one non-zero level of magnitude a, over every
// suffixLength the block can reach (<= sl_max, 9.2.2.1). With per-TotalCoeff maxima for
// coeff_token / total_zeros and a 3n+8 bound on run_before this dominates the exact
// nC-free bound, so bound <= budget implies exact <= budget. (lc >> sl) + 1 + sl is
// convex in sl and the escape (28) region is a prefix of sl, so the maximum over
// sl in [1, sl_max] sits at an end point: two evaluations instead of six.
SK_HD int level_bits_bound(int a, int sl_max) {
    int lc = 2 * a - 1;
    int best = lc < 14 ? lc + 1 : (lc < 30 ? 19 : 28);
    const int b1 = lc < 30 ? (lc >> 1) + 2 : 28;
    const int bs = lc < (15 << sl_max) ? (lc >> sl_max) + 1 + sl_max : 28;
    return sk_max(best, sk_max(b1, bs));
}
SK_HD int suffix_len_cap(int maxabs) {
    return sk_min(6, 1 + (maxabs > 3) + (maxabs > 6) + (maxabs > 12) + (maxabs > 24) + (maxabs > 48));
}
// Conservative bits of one residual block (levels in scan order, maxn 16 or 15 = AC).
SK_HD int block_bits_crude(const int16_t* c, int maxn, const CavlcTables& T) {
    int n = 0, last = -1, mx = 0;
    for (int k = 0; k < 16; k++)
        if (c[k]) {
            n++;
            last = k;
            mx = sk_max(mx, sk_abs((int)c[k]));
        }
    if (n == 0) return 6;
    const int sl = suffix_len_cap(mx);
    int lv = 0;
    for (int k = 0; k < 16; k++)
        if (c[k]) lv += level_bits_bound(sk_abs((int)c[k]), sl);
    const int tz = (maxn == 16 ? last + 1 : last) - n;   // AC blocks (15) start at scan index 1
    int b = T.ct_max_tc[n] + lv;
    if (n < maxn) b += T.tz_len[n - 1][tz];
    if (n > 1 && tz > 0) b += tz <= 2 ? 2 * (n - 1) : (tz <= 6 ? 3 * (n - 1) : 3 * (n - 1) + 8);
    return b;
}
// Conservative macroblock size of an Intra16x16 MB (the same terms the lane-parallel
// GPU bound sums in quant_mb_lanes): 96 bits of header allowance, the AC blocks when
// coded, the luma DC block and the chroma blocks.
SK_HD int mb_bits_crude_i16(const MbInfo& mb, const int16_t* coef, const CavlcTables& T) {
    const int cbp_l = mb.cbp & 15, cbp_c = (mb.cbp >> 4) & 3;
    int total = 96;
    if (mb.type == MB_I4x4) {   // 16-coefficient luma blocks of the coded 8x8s, no luma DC block
        for (int b = 0; b < 16; b++)
            if (cbp_l & (1 << (b >> 2))) total += block_bits_crude(coef + kCoefLuma + b * 16, 16, T);
        if (cbp_c == 2)
            for (int b = 0; b < 8; b++) total += block_bits_crude(coef + kCoefChromaAC + b * 16, 15, T);
        if (cbp_c) {
            int n0 = 0, n1 = 0, cc = 0;
            for (int k = 0; k < 8; k++) {
                const int a = sk_abs((int)coef[kCoefChromaDC + k]);
                if (a) { (k < 4 ? n0 : n1)++; cc += level_bits_bound(a, 6) + 3; }
            }
            total += (n0 > 0 ? 11 : 2) + (n1 > 0 ? 11 : 2) + cc;
        }
        return total;
    }
    if (cbp_l)
        for (int b = 0; b < 16; b++) total += block_bits_crude(coef + kCoefLuma + b * 16, 15, T);
    if (cbp_c == 2)
        for (int b = 0; b < 8; b++) total += block_bits_crude(coef + kCoefChromaAC + b * 16, 15, T);
    int dn = 0, dc = 0;
    for (int k = 0; k < 16; k++) {
        const int a = sk_abs((int)coef[kCoefLumaDC + k]);
        if (a) { dn++; dc += level_bits_bound(a, 6) + 3; }
    }
    total += dn > 0 ? T.ct_max_tc[dn] + (dn < 16 ? T.tz_max_tc[dn] : 0) + 8 + dc : 6;
    if (cbp_c) {
        int n0 = 0, n1 = 0, cc = 0;
        for (int k = 0; k < 8; k++) {
            const int a = sk_abs((int)coef[kCoefChromaDC + k]);
            if (a) { (k < 4 ? n0 : n1)++; cc += level_bits_bound(a, 6) + 3; }
        }
        total += (n0 > 0 ? 11 : 2) + (n1 > 0 ? 11 : 2) + cc;
    }
    return total;
}

// Escalation threshold: the exact nC-free count of inter MBs is held to kMbBitBudget;
// the conservative bound of Intra16x16 MBs (header allowance 96 bits >= the <= 25 bits
// of an I16 header) may use the whole A.3.1 limit, since bound <= limit already implies
// compliance.
SK_HD int mb_bit_budget(bool intra16) { return intra16 ? kMaxMbBits : kMbBitBudget; }

// Quantise with QP escalation so a macroblock never exceeds the A.3.1 bit limit.
// Intra16x16 MBs (I slices: the keyframe wavefront) escalate on the conservative bound
// alone; inter MBs fall back to the exact nC-free CAVLC count when it is exceeded.
// Returns the final QP; fills mb.cbp / nnz and coef.
// `start_qp` is the first QP tried: the AQ start QP, or (intra) the QP the open-loop
// pre-pass already found to be needed.
SK_HD int quant_mb_with_budget(const MbTransform& t, int slice_qp, bool intra16, MbInfo& mb,
                               int16_t* coef, const CavlcTables& T, int start_qp = -1) {
    int qp = start_qp >= 0 ? start_qp : slice_qp;
    int qp_cap = sk_min(51, slice_qp + 24);
    for (;;) {
        int cbp_l = quant_luma(t, qp, intra16, coef, mb.nnz);
        int cbp_c = quant_chroma(t, qp, intra16, coef, mb.nnz);
        mb.cbp = (uint8_t)(cbp_l | (cbp_c << 4));
        mb.qp = (uint8_t)qp;
        if (qp + 6 > qp_cap) break;
        if ((intra16 ? mb_bits_crude_i16(mb, coef, T) : mb_bits_bound(mb, coef, T)) <= mb_bit_budget(intra16)) break;
        qp += 6;
    }
    return qp;
}

// ---------------------------------------------------------------------------
// Intra_4x4 (8.3.1): nine directional modes per 4x4 luma block, predicted mode from
// the left / top blocks, top-right availability by decoding order.
enum I4Mode { I4_V = 0, I4_H, I4_DC, I4_DDL, I4_DDR, I4_VR, I4_HD, I4_VL, I4_HU };

// Neighbour samples of one 4x4 block: t[0..7] = p[0..7, -1] (p[4..7, -1] replaced by
// p[3, -1] when the top-right block is not decoded yet), l[0..3] = p[-1, 0..3], m = p[-1, -1].
struct I4Ref {
    int t[8], l[4], m;
    bool hasT, hasL;
    SK_HD int T(int i) const { return i < 0 ? m : t[i]; }   // p[i, -1], i = -1..7
    SK_HD int L(int i) const { return i < 0 ? m : l[i]; }   // p[-1, i], i = -1..3
};
// The same samples packed in 13 bytes (p[0] corner, p[1..8] top, p[9..12] left), e.g. in
// LDS on the GPU, so a lane-dependent index never lands in a private array.
struct I4RefView {
    const uint8_t* p;
    bool hasT, hasL;
    SK_HD int T(int i) const { return p[1 + i]; }
    SK_HD int L(int i) const { return i < 0 ? p[0] : p[9 + i]; }
};

// p[4..7, -1] of block b exists: above MB for blocks 0, 1, 4; above-right MB for 5;
// inside the MB only when that block precedes b in decoding order.
SK_HD bool i4_tr_avail(int b, bool aT, bool aTR) {
    if (b == 0 || b == 1 || b == 4) return aT;
    if (b == 5) return aTR;
    return !(b == 3 || b == 7 || b == 11 || b == 13 || b == 15);
}
SK_HD bool i4_mode_ok(int m, bool hasT, bool hasL) {
    if (m == I4_V || m == I4_DDL || m == I4_VL) return hasT;
    if (m == I4_H || m == I4_HU) return hasL;
    if (m == I4_DC) return true;
    return hasT && hasL;   // DDR, VR, HD also read p[-1, -1]
}
SK_HD bool i4_has_top(int b, bool aT) { return blk_y(b) > 0 || aT; }
SK_HD bool i4_has_left(int b, bool aL) { return blk_x(b) > 0 || aL; }

// Reference sample k (I4RefView packing) of block b; sample(x, y) reads MB-relative luma.
template <class S>
SK_HD int i4_ref_sample(S sample, int b, bool aT, bool aL, bool aTR, int k) {
    const int bx = blk_x(b) * 4, by = blk_y(b) * 4;
    const bool hasT = i4_has_top(b, aT), hasL = i4_has_left(b, aL);
    if (k == 0) return (hasT && hasL) ? sample(bx - 1, by - 1) : 0;
    if (k <= 8) {
        int i = k - 1;
        if (!hasT) return 0;
        if (i >= 4 && !i4_tr_avail(b, aT, aTR)) i = 3;
        return sample(bx + i, by - 1);
    }
    return hasL ? sample(bx - 1, by + k - 9) : 0;
}

// Reference samples of block b; sample(x, y) reads MB-relative luma (x, y >= -1).
template <class S>
SK_HD void i4_ref(S sample, int b, bool aT, bool aL, bool aTR, I4Ref& r) {
    r.hasT = i4_has_top(b, aT);
    r.hasL = i4_has_left(b, aL);
    r.m = i4_ref_sample(sample, b, aT, aL, aTR, 0);
    for (int i = 0; i < 8; i++) r.t[i] = i4_ref_sample(sample, b, aT, aL, aTR, 1 + i);
    for (int i = 0; i < 4; i++) r.l[i] = i4_ref_sample(sample, b, aT, aL, aTR, 9 + i);
}

// Prediction sample (x, y) of mode m (8.3.1.2.1 - 8.3.1.2.9); R gives T(i) = p[i, -1]
// (i = -1..7), L(i) = p[-1, i] (i = -1..3) and the hasT / hasL flags.
template <class R>
SK_HD int i4_pred_px(int m, const R& r, int x, int y) {
    switch (m) {
        case I4_V: return r.T(x);
        case I4_H: return r.L(y);
        case I4_DC:
            if (r.hasT && r.hasL)
                return (r.T(0) + r.T(1) + r.T(2) + r.T(3) + r.L(0) + r.L(1) + r.L(2) + r.L(3) + 4) >> 3;
            if (r.hasL) return (r.L(0) + r.L(1) + r.L(2) + r.L(3) + 2) >> 2;
            if (r.hasT) return (r.T(0) + r.T(1) + r.T(2) + r.T(3) + 2) >> 2;
            return 128;
        case I4_DDL:
            if (x == 3 && y == 3) return (r.T(6) + 3 * r.T(7) + 2) >> 2;
            return (r.T(x + y) + 2 * r.T(x + y + 1) + r.T(x + y + 2) + 2) >> 2;
        case I4_DDR:
            if (x > y) return (r.T(x - y - 2) + 2 * r.T(x - y - 1) + r.T(x - y) + 2) >> 2;
            if (x < y) return (r.L(y - x - 2) + 2 * r.L(y - x - 1) + r.L(y - x) + 2) >> 2;
            return (r.T(0) + 2 * r.T(-1) + r.L(0) + 2) >> 2;
        case I4_VR: {
            const int z = 2 * x - y, k = x - (y >> 1);
            if (z >= 0)
                return (z & 1) ? (r.T(k - 2) + 2 * r.T(k - 1) + r.T(k) + 2) >> 2 : (r.T(k - 1) + r.T(k) + 1) >> 1;
            if (z == -1) return (r.L(0) + 2 * r.T(-1) + r.T(0) + 2) >> 2;
            return (r.L(y - 1) + 2 * r.L(y - 2) + r.L(y - 3) + 2) >> 2;
        }
        case I4_HD: {
            const int z = 2 * y - x, k = y - (x >> 1);
            if (z >= 0)
                return (z & 1) ? (r.L(k - 2) + 2 * r.L(k - 1) + r.L(k) + 2) >> 2 : (r.L(k - 1) + r.L(k) + 1) >> 1;
            if (z == -1) return (r.L(0) + 2 * r.T(-1) + r.T(0) + 2) >> 2;
            return (r.T(x - 1) + 2 * r.T(x - 2) + r.T(x - 3) + 2) >> 2;
        }
        case I4_VL: {
            const int k = x + (y >> 1);
            return (y & 1) ? (r.T(k) + 2 * r.T(k + 1) + r.T(k + 2) + 2) >> 2 : (r.T(k) + r.T(k + 1) + 1) >> 1;
        }
        default: {   // I4_HU
            const int z = x + 2 * y, k = y + (x >> 1);
            if (z > 5) return r.L(3);
            if (z == 5) return (r.L(2) + 3 * r.L(3) + 2) >> 2;
            return (z & 1) ? (r.L(k) + 2 * r.L(k + 1) + r.L(k + 2) + 2) >> 2 : (r.L(k) + r.L(k + 1) + 1) >> 1;
        }
    }
}

// SAD cost weight of the mode bits (1 bit when the mode equals the predicted one, else 4).
SK_HD int i4_lambda(int qp) { return 1 << ((qp > 12 ? qp - 12 : 0) / 6); }

// Open-loop Intra4x4 decision over SOURCE samples (the pre-pass, every MB on its own):
// per block in decoding order the mode of least SAD + lambda * mode bits, the predicted
// mode taken from the blocks already decided in this MB (DC for neighbours in other
// MBs). Returns the summed cost and fills the modes of `mb`.
template <class S>
SK_HD int i4_decide(S src, const uint8_t* sy, bool aT, bool aL, bool aTR, int qp, MbInfo& mb) {
    const int lam = i4_lambda(qp);
    MbInfo sideL, sideT;   // stand-ins for the neighbour MBs: any non-Intra4x4 type counts as DC
    sideL.type = sideT.type = MB_I16x16;
    int total = 0;
    for (int b = 0; b < 16; b++) {
        I4Ref r;
        i4_ref(src, b, aT, aL, aTR, r);
        const int pm = i4_predicted(i4_left_mode(mb, aL ? &sideL : nullptr, b), i4_top_mode(mb, aT ? &sideT : nullptr, b));
        const int bx = blk_x(b) * 4, by = blk_y(b) * 4;
        int best = 0x7fffffff, bm = I4_DC;
        for (int m = 0; m < 9; m++) {
            if (!i4_mode_ok(m, r.hasT, r.hasL)) continue;
            int cost = lam * (m == pm ? 1 : 4);
            for (int y = 0; y < 4; y++)
                for (int x = 0; x < 4; x++) cost += sk_abs((int)sy[(by + y) * 16 + bx + x] - i4_pred_px(m, r, x, y));
            if (cost < best) { best = cost; bm = m; }
        }
        set_i4_mode(mb, b, bm);
        total += best;
    }
    return total;
}
// Intra4x4 wins over the best Intra16x16 SAD when clearly cheaper (its header is larger).
SK_HD bool i4_wins(int cost4, int sad16, int qp) { return cost4 + 8 * i4_lambda(qp) < sad16; }

// One Intra4x4 luma block: quantise the raster transform w into scan-order levels c
// (intra rounding, all 16 coefficients, no decimation); returns TotalCoeff.
SK_HD int quant_block_i4(const int* w, int qp, int16_t* c) {
    const int qbits = 15 + qp / 6, f = quant_f(qbits, true);
    const int* mf = H264_QUANT_MF[qp % 6];
    int n = 0;
    for (int k = 0; k < 16; k++) {
        const int pos = zigzag4x4(k);
        c[k] = (int16_t)quant_coef(w[pos], sel3(pos_class(pos), mf[0], mf[1], mf[2]), f, qbits);
        n += c[k] != 0;
    }
    return n;
}
// Reconstruction of one Intra4x4 block from its levels: rec = clip(pred + residual).
SK_HD void recon_block_i4(const int16_t* c, int qp, const int* pred, int* rec) {
    int d[16], r[16];
    for (int k = 0; k < 16; k++) {
        const int pos = zigzag4x4(k);
        d[pos] = dequant_coef(c[k], qp, pos);
    }
    idct4x4(d, r);
    for (int i = 0; i < 16; i++) rec[i] = sk_clip255(pred[i] + r[i]);
}

}  // namespace h264
}  // namespace sk
