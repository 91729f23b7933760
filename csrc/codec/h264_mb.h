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

// Quantise with QP escalation so a macroblock never exceeds the A.3.1 bit limit.
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
        if (mb_bits_bound(mb, coef, T) <= kMbBitBudget) break;
        qp += 6;
    }
    return qp;
}

}  // namespace h264
}  // namespace sk
