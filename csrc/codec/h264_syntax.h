// H.264 syntax writers (7.3): macroblock_layer for CAVLC Constrained Baseline,
// slice header, neighbour-dependent nC derivation. SK_HD so the GPU entropy
// kernel and the CPU reference share one definition of the bitstream.
#pragma once
#include "h264_core.h"

namespace sk {
namespace h264 {

constexpr int kLog2MaxFrameNum = 16;

struct SliceHeaderParams {
    int first_mb;
    int slice_type;   // 0 = P, 2 = I
    int idr;          // nal_unit_type 5
    int frame_num;
    int idr_pic_id;
    int slice_qp;
    int deblock;      // 1: filter inside the slice (idc 2), 0: filter off (idc 1)
    int num_refs;     // P: active references (> 1 overrides the PPS default of 1)
};

template <class W>
SK_HD void write_slice_header(W& w, const SliceHeaderParams& h) {
    put_ue(w, (uint32_t)h.first_mb);
    put_ue(w, (uint32_t)h.slice_type);
    put_ue(w, 0);  // pic_parameter_set_id
    w.put((uint32_t)h.frame_num & ((1u << kLog2MaxFrameNum) - 1), kLog2MaxFrameNum);
    if (h.idr) put_ue(w, (uint32_t)h.idr_pic_id);
    // pic_order_cnt_type == 2: no POC syntax
    if (h.slice_type == 0) {
        if (h.num_refs > 1) {
            w.put(1, 1);  // num_ref_idx_active_override_flag
            put_ue(w, (uint32_t)(h.num_refs - 1));
        } else {
            w.put(0, 1);
        }
        w.put(0, 1);  // ref_pic_list_modification_flag_l0 (default order: most recent first)
    }
    // dec_ref_pic_marking() (nal_ref_idc != 0)
    if (h.idr) {
        w.put(0, 1);  // no_output_of_prior_pics_flag
        w.put(0, 1);  // long_term_reference_flag
    } else {
        w.put(0, 1);  // adaptive_ref_pic_marking_mode_flag
    }
    put_se(w, h.slice_qp - 26);
    if (h.deblock) {
        put_ue(w, 2);  // disable_deblocking_filter_idc = 2: no filtering across slice edges
        put_se(w, 0);  // slice_alpha_c0_offset_div2
        put_se(w, 0);  // slice_beta_offset_div2
    } else {
        put_ue(w, 1);  // disable_deblocking_filter_idc = 1 (filter off)
    }
}

// Neighbour context of one macroblock for nC prediction.
struct MbNeighbours {
    const MbInfo* left;  // nullptr when unavailable (outside slice/picture)
    const MbInfo* top;
};

// nC of luma block `blk` (luma4x4BlkIdx) of macroblock `cur`.
SK_HD int luma_nc(const MbInfo& cur, MbNeighbours nb, int blk) {
    int bx = blk_x(blk), by = blk_y(blk);
    bool aA, aB;
    int nA = 0, nB = 0;
    if (bx > 0) { aA = true; nA = cur.nnz[blk_from_xy(bx - 1, by)]; }
    else { aA = nb.left != nullptr; if (aA) nA = nb.left->nnz[blk_from_xy(3, by)]; }
    if (by > 0) { aB = true; nB = cur.nnz[blk_from_xy(bx, by - 1)]; }
    else { aB = nb.top != nullptr; if (aB) nB = nb.top->nnz[blk_from_xy(bx, 3)]; }
    return nc_from(aA, nA, aB, nB);
}

// nC of chroma AC block b (0..3, raster in 2x2) of component comp (0 Cb, 1 Cr).
SK_HD int chroma_nc(const MbInfo& cur, MbNeighbours nb, int comp, int b) {
    int bx = b & 1, by = b >> 1;
    int base = 16 + comp * 4;
    bool aA, aB;
    int nA = 0, nB = 0;
    if (bx > 0) { aA = true; nA = cur.nnz[base + by * 2]; }
    else { aA = nb.left != nullptr; if (aA) nA = nb.left->nnz[base + by * 2 + 1]; }
    if (by > 0) { aB = true; nB = cur.nnz[base + bx]; }
    else { aB = nb.top != nullptr; if (aB) nB = nb.top->nnz[base + 2 + bx]; }
    return nc_from(aA, nA, aB, nB);
}

// intraMxMPredModeA / B of block b (8.3.1.1): inside the MB from `cur`; from the left /
// top macroblock otherwise, 2 when that one is not Intra4x4, -1 when it is unavailable.
SK_HD int i4_left_mode(const MbInfo& cur, const MbInfo* left, int b) {
    const int bx = blk_x(b), by = blk_y(b);
    if (bx > 0) return i4_mode(cur, blk_from_xy(bx - 1, by));
    if (!left) return -1;
    return left->type == MB_I4x4 ? i4_mode(*left, blk_from_xy(3, by)) : 2;
}
SK_HD int i4_top_mode(const MbInfo& cur, const MbInfo* top, int b) {
    const int bx = blk_x(b), by = blk_y(b);
    if (by > 0) return i4_mode(cur, blk_from_xy(bx, by - 1));
    if (!top) return -1;
    return top->type == MB_I4x4 ? i4_mode(*top, blk_from_xy(bx, 3)) : 2;
}
SK_HD int i4_predicted(int a, int b) { return (a < 0 || b < 0) ? 2 : sk_min(a, b); }

// macroblock_layer() header part (everything before residual()).
// qp_delta is only written when the syntax carries it; `nb` (left / top MBs of the
// slice) gives the predicted Intra4x4 modes.
template <class W>
SK_HD void write_mb_header(W& w, const MbInfo& mb, bool p_slice, int qp_delta, int num_refs = 1,
                           MbNeighbours nb = MbNeighbours{nullptr, nullptr}) {
    int cbp_l = mb.cbp & 15, cbp_c = (mb.cbp >> 4) & 3;
    if (mb.type == MB_I4x4) {   // I_NxN (7.3.5.1 mb_pred, transform_size_8x8_flag absent in Baseline)
        put_ue(w, p_slice ? 5u : 0u);
        for (int b = 0; b < 16; b++) {
            const int m = i4_mode(mb, b);
            const int pm = i4_predicted(i4_left_mode(mb, nb.left, b), i4_top_mode(mb, nb.top, b));
            if (m == pm) {
                w.put(1u, 1);
            } else {
                w.put(0u, 1);
                w.put((uint32_t)(m < pm ? m : m - 1), 3);
            }
        }
        put_ue(w, mb.chroma_mode);
        put_ue(w, H264_CBP_TO_CODE_INTRA[cbp_l | (cbp_c << 4)]);
        if (mb.cbp) put_se(w, qp_delta);
    } else if (mb.type == MB_I16x16) {
        put_ue(w, (uint32_t)((p_slice ? 5 : 0) + i16_mb_type(mb.i16_mode, cbp_l, cbp_c)));
        put_ue(w, mb.chroma_mode);
        put_se(w, qp_delta);
    } else {  // P_L0_16x16
        put_ue(w, 0);
        if (num_refs == 2) w.put(mb.ref ? 0u : 1u, 1);      // ref_idx_l0 te(v), range 1: one inverted bit
        else if (num_refs > 2) put_ue(w, mb.ref);
        put_se(w, mb.mvdx);
        put_se(w, mb.mvdy);
        put_ue(w, H264_CBP_TO_CODE_INTER[cbp_l | (cbp_c << 4)]);
        if (mb.cbp) put_se(w, qp_delta);
    }
}

SK_HD bool mb_has_qp_delta(const MbInfo& mb) {
    return mb.type == MB_I16x16 || ((mb.type == MB_P_16x16 || mb.type == MB_I4x4) && mb.cbp != 0);
}

// residual() for one macroblock; `coef` points at the MB's kCoefPerMb levels.
template <class W>
SK_HD void write_mb_residual(W& w, const MbInfo& mb, MbNeighbours nb, const int16_t* coef,
                             const CavlcTables& T) {
    int cbp_l = mb.cbp & 15, cbp_c = (mb.cbp >> 4) & 3;
    if (mb.type == MB_I16x16) {
        cavlc_block(w, coef + kCoefLumaDC, 16, luma_nc(mb, nb, 0), T);
        if (cbp_l) {
            for (int blk = 0; blk < 16; blk++)
                cavlc_block(w, coef + kCoefLuma + blk * 16 + 1, 15, luma_nc(mb, nb, blk), T);
        }
    } else {
        for (int b8 = 0; b8 < 4; b8++) {
            if (!(cbp_l & (1 << b8))) continue;
            for (int i = 0; i < 4; i++) {
                int blk = b8 * 4 + i;
                cavlc_block(w, coef + kCoefLuma + blk * 16, 16, luma_nc(mb, nb, blk), T);
            }
        }
    }
    if (cbp_c) {
        cavlc_block(w, coef + kCoefChromaDC + 0, 4, -1, T);
        cavlc_block(w, coef + kCoefChromaDC + 4, 4, -1, T);
    }
    if (cbp_c == 2) {
        for (int comp = 0; comp < 2; comp++)
            for (int b = 0; b < 4; b++)
                cavlc_block(w, coef + kCoefChromaAC + (comp * 4 + b) * 16 + 1, 15,
                            chroma_nc(mb, nb, comp, b), T);
    }
}

// Conservative (nC-independent) size bound of a coded macroblock in bits.
SK_HD int mb_bits_bound(const MbInfo& mb, const int16_t* coef, const CavlcTables& T) {
    int bits = 96;  // mb_type, pred modes, mvd, cbp, qp_delta, skip_run: generous
    int cbp_l = mb.cbp & 15, cbp_c = (mb.cbp >> 4) & 3;
    if (mb.type == MB_I16x16) {
        bits += cavlc_block_bits_bound(coef + kCoefLumaDC, 16, T);
        if (cbp_l)
            for (int blk = 0; blk < 16; blk++)
                bits += cavlc_block_bits_bound(coef + kCoefLuma + blk * 16 + 1, 15, T);
    } else {
        for (int blk = 0; blk < 16; blk++)
            if (cbp_l & (1 << (blk >> 2))) bits += cavlc_block_bits_bound(coef + kCoefLuma + blk * 16, 16, T);
    }
    if (cbp_c) {
        BitCounter bc;
        cavlc_block(bc, coef + kCoefChromaDC, 4, -1, T);
        cavlc_block(bc, coef + kCoefChromaDC + 4, 4, -1, T);
        bits += bc.n;
    }
    if (cbp_c == 2)
        for (int b = 0; b < 8; b++) bits += cavlc_block_bits_bound(coef + kCoefChromaAC + b * 16 + 1, 15, T);
    return bits;
}

}  // namespace h264
}  // namespace sk
