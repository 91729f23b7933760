// H.265 / HEVC Main-profile primitives shared by the CPU reference encoder
// (hevc_cpu.cpp) and the gfx950 kernels (kernels/hevc_kernels.hip): transforms,
// (de)quantisation, intra prediction, chroma motion compensation, merge / AMVP
// candidate lists, the syntax binarisation into CABAC bins and the CABAC
// arithmetic coder itself.
//
// Coding structure (fixed by the parameter sets in hevc_params.cpp):
//   CTB 32x32 with a coding quadtree over a 16x16 analysis grid ("units": the front end's
//   macroblocks, one CuInfo / coefficient / bin slot each). A CTB is either one 32x32 CU
//   (inter: PART_2Nx2N, 2NxN or Nx2N, each PU the motion of its units; a 32x32 TU or the
//   residual quadtree split into four 16x16 nodes) or four 16x16 CUs; an intra 16x16 CU is
//   either one CU (PART_2Nx2N) or four 8x8 CUs (min CB 8), each PART_2Nx2N or PART_NxN
//   (four 4x4 PUs with their own modes). Under a 16x16 CU (or node) the residual quadtree
//   has two more levels: one 16x16 TU or four 8x8 nodes, every node one 8x8 TU or four 4x4
//   ones (DST for intra luma 4x4, transform skip per 4x4 TU) (max TB 32, the encoder's RD
//   choice), intra prediction per TU, mode-dependent scans, one reference picture (previous
//   picture), quarter-pel motion (8-tap luma / 4-tap chroma MC), merge candidates A1 B1 B0
//   A0 B2 on the z-scan availability of the CTB, deblocking on (TU and PU edges,
//   deblock_picture), SAO per CTB (hevc_sao.h), no sign hiding,
//   entropy_coding_sync (WPP): one CABAC substream per CTB row, slices = stripes of
//   whole CTB rows; intra slices split every row into slices of ~kIntraSegCtbs CTBs
//   (SliceMap: a key frame's CTB chain is a segment, not a row).
//   Coding order: CTBs in raster order, the units of a CTB in z order (unit z = x | y << 1);
//   the substream of a CTB row is the sequence of its units' bin chunks in that order.
// Decoder-side operations (inverse transform, dequantisation, intra prediction,
// chroma interpolation, merge/AMVP derivation, context selection) follow the
// normative processes of ITU-T H.265 (04/2013) clauses 8 and 9 exactly; forward
// transform and quantisation are encoder choice (rounding offsets: quant_level).
#pragma once
#include <stddef.h>
#include "sk_common.h"
#include "h264_encoder.h"   // h264::SliceTask (the front end's slice decisions)

namespace sk {
namespace hevc {

// Slice layout of a picture, in CTBs (32x32). Slices are stripes of rows_per_slice CTB
// rows (one WPP substream per row). A row of an intra slice is instead cut into K slices of
// about mb_w / K CTBs each, K = ceil(mb_w / kIntraSegCtbs): the closed-loop intra coding
// of a CTB waits for its left neighbour, so a key frame's longest serial chain is one
// segment (10 CTBs = 40 units at 4K, hevc_encoder.h intra_seg_k) instead of one row (120
// CTBs) - the same cut as the H.264
// IDR sub-slices (h264_encoder.h intra_split). Such a slice starts mid-row and ends in the
// same row, as 7.4.7.1 requires under entropy_coding_sync; it has no top neighbours
// and restarts CABAC, so the cost is some intra and context-adaptation efficiency.
// Neighbours in another slice are unavailable to prediction, CABAC context selection,
// SAO merging, and (pps_loop_filter_across_slices_enabled_flag = 0) to deblocking and
// SAO edge offsets. Per-segment arrays are indexed by slot = cy * K + k.
// (mb_w here: CTBs per row.)
constexpr int kIntraSegCtbs = 20;
SK_HD int intra_seg_count(int mb_w, int seg_ctbs) {
    return seg_ctbs > 0 && mb_w > seg_ctbs ? (mb_w + seg_ctbs - 1) / seg_ctbs : 1;
}
struct SliceMap {
    const h264::SliceTask* tasks;
    int mb_w, rows_per_slice, K;
    SK_HD bool split(int cy) const { return K > 1 && tasks[cy / rows_per_slice].final_action == h264::ACT_I; }
    SK_HD int nseg(int cy) const { return split(cy) ? K : 1; }
    SK_HD int seg(int cx, int cy) const { return split(cy) ? ((cx + 1) * K - 1) / mb_w : 0; }
    SK_HD int x0(int cy, int k) const { return split(cy) ? k * mb_w / K : 0; }
    SK_HD int x1(int cy, int k) const { return split(cy) ? (k + 1) * mb_w / K : mb_w; }
    SK_HD int slot(int cx, int cy) const { return cy * K + seg(cx, cy); }
    SK_HD int id(int cx, int cy) const { return split(cy) ? 2 * (cy * K + seg(cx, cy)) + 1 : 2 * (cy / rows_per_slice); }
    SK_HD bool same(int ax, int ay, int bx, int by) const { return id(ax, ay) == id(bx, by); }
    // neighbour CTBs available to (cx, cy): decoded before it (raster order) and in its slice
    SK_HD bool left(int cx, int cy) const { return cx > 0 && same(cx - 1, cy, cx, cy); }
    SK_HD bool top(int cx, int cy) const { return cy > 0 && same(cx, cy - 1, cx, cy); }
    SK_HD bool top_right(int cx, int cy) const { return cy > 0 && cx + 1 < mb_w && same(cx + 1, cy - 1, cx, cy); }
    // the same on the unit grid (unit (ux, uy) lies in CTB (ux >> 1, uy >> 1))
    SK_HD bool same_u(int ax, int ay, int bx, int by) const { return same(ax >> 1, ay >> 1, bx >> 1, by >> 1); }
};

// Units (16x16) of the picture and their CTBs: W16 x H16 units, CTB (c, r) holds units
// (2c + (z & 1), 2r + (z >> 1)) that lie inside the picture.
struct UnitGrid {
    int W16, H16;
    SK_HD int cw() const { return (W16 + 1) >> 1; }
    SK_HD int ch() const { return (H16 + 1) >> 1; }
    SK_HD bool inside(int ux, int uy) const { return ux >= 0 && uy >= 0 && ux < W16 && uy < H16; }
    SK_HD bool complete(int c, int r) const { return 2 * c + 1 < W16 && 2 * r + 1 < H16; }
    // z-scan order (6.4.1) between two units inside the picture: a decoded before b
    SK_HD bool before(int ax, int ay, int bx, int by) const {
        const int ca = (ay >> 1) * cw() + (ax >> 1), cb = (by >> 1) * cw() + (bx >> 1);
        if (ca != cb) return ca < cb;
        return ((ax & 1) | ((ay & 1) << 1)) < ((bx & 1) | ((by & 1) << 1));
    }
    // neighbour unit (nx, ny) available to unit (ux, uy): inside, decoded before, same slice
    SK_HD bool avail(const SliceMap& m, int ux, int uy, int nx, int ny) const {
        return inside(nx, ny) && before(nx, ny, ux, uy) && m.same_u(nx, ny, ux, uy);
    }
    // chunks (units in coding order) of CTB row r: units of rows 2r, 2r + 1
    SK_HD bool two_rows(int r) const { return 2 * r + 1 < H16; }
    SK_HD int row_chunks(int r) const { return two_rows(r) ? 2 * W16 : W16; }
    SK_HD int ctb_chunk0(int r, int c) const { return two_rows(r) ? 4 * c : 2 * c; }   // first chunk of CTB c
    SK_HD int chunk_unit(int r, int j) const {   // unit index of chunk j of CTB row r
        const int y0 = 2 * r;
        if (!two_rows(r)) return y0 * W16 + j;
        const int full = W16 >> 1;
        if (j < 4 * full) return (y0 + ((j >> 1) & 1)) * W16 + 2 * (j >> 2) + (j & 1);
        return (y0 + (j - 4 * full)) * W16 + W16 - 1;   // odd width: the last CTB's z0, z2
    }
    SK_HD int unit_chunk(int ux, int uy) const {   // inverse: chunk of unit (ux, uy) in its CTB row
        if (!two_rows(uy >> 1)) return ux;
        const int full = W16 >> 1;
        if (ux < 2 * full) return 4 * (ux >> 1) + 2 * (uy & 1) + (ux & 1);
        return 4 * full + (uy & 1);
    }
};

constexpr int kCtb = 32;
constexpr int kCoefPerCu = 384;     // per unit: 16x16 luma | 8x8 Cb | 8x8 Cr, raster [y][x] per TU; split
                                    // units: luma node q (z order) at 64q (one 8x8 TU, or 4x4 TU j at
                                    // 64q + 16j), Cb at 256 + 16q, Cr at 320 + 16q. A CU32 with one 32x32
                                    // TU keeps its 1536 levels (luma 32x32 | Cb 16x16 | Cr 16x16, raster)
                                    // across the slots of its units z0..z3 (kT32Cb / kT32Cr offsets)
constexpr int kCoefCb = 256, kCoefCr = 320;
constexpr int kT32Cb = 1024, kT32Cr = 1280, kT32Coefs = 1536;
constexpr int kCuBinCap = 4096;     // bin entries per CU slot (worst case ~3950, see bin_bound)
constexpr int kSubstreamCtbBytes = 4608;   // worst-case CABAC bytes per CTB (>= 6 bits x ctx bins)

// ---------------------------------------------------------------------------
// Per-unit decisions (40 bytes, shared by CPU and GPU buffers; tests diff them).
enum CuMode : uint8_t { CU_SKIP = 0, CU_MERGE = 1, CU_AMVP = 2, CU_INTRA = 3 };
enum Part : uint8_t { PART_2Nx2N = 0, PART_2NxN = 1, PART_Nx2N = 2 };
struct CuInfo {
    uint8_t mode;         // CuMode (a CU32 member: the mode of the PU holding the unit)
    uint8_t merge_idx;    // SKIP / MERGE
    uint8_t mvp_idx;      // AMVP
    uint8_t intra_mode;   // IntraPredModeY (a CU8-split unit: of CU8 0's first PU); chroma: DM
    uint8_t cbf;          // bit0 Y, bit1 Cb, bit2 Cr (split CUs: any TU of the component)
    uint8_t qp;
    uint8_t tu;           // bit 4: four 8x8 nodes (split_transform_flag); bits 0..3: node q in four 4x4 TUs
    uint8_t tuc;          // split CUs: bits 0..3 cbf_cb, bits 4..7 cbf_cr of the four nodes
    int16_t mvx, mvy;     // quarter-pel
    int16_t mvdx, mvdy;   // AMVP: mv - predictor
    uint16_t ycbf;        // cbf_luma of the TU covering each 4x4 unit (bit = z-order index)
    uint16_t tsy;         // transform_skip_flag of the 4x4 luma TUs (bit = z-order index)
    uint8_t tsc;          // transform_skip_flag of the nodes' 4x4 chroma TUs: bits 0..3 Cb, 4..7 Cr
    uint8_t cu8;          // intra: bit 4 = four 8x8 CUs; bit q = CU8 q is PART_NxN
    uint8_t c32;          // bit 0: the unit is part of a 32x32 CU; bits 1..2 its Part; bit 3: one 32x32 TU
    uint8_t rsv;
    uint8_t ipm[16];      // IntraPredModeY per 4x4 block (z order): MPM neighbours, per-TU prediction
};
static_assert(sizeof(CuInfo) == 40, "CuInfo layout");
constexpr uint8_t kC32 = 1, kC32Tu = 8;
SK_HD int c32_part(const CuInfo& c) { return (c.c32 >> 1) & 3; }
// CtDepth of the unit's CU (split_cu_flag contexts): 0 CU32, 1 CU16, 2 CU8
SK_HD int cu_depth(const CuInfo& c) { return (c.c32 & kC32) ? 0 : ((c.cu8 & 16) ? 2 : 1); }

// ---------------------------------------------------------------------------
// Tables.
SK_TABLE int8_t HEVC_T16[16][16] = {
    {64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64},
    {90, 87, 80, 70, 57, 43, 25, 9, -9, -25, -43, -57, -70, -80, -87, -90},
    {89, 75, 50, 18, -18, -50, -75, -89, -89, -75, -50, -18, 18, 50, 75, 89},
    {87, 57, 9, -43, -80, -90, -70, -25, 25, 70, 90, 80, 43, -9, -57, -87},
    {83, 36, -36, -83, -83, -36, 36, 83, 83, 36, -36, -83, -83, -36, 36, 83},
    {80, 9, -70, -87, -25, 57, 90, 43, -43, -90, -57, 25, 87, 70, -9, -80},
    {75, -18, -89, -50, 50, 89, 18, -75, -75, 18, 89, 50, -50, -89, -18, 75},
    {70, -43, -87, 9, 90, 25, -80, -57, 57, 80, -25, -90, -9, 87, 43, -70},
    {64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64},
    {57, -80, -25, 90, -9, -87, 43, 70, -70, -43, 87, 9, -90, 25, 80, -57},
    {50, -89, 18, 75, -75, -18, 89, -50, -50, 89, -18, -75, 75, 18, -89, 50},
    {43, -90, 57, 25, -87, 70, 9, -80, 80, -9, -70, 87, -25, -57, 90, -43},
    {36, -83, 83, -36, -36, 83, -83, 36, 36, -83, 83, -36, -36, 83, -83, 36},
    {25, -70, 90, -80, 43, 9, -57, 87, -87, 57, -9, -43, 80, -90, 70, -25},
    {18, -50, 75, -89, 89, -75, 50, -18, -18, 50, -75, 89, -89, 75, -50, 18},
    {9, -25, 43, -57, 70, -80, 87, -90, 90, -87, 80, -70, 57, -43, 25, -9}};
// 32-point matrix (8.6.4.2 transMatrix): the even rows restricted to 16 columns are the
// 16-point matrix, the odd rows use 90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4.
SK_TABLE int8_t HEVC_T32[32][32] = {
    {64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64, 64},
    {90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4, -4, -13, -22, -31, -38, -46, -54, -61, -67, -73, -78, -82, -85, -88, -90, -90},
    {90, 87, 80, 70, 57, 43, 25, 9, -9, -25, -43, -57, -70, -80, -87, -90, -90, -87, -80, -70, -57, -43, -25, -9, 9, 25, 43, 57, 70, 80, 87, 90},
    {90, 82, 67, 46, 22, -4, -31, -54, -73, -85, -90, -88, -78, -61, -38, -13, 13, 38, 61, 78, 88, 90, 85, 73, 54, 31, 4, -22, -46, -67, -82, -90},
    {89, 75, 50, 18, -18, -50, -75, -89, -89, -75, -50, -18, 18, 50, 75, 89, 89, 75, 50, 18, -18, -50, -75, -89, -89, -75, -50, -18, 18, 50, 75, 89},
    {88, 67, 31, -13, -54, -82, -90, -78, -46, -4, 38, 73, 90, 85, 61, 22, -22, -61, -85, -90, -73, -38, 4, 46, 78, 90, 82, 54, 13, -31, -67, -88},
    {87, 57, 9, -43, -80, -90, -70, -25, 25, 70, 90, 80, 43, -9, -57, -87, -87, -57, -9, 43, 80, 90, 70, 25, -25, -70, -90, -80, -43, 9, 57, 87},
    {85, 46, -13, -67, -90, -73, -22, 38, 82, 88, 54, -4, -61, -90, -78, -31, 31, 78, 90, 61, 4, -54, -88, -82, -38, 22, 73, 90, 67, 13, -46, -85},
    {83, 36, -36, -83, -83, -36, 36, 83, 83, 36, -36, -83, -83, -36, 36, 83, 83, 36, -36, -83, -83, -36, 36, 83, 83, 36, -36, -83, -83, -36, 36, 83},
    {82, 22, -54, -90, -61, 13, 78, 85, 31, -46, -90, -67, 4, 73, 88, 38, -38, -88, -73, -4, 67, 90, 46, -31, -85, -78, -13, 61, 90, 54, -22, -82},
    {80, 9, -70, -87, -25, 57, 90, 43, -43, -90, -57, 25, 87, 70, -9, -80, -80, -9, 70, 87, 25, -57, -90, -43, 43, 90, 57, -25, -87, -70, 9, 80},
    {78, -4, -82, -73, 13, 85, 67, -22, -88, -61, 31, 90, 54, -38, -90, -46, 46, 90, 38, -54, -90, -31, 61, 88, 22, -67, -85, -13, 73, 82, 4, -78},
    {75, -18, -89, -50, 50, 89, 18, -75, -75, 18, 89, 50, -50, -89, -18, 75, 75, -18, -89, -50, 50, 89, 18, -75, -75, 18, 89, 50, -50, -89, -18, 75},
    {73, -31, -90, -22, 78, 67, -38, -90, -13, 82, 61, -46, -88, -4, 85, 54, -54, -85, 4, 88, 46, -61, -82, 13, 90, 38, -67, -78, 22, 90, 31, -73},
    {70, -43, -87, 9, 90, 25, -80, -57, 57, 80, -25, -90, -9, 87, 43, -70, -70, 43, 87, -9, -90, -25, 80, 57, -57, -80, 25, 90, 9, -87, -43, 70},
    {67, -54, -78, 38, 85, -22, -90, 4, 90, 13, -88, -31, 82, 46, -73, -61, 61, 73, -46, -82, 31, 88, -13, -90, -4, 90, 22, -85, -38, 78, 54, -67},
    {64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64, 64, -64, -64, 64},
    {61, -73, -46, 82, 31, -88, -13, 90, -4, -90, 22, 85, -38, -78, 54, 67, -67, -54, 78, 38, -85, -22, 90, 4, -90, 13, 88, -31, -82, 46, 73, -61},
    {57, -80, -25, 90, -9, -87, 43, 70, -70, -43, 87, 9, -90, 25, 80, -57, -57, 80, 25, -90, 9, 87, -43, -70, 70, 43, -87, -9, 90, -25, -80, 57},
    {54, -85, -4, 88, -46, -61, 82, 13, -90, 38, 67, -78, -22, 90, -31, -73, 73, 31, -90, 22, 78, -67, -38, 90, -13, -82, 61, 46, -88, 4, 85, -54},
    {50, -89, 18, 75, -75, -18, 89, -50, -50, 89, -18, -75, 75, 18, -89, 50, 50, -89, 18, 75, -75, -18, 89, -50, -50, 89, -18, -75, 75, 18, -89, 50},
    {46, -90, 38, 54, -90, 31, 61, -88, 22, 67, -85, 13, 73, -82, 4, 78, -78, -4, 82, -73, -13, 85, -67, -22, 88, -61, -31, 90, -54, -38, 90, -46},
    {43, -90, 57, 25, -87, 70, 9, -80, 80, -9, -70, 87, -25, -57, 90, -43, -43, 90, -57, -25, 87, -70, -9, 80, -80, 9, 70, -87, 25, 57, -90, 43},
    {38, -88, 73, -4, -67, 90, -46, -31, 85, -78, 13, 61, -90, 54, 22, -82, 82, -22, -54, 90, -61, -13, 78, -85, 31, 46, -90, 67, 4, -73, 88, -38},
    {36, -83, 83, -36, -36, 83, -83, 36, 36, -83, 83, -36, -36, 83, -83, 36, 36, -83, 83, -36, -36, 83, -83, 36, 36, -83, 83, -36, -36, 83, -83, 36},
    {31, -78, 90, -61, 4, 54, -88, 82, -38, -22, 73, -90, 67, -13, -46, 85, -85, 46, 13, -67, 90, -73, 22, 38, -82, 88, -54, -4, 61, -90, 78, -31},
    {25, -70, 90, -80, 43, 9, -57, 87, -87, 57, -9, -43, 80, -90, 70, -25, -25, 70, -90, 80, -43, -9, 57, -87, 87, -57, 9, 43, -80, 90, -70, 25},
    {22, -61, 85, -90, 73, -38, -4, 46, -78, 90, -82, 54, -13, -31, 67, -88, 88, -67, 31, 13, -54, 82, -90, 78, -46, 4, 38, -73, 90, -85, 61, -22},
    {18, -50, 75, -89, 89, -75, 50, -18, -18, 50, -75, 89, -89, 75, -50, 18, 18, -50, 75, -89, 89, -75, 50, -18, -18, 50, -75, 89, -89, 75, -50, 18},
    {13, -38, 61, -78, 88, -90, 85, -73, 54, -31, 4, 22, -46, 67, -82, 90, -90, 82, -67, 46, -22, -4, 31, -54, 73, -85, 90, -88, 78, -61, 38, -13},
    {9, -25, 43, -57, 70, -80, 87, -90, 90, -87, 80, -70, 57, -43, 25, -9, -9, 25, -43, 57, -70, 80, -87, 90, -90, 87, -80, 70, -57, 43, -25, 9},
    {4, -13, 22, -31, 38, -46, 54, -61, 67, -73, 78, -82, 85, -88, 90, -90, 90, -90, 88, -85, 82, -78, 73, -67, 61, -54, 46, -38, 31, -22, 13, -4}};
// The 8-point matrix is rows 0, 2, 4, ... of the 16-point one restricted to 8 columns.
SK_HD int dct_coef(int log2n, int k, int n) { return log2n == 5 ? HEVC_T32[k][n] : HEVC_T16[k << (4 - log2n)][n]; }
// 4x4 DST-VII (8.6.4.2, intra luma 4x4 TUs).
SK_TABLE int8_t HEVC_DST4[4][4] = {{29, 55, 74, 84}, {74, 74, 0, -74}, {84, -29, -74, 55}, {55, -84, 74, -29}};
SK_HD int tx_coef(int log2n, bool dst, int k, int n) { return dst ? HEVC_DST4[k][n] : dct_coef(log2n, k, n); }
// z-order index of 4x4 unit (x, y) of a 16x16 CU (x, y = 0..3).
SK_HD int zorder4(int x, int y) { return (x & 1) | ((y & 1) << 1) | ((x & 2) << 1) | ((y & 2) << 2); }

// Up-right diagonal scan of a 4x4 (sub-)block: scan position -> raster (y*4+x), and back.
SK_HD int diag4_raster(int n) { return (int)((0xfbe7ad369c258140ULL >> (4 * n)) & 15); }
SK_HD int diag4_scanpos(int r) { return (int)((0xfda6eb73c8419520ULL >> (4 * r)) & 15); }
// Sub-block scans: 2x2 for 8x8 TUs, 4x4 for 16x16 TUs, 8x8 for 32x32 TUs (same diagonal rule).
SK_HD int diag2_raster(int n) { return (int)((0x3120u >> (4 * n)) & 15); }   // (0,0),(0,1),(1,0),(1,1) as y*2+x
SK_TABLE uint8_t HEVC_DIAG8[64] = {0,  8,  1,  16, 9,  2,  24, 17, 10, 3,  32, 25, 18, 11, 4,  40, 33, 26, 19, 12, 5,  48,
                                   41, 34, 27, 20, 13, 6,  56, 49, 42, 35, 28, 21, 14, 7,  57, 50, 43, 36, 29, 22, 15, 58,
                                   51, 44, 37, 30, 23, 59, 52, 45, 38, 31, 60, 53, 46, 39, 61, 54, 47, 62, 55, 63};
SK_HD int sb_raster(int log2n, int i) {   // sub-block scan index -> raster index in the sub-block grid
    return log2n == 5 ? HEVC_DIAG8[i] : (log2n == 4 ? diag4_raster(i) : (log2n == 3 ? diag2_raster(i) : 0));
}
// scanIdx (7.4.9.11): 0 up-right diagonal, 1 horizontal, 2 vertical. The horizontal and
// vertical scans occur for 4x4 / 8x8 TUs only (mode-dependent intra scans).
enum Scan { SCAN_DIAG = 0, SCAN_HOR = 1, SCAN_VER = 2 };
SK_HD int scan4_raster(int scan, int k) {   // position k of a 4x4 sub-block -> raster (y*4 + x)
    return scan == SCAN_DIAG ? diag4_raster(k) : (scan == SCAN_HOR ? k : ((k & 3) << 2) | (k >> 2));
}
SK_HD int sb_scan_raster(int log2n, int scan, int i) {   // sub-block i -> raster in the sub-block grid
    if (scan == SCAN_DIAG || log2n != 3) return sb_raster(log2n, i);
    return scan == SCAN_HOR ? i : ((i & 1) << 1) | (i >> 1);
}
// Intra scans (8.4.4? / 7.4.9.11): luma 4x4 / 8x8 and chroma 4x4 TUs of intra CUs.
SK_HD int intra_scan(int mode, int log2n, int cidx) {
    if (!(log2n == 2 || (log2n == 3 && cidx == 0))) return SCAN_DIAG;
    if (mode >= 6 && mode <= 14) return SCAN_VER;
    if (mode >= 22 && mode <= 30) return SCAN_HOR;
    return SCAN_DIAG;
}

// CABAC (shared with H.264): LPS ranges and LPS state transitions.
SK_TABLE uint8_t CABAC_LPS[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205}, {116, 142, 169, 195},
    {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166}, {95, 116, 137, 158}, {90, 110, 130, 150},
    {85, 104, 123, 142},  {81, 99, 117, 135},   {77, 94, 111, 128},   {73, 89, 105, 122},  {69, 85, 100, 116},
    {66, 80, 95, 110},    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},    {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},    {41, 50, 59, 69},
    {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},     {33, 41, 48, 56},    {32, 39, 46, 53},
    {30, 37, 43, 50},     {29, 35, 41, 48},     {27, 33, 39, 45},     {26, 31, 37, 43},    {24, 30, 35, 41},
    {23, 28, 33, 39},     {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},    {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},    {14, 18, 21, 24},
    {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},     {12, 14, 17, 20},    {11, 14, 16, 19},
    {11, 13, 15, 18},     {10, 12, 15, 17},     {10, 12, 14, 16},     {9, 11, 13, 15},     {9, 11, 12, 14},
    {8, 10, 12, 14},      {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},      {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
SK_TABLE uint8_t CABAC_NEXT_LPS[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                       13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                       24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                       33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

// ---------------------------------------------------------------------------
// Context index space (flat). initValues per initType (0 = I, 1 = P with
// cabac_init_flag 0): Tables 9-5 .. 9-37 of H.265.
enum Ctx : int {
    CTX_SKIP = 0,            // 3 (ctxInc = condL + condA)
    CTX_PRED_MODE = 3,
    CTX_PART_MODE = 4,       // first bin only (2Nx2N)
    CTX_PREV_INTRA = 5,
    CTX_CHROMA_PRED = 6,
    CTX_MERGE_FLAG = 7,
    CTX_MERGE_IDX = 8,
    CTX_MVP = 9,
    CTX_RQT_ROOT_CBF = 10,
    CTX_MVD_G0 = 11,
    CTX_MVD_G1 = 12,
    CTX_CBF_LUMA = 13,       // 2
    CTX_CBF_CHROMA = 15,     // 4
    CTX_LAST_X = 19,         // 18
    CTX_LAST_Y = 37,         // 18
    CTX_CSBF = 55,           // 4
    CTX_SIG = 59,            // 42
    CTX_GT1 = 101,           // 24
    CTX_GT2 = 125,           // 6
    CTX_SAO_MERGE = 131,     // sao_merge_left_flag / sao_merge_up_flag
    CTX_SAO_TYPE = 132,      // first bin of sao_type_idx_luma / _chroma
    CTX_SPLIT_TF = 133,      // 3 split_transform_flag (ctxInc 5 - log2TrafoSize)
    CTX_TS = 136,            // 2 transform_skip_flag (luma, chroma)
    CTX_SPLIT_CU = 138,      // 3 split_cu_flag (ctxInc = condL + condA on CtDepth)
    CTX_PART_MODE1 = 141,    // part_mode bin 1 (inter: 2NxN "01" / Nx2N "00")
    CTX_COUNT = 142,
    CTX_TERM = 255           // terminating bin (end_of_slice_segment_flag / end_of_subset_one_bit)
};
SK_TABLE uint8_t HEVC_CTX_INIT[2][CTX_COUNT] = {
    {// I slices
     154, 154, 154,                 // skip (n/a)
     154,                           // pred_mode (n/a)
     184,                           // part_mode
     184,                           // prev_intra_luma_pred_flag
     63,                            // intra_chroma_pred_mode
     154, 154, 154, 154,            // merge_flag, merge_idx, mvp, rqt_root_cbf (n/a)
     154, 154,                      // mvd (n/a)
     111, 141,                      // cbf_luma
     94, 138, 182, 154,             // cbf_cb/cr
     110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,   // last x
     110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,   // last y
     91, 171, 134, 141,             // coded_sub_block_flag
     111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153, 125,
     107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153, 136, 139, 111, 136, 139, 111,
     140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179, 166, 182, 140, 227,
     122, 197,                      // greater1
     138, 153, 136, 167, 152, 152,  // greater2
     153, 200,                      // sao merge, sao type
     153, 138, 138,                 // split_transform_flag
     139, 139,                      // transform_skip_flag
     139, 141, 157,                 // split_cu_flag
     154},                          // part_mode bin 1 (n/a)
    {// P slices (cabac_init_flag = 0)
     197, 185, 201,                 // cu_skip_flag
     149,                           // pred_mode_flag
     154,                           // part_mode
     154,                           // prev_intra_luma_pred_flag
     152,                           // intra_chroma_pred_mode
     110, 122, 168, 79,             // merge_flag, merge_idx, mvp_l0_flag, rqt_root_cbf
     140, 198,                      // abs_mvd_greater0 / greater1
     153, 111,                      // cbf_luma
     149, 107, 167, 154,            // cbf_cb/cr
     125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108,     // last x
     125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108,     // last y
     121, 140, 61, 154,             // coded_sub_block_flag
     155, 154, 139, 153, 139, 123, 123, 63, 153, 166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153, 154,
     166, 183, 140, 136, 153, 154, 170, 153, 138, 138, 122, 121, 122, 121, 167, 151, 183, 140, 151, 183, 140,
     154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137, 169, 194, 166, 167, 154, 167,
     137, 182,                      // greater1
     107, 167, 91, 122, 107, 167,   // greater2
     153, 185,                      // sao merge, sao type
     124, 138, 94,                  // split_transform_flag
     139, 139,                      // transform_skip_flag
     107, 139, 126,                 // split_cu_flag
     139}};                         // part_mode bin 1

// Context state byte: (pStateIdx << 1) | valMps (9.3.2.2).
SK_HD uint8_t ctx_init_state(int init_value, int slice_qp) {
    const int slope = init_value >> 4, offset = init_value & 15;
    const int m = slope * 5 - 45, n = (offset << 3) - 16;
    const int pre = sk_clip(((m * sk_clip(slice_qp, 0, 51)) >> 4) + n, 1, 126);
    const int mps = pre <= 63 ? 0 : 1;
    const int st = mps ? pre - 64 : 63 - pre;
    return (uint8_t)((st << 1) | mps);
}
SK_HD void ctx_init_all(uint8_t* st, int init_type, int slice_qp) {
    for (int i = 0; i < CTX_COUNT; i++) st[i] = ctx_init_state(HEVC_CTX_INIT[init_type][i], slice_qp);
}
// Context adaptation only (no arithmetic coding): used to derive WPP sync states.
SK_HD void ctx_update(uint8_t& s, int bin) {
    int st = s >> 1, mps = s & 1;
    if (bin == mps) st = st < 62 ? st + 1 : 62;
    else {
        if (st == 0) mps ^= 1;
        st = CABAC_NEXT_LPS[st];
    }
    s = (uint8_t)((st << 1) | mps);
}

// ---------------------------------------------------------------------------
// Bin entries (uint16), produced by the binariser and consumed by the CABAC coder:
//   context bin  : bit15 = 0, bit8 = bin value, bits 0..7 = context index (CTX_TERM: terminate)
//   bypass run   : bit15 = 1, bits 12..14 = n - 1 (n = 1..8 bins), bits 0..7 = the bins (MSB first)
struct BinBuf {
    static constexpr bool kWave = false;
    uint16_t* p;
    int n;
    SK_HD void ctx(int c, int b) { p[n++] = (uint16_t)(((b & 1) << 8) | c); }
    SK_HD void term(int b) { p[n++] = (uint16_t)(((b & 1) << 8) | CTX_TERM); }
    SK_HD void bypass(uint32_t v, int nb) {
        while (nb > 0) {
            const int k = nb > 8 ? 8 : nb;
            nb -= k;
            p[n++] = (uint16_t)(0x8000u | ((uint32_t)(k - 1) << 12) | ((v >> nb) & ((1u << k) - 1)));
        }
    }
};
struct BinCount {   // same interface, counts entries
    static constexpr bool kWave = false;
    int n = 0;
    SK_HD void ctx(int, int) { n++; }
    SK_HD void term(int) { n++; }
    SK_HD void bypass(uint32_t, int nb) { n += (nb + 7) >> 3; }
};

// ---------------------------------------------------------------------------
// CABAC arithmetic encoder (9.3.4.3 encoder side, HM TEncBinCABAC arithmetic).
// Output is a byte-aligned substream; finish() appends the terminating bits and the
// byte_alignment() / rbsp stop bit ('1' + zeros).
struct CabacEncoder {
    uint32_t low, range;
    int32_t bits_left, num_buffered;
    uint32_t buffered;
    uint8_t* out;
    uint32_t pos;   // bytes written
    SK_HD void start(uint8_t* o) {
        out = o;
        pos = 0;
        low = 0;
        range = 510;
        bits_left = 23;
        num_buffered = 0;
        buffered = 0xff;
    }
    SK_HD void put(uint32_t b) { out[pos++] = (uint8_t)b; }
    SK_HD void write_out() {
        const uint32_t lead = low >> (24 - bits_left);
        bits_left += 8;
        low &= 0xffffffffu >> bits_left;
        if (lead == 0xff) {
            num_buffered++;
        } else if (num_buffered > 0) {
            const uint32_t carry = lead >> 8;
            put(buffered + carry);
            buffered = lead & 0xff;
            const uint32_t fill = (0xff + carry) & 0xff;
            while (num_buffered > 1) {
                put(fill);
                num_buffered--;
            }
        } else {
            num_buffered = 1;
            buffered = lead;
        }
    }
    SK_HD void test_write() {
        if (bits_left < 12) write_out();
    }
    SK_HD void encode(int bin, uint8_t& s) {
        const int st = s >> 1, mps = s & 1;
        const uint32_t lps = CABAC_LPS[st][(range >> 6) & 3];
        range -= lps;
        if (bin != mps) {
            const int nbits = 8 - (31 - __builtin_clz(lps));   // renormalisation shift
            low = (low + range) << nbits;
            range = lps << nbits;
            bits_left -= nbits;
            s = (uint8_t)((CABAC_NEXT_LPS[st] << 1) | (st == 0 ? mps ^ 1 : mps));
        } else {
            s = (uint8_t)(((st < 62 ? st + 1 : 62) << 1) | mps);
            if (range >= 256) return;
            low <<= 1;
            range <<= 1;
            bits_left--;
        }
        test_write();
    }
    SK_HD void bypass(uint32_t bins, int n) {   // n <= 8
        low = (low << n) + range * bins;
        bits_left -= n;
        test_write();
    }
    SK_HD void terminate(int bin) {
        range -= 2;
        if (bin) {
            low += range;
            low <<= 7;
            range = 2 << 7;
            bits_left -= 7;
        } else if (range >= 256) {
            return;
        } else {
            low <<= 1;
            range <<= 1;
            bits_left--;
        }
        test_write();
    }
    // After terminate(1): flush, then the '1' alignment bit and zero bits to a byte boundary.
    SK_HD void finish() {
        if (low >> (32 - bits_left)) {
            put(buffered + 1);
            while (num_buffered > 1) {
                put(0x00);
                num_buffered--;
            }
            low -= 1u << (32 - bits_left);
        } else {
            if (num_buffered > 0) put(buffered);
            while (num_buffered > 1) {
                put(0xff);
                num_buffered--;
            }
        }
        // remaining 24 - bits_left bits of low >> 8, then '1', then zeros
        const int nb = 24 - bits_left;
        uint64_t acc = ((uint64_t)(low >> 8) & ((1ull << nb) - 1)) << 1 | 1ull;
        int total = nb + 1;
        const int pad = (8 - (total & 7)) & 7;
        acc <<= pad;
        total += pad;
        for (int i = total - 8; i >= 0; i -= 8) put((uint32_t)(acc >> i) & 0xff);
    }
    // Codes one bin entry (see BinBuf) with context states `ctx`.
    SK_HD void code_entry(uint16_t e, uint8_t* ctx) {
        if (e & 0x8000u) {
            bypass(e & 0xffu, ((e >> 12) & 7) + 1);
        } else if ((e & 0xffu) == CTX_TERM) {
            terminate((e >> 8) & 1);
        } else {
            encode((e >> 8) & 1, ctx[e & 0xffu]);
        }
    }
};

// ---------------------------------------------------------------------------
// Transforms. Residual / coefficient blocks are raster [y][x] int arrays.
// Forward (encoder choice, HM partial butterflies as matrix products):
// shift1 = log2n + bitDepth - 9, shift2 = log2n + 6.
SK_HD void fwd_transform(const int* res, int log2n, int* coef, bool dst = false) {
    const int n = 1 << log2n;
    const int sh1 = log2n - 1, sh2 = log2n + 6;
    int tmp[1024];
    for (int y = 0; y < n; y++)          // horizontal: tmp[y][u]
        for (int u = 0; u < n; u++) {
            int s = 0;
            for (int x = 0; x < n; x++) s += tx_coef(log2n, dst, u, x) * res[y * n + x];
            tmp[y * n + u] = (s + (1 << (sh1 - 1))) >> sh1;
        }
    for (int v = 0; v < n; v++)          // vertical: coef[v][u]
        for (int u = 0; u < n; u++) {
            int s = 0;
            for (int y = 0; y < n; y++) s += tx_coef(log2n, dst, v, y) * tmp[y * n + u];
            coef[v * n + u] = (s + (1 << (sh2 - 1))) >> sh2;
        }
}
// Inverse (8.6.4.2): columns first, clip to 16 bits after (e + 64) >> 7, then rows,
// residual = (r + 2048) >> 12 for 8-bit video.
SK_HD void inv_transform(const int* d, int log2n, int* res, bool dst = false) {
    const int n = 1 << log2n;
    int g[1024];
    for (int x = 0; x < n; x++)
        for (int y = 0; y < n; y++) {
            int s = 0;
            for (int j = 0; j < n; j++) s += tx_coef(log2n, dst, j, y) * d[j * n + x];
            g[y * n + x] = sk_clip((s + 64) >> 7, -32768, 32767);
        }
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) {
            int s = 0;
            for (int j = 0; j < n; j++) s += tx_coef(log2n, dst, j, x) * g[y * n + j];
            res[y * n + x] = (s + 2048) >> 12;
        }
}

// Transform skip (4x4, 8.6.4.2): the decoder's residual is (d << 7 + 2^11) >> 12; the
// encoder's "coefficients" are the residual << 5 (the 4x4 transform's scale).
SK_HD void ts_forward(const int* res, int* coef) {
    for (int i = 0; i < 16; i++) coef[i] = res[i] * 32;
}
SK_HD void ts_inverse(const int* d, int* res) {
    for (int i = 0; i < 16; i++) res[i] = (d[i] * 128 + 2048) >> 12;
}

// Quantisation (HM: quantScale, QUANT_SHIFT 14, transform shift 15 - 8 - log2n,
// dead-zone offset 171/512 intra, 85/512 inter) and dequantisation (8.6.3, flat m = 16).
SK_HD int quant_scale(int r) { return r == 0 ? 26214 : r == 1 ? 23302 : r == 2 ? 20560 : r == 3 ? 18396 : r == 4 ? 16384 : 14564; }
SK_HD int level_scale(int r) { return r == 0 ? 40 : r == 1 ? 45 : r == 2 ? 51 : r == 3 ? 57 : r == 4 ? 64 : 72; }
constexpr int kMaxLevel = 32767;
// Rounding offsets of the quantiser (Q9: 240 / 512 = 0.47 intra, 150 / 512 = 0.29 inter).
// The RD zeroing of whole TUs (J = SSE + lambda R) removes what does not pay, so the levels
// themselves round nearer than HM's 1/3 and 1/6 dead zones: -1.8 % (desktop) / -1.2 %
// (motion) BD-rate at 640x360 (tools/rd_codecs.py, CPU, 8 frames per point).
constexpr int kQuantRoundIntra = 240, kQuantRoundInter = 150;
SK_HD int quant_level(int c, int qp, int log2n, bool intra) {
    const int qbits = 14 + qp / 6 + (7 - log2n);
    const int64_t add = (int64_t)(intra ? kQuantRoundIntra : kQuantRoundInter) << (qbits - 9);
    const int a = sk_abs(c);
    int l = (int)(((int64_t)a * quant_scale(qp % 6) + add) >> qbits);
    l = sk_min(l, kMaxLevel);
    return c < 0 ? -l : l;
}
SK_HD int dequant_level(int l, int qp, int log2n) {
    // d = Clip3(-32768, 32767, (l * m * levelScale[qp % 6] << (qp / 6)) + (1 << (bdShift - 1)) >> bdShift),
    // m = 16 (flat), bdShift = BitDepth + log2n - 5
    const int bdshift = 3 + log2n;
    const int64_t v = ((int64_t)l * 16 * level_scale(qp % 6) * ((int64_t)1 << (qp / 6)) + (1 << (bdshift - 1))) >> bdshift;
    return (int)(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
}
// QpC for ChromaArrayType 1 (Table 8-10): qPi < 30 -> qPi; 30..43 -> table; > 43 -> qPi - 6.
SK_HD int chroma_qp(int qpi) {
    if (qpi < 30) return qpi;
    if (qpi > 43) return qpi - 6;
    return 29 + (int)((0x88776655443210ull >> (4 * (qpi - 30))) & 15);
}

// ---------------------------------------------------------------------------
// Intra prediction (8.4.4.2). ref[] is the linear reference array of a TU of size
// N: ref[0] = p[-1][2N-1] (bottom of the left column) ... ref[2N-1] = p[-1][0],
// ref[2N] = p[-1][-1], ref[2N+1+x] = p[x][-1] (x = 0..2N-1). avail[] flags per
// entry. Substitution (8.4.4.2.2) in place.
SK_HD void intra_substitute(uint8_t* ref, const uint8_t* avail, int n) {
    const int len = 4 * n + 1;
    int first = -1;
    for (int i = 0; i < len; i++)
        if (avail[i]) { first = i; break; }
    if (first < 0) {
        for (int i = 0; i < len; i++) ref[i] = 128;
        return;
    }
    for (int i = 0; i < first; i++) ref[i] = ref[first];
    for (int i = first + 1; i < len; i++)
        if (!avail[i]) ref[i] = ref[i - 1];
}
// [1 2 1] smoothing (8.4.4.2.3) when filterFlag: luma, mode != DC, N > 4 and
// min(|mode - 26|, |mode - 10|) > thres(N) (7 for 8x8, 1 for 16x16, 0 for 32x32).
SK_HD bool intra_filter_flag(int mode, int log2n, int cidx) {
    if (cidx != 0 || mode == 1 || log2n == 2) return false;
    const int d = sk_min(sk_abs(mode - 26), sk_abs(mode - 10));
    const int thres = log2n == 3 ? 7 : (log2n == 4 ? 1 : 0);
    return d > thres;
}
SK_HD void intra_filter(const uint8_t* ref, int n, uint8_t* out) {
    const int len = 4 * n + 1;
    out[0] = ref[0];
    out[len - 1] = ref[len - 1];
    for (int i = 1; i < len - 1; i++) out[i] = (uint8_t)((ref[i - 1] + 2 * ref[i] + ref[i + 1] + 2) >> 2);
}
SK_TABLE int8_t HEVC_INTRA_ANGLE[35] = {0,   0,   32,  26,  21,  17,  13,  9,   5,   2,   0,   -2,
                                        -5,  -9,  -13, -17, -21, -26, -32, -26, -21, -17, -13, -9,
                                        -5,  -2,  0,   2,   5,   9,   13,  17,  21,  26,  32};
SK_HD int intra_inv_angle(int mode) {   // modes 11..25
    const int a = sk_abs(HEVC_INTRA_ANGLE[mode]);
    return a == 2 ? -4096 : a == 5 ? -1638 : a == 9 ? -910 : a == 13 ? -630 : a == 17 ? -482 : a == 21 ? -390
                  : a == 26 ? -315 : -256;
}
// Prediction sample (x, y) of an N x N block from the (filtered) linear reference.
// R: reference accessor, i -> ref[i] (an array, or LDS / cross-lane reads on the GPU).
template <class R>
SK_HD int intra_pred_at(R ref, int n, int log2n, int mode, int cidx, int x, int y) {
    auto L = [&](int yy) { return (int)ref(2 * n - 1 - yy); };   // p[-1][yy], yy = -1 .. 2N-1
    auto T = [&](int xx) { return (int)ref(2 * n + 1 + xx); };   // p[xx][-1], xx = -1 .. 2N-1
    if (mode == 0) {
        return ((n - 1 - x) * L(y) + (x + 1) * T(n) + (n - 1 - y) * T(x) + (y + 1) * L(n) + n) >> (log2n + 1);
    }
    if (mode == 1) {
        int s = n;
        for (int i = 0; i < n; i++) s += T(i) + L(i);
        const int dc = s >> (log2n + 1);
        if (cidx == 0 && n < 32) {
            if (x == 0 && y == 0) return (L(0) + 2 * dc + T(0) + 2) >> 2;
            if (y == 0) return (T(x) + 3 * dc + 2) >> 2;
            if (x == 0) return (L(y) + 3 * dc + 2) >> 2;
        }
        return dc;
    }
    // main reference array (8.4.4.2.6) in closed form: refm(k), k = -N .. 2N, the main
    // side for k >= 0, the other side projected through invAngle for k < 0 (read only
    // for the negative angles that need it)
    const int angle = HEVC_INTRA_ANGLE[mode];
    const bool vert = mode >= 18;
    auto refm = [&](int k) {
        if (k >= 0) return vert ? T(k - 1) : L(k - 1);
        const int j = (k * intra_inv_angle(mode) + 128) >> 8;
        return vert ? L(j - 1) : T(j - 1);
    };
    const int a = vert ? y : x, b = vert ? x : y;   // a: distance from the main side, b: along it
    const int idx = ((a + 1) * angle) >> 5, fact = ((a + 1) * angle) & 31;
    const int k0 = b + idx + 1;
    int v = fact ? ((32 - fact) * refm(k0) + fact * refm(k0 + 1) + 16) >> 5 : refm(k0);
    if (cidx == 0 && n < 32) {
        if (mode == 26 && x == 0) v = sk_clip255(T(0) + ((L(y) - L(-1)) >> 1));
        if (mode == 10 && y == 0) v = sk_clip255(L(0) + ((T(x) - T(-1)) >> 1));
    }
    return v;
}
SK_HD int intra_pred_sample(const uint8_t* ref, int n, int log2n, int mode, int cidx, int x, int y) {
    return intra_pred_at([&](int i) { return (int)ref[i]; }, n, log2n, mode, cidx, x, y);
}

// Encoder mode decision (open loop, every CU in parallel, so no MPM-dependent cost):
// all 35 luma modes in this order, first minimum of SAD + bias wins (SAD of the sixteen
// 4x4 blocks, each predicted from its source neighbours). The four
// non-directional / axis modes carry no bias; the 31 other directions pay about six
// bits at the SAD lambda of the QP.
SK_TABLE int8_t HEVC_INTRA_ORDER[35] = {1,  0,  26, 10, 2,  3,  4,  5,  6,  7,  8,  9,  11, 12, 13, 14, 15, 16,
                                        17, 18, 19, 20, 21, 22, 23, 24, 25, 27, 28, 29, 30, 31, 32, 33, 34};
SK_HD bool intra_mode_basic(int mode) { return mode <= 1 || mode == 10 || mode == 26; }
// CU8 decision (hevc_cpu.cpp intra_decide, k_hevc_intra_prep): penalties of the split and
// of PART_NxN in SAD units (x intra_lam_sad) for their extra signalling.
SK_HD int intra_lam_sad(int qp) { return qp < 12 ? 1 : 1 << ((qp - 12) / 6); }
constexpr int kPenSplit = 8, kPenNxN = 32;   // tuned on tools/rd_codecs.py content (open-loop SADs favour NxN)
SK_HD int intra_mode_bias(int mode, int qp) {   // 2 x lambda_sad (tuned with the CU quadtree)
    return intra_mode_basic(mode) ? 0 : 2 * (qp < 12 ? 1 : 1 << ((qp - 12) / 6));
}

// Neighbour availability of transform blocks (z order inside the unit) for the intra
// reference samples: bit 0 below-left, 1 left, 2 above-left, 3 above, 4 above-right.
// `nbm`: the same bits for the unit's neighbour units (unit_nbm: z-scan availability on
// the CTB grid - the unit below-left is decoded for a CTB's z0, the one above-right is not
// for its z3).
enum { AV_BL = 1, AV_L = 2, AV_TL = 4, AV_T = 8, AV_TR = 16 };
SK_HD int unit_nbm(const UnitGrid& g, const SliceMap& m, int ux, int uy) {
    return (g.avail(m, ux, uy, ux - 1, uy + 1) ? AV_BL : 0) | (g.avail(m, ux, uy, ux - 1, uy) ? AV_L : 0) |
           (g.avail(m, ux, uy, ux - 1, uy - 1) ? AV_TL : 0) | (g.avail(m, ux, uy, ux, uy - 1) ? AV_T : 0) |
           (g.avail(m, ux, uy, ux + 1, uy - 1) ? AV_TR : 0);
}
// 16x16 TU (the whole unit): its references are the neighbour units'.
SK_HD int cu_avail(int nbm) { return nbm; }
// Whether 4x4 block (ux, uy) of the unit's neighbourhood (-1 .. 7) is decoded before the
// block with z-order index z of the unit.
SK_HD bool unit_avail(int ux, int uy, int z, int nbm) {
    if (uy < 0) return ux < 0 ? (nbm & AV_TL) != 0 : (ux < 4 ? (nbm & AV_T) != 0 : (ux < 8 && (nbm & AV_TR)));
    if (ux >= 4) return false;
    if (uy >= 4) return ux < 0 && uy < 8 && (nbm & AV_BL);
    if (ux < 0) return (nbm & AV_L) != 0;
    return zorder4(ux, uy) < z;
}
// The TU of s x s blocks (s = 1, 2) at block (bx, by) of the unit: its neighbour segments
// are whole blocks of earlier TUs or outside units, so their first block decides.
SK_HD int tu_avail_at(int bx, int by, int s, int nbm) {
    const int z = zorder4(bx, by);
    return (unit_avail(bx - 1, by + s, z, nbm) ? AV_BL : 0) | (unit_avail(bx - 1, by, z, nbm) ? AV_L : 0) |
           (unit_avail(bx - 1, by - 1, z, nbm) ? AV_TL : 0) | (unit_avail(bx, by - 1, z, nbm) ? AV_T : 0) |
           (unit_avail(bx + s, by - 1, z, nbm) ? AV_TR : 0);
}
// 8x8 luma / 4x4 chroma node q of a split unit.
SK_HD int tu_avail(int q, int nbm) { return tu_avail_at(2 * (q & 1), 2 * (q >> 1), 2, nbm); }

// Encoder RD model shared by the CPU reference and the kernels (TU split and TU zeroing
// decisions): J = 512 * SSE + lambda_q8 * R, R in half bits, lambda = 0.57 * 2^((QP - 12) / 3)
// (HM's), a coded TU ~4 bits plus, per non-zero level, 2.5 bits + 2 bits per doubling.
SK_HD int rd_lambda_q8(int qp) {
    qp = qp < 69 ? qp : 69;   // qp + the rate controller's lam_boost (ratecontrol.h kLamBoostMax)
    const int e = qp > 12 ? qp - 12 : 0;
    const int b = e % 3 == 0 ? 146 : (e % 3 == 1 ? 184 : 232);
    return b << (e / 3);
}
SK_HD int level_rate_half(int l) {
    if (!l) return 0;
    const uint32_t a = (uint32_t)sk_abs(l);
    return 5 + 4 * (31 - __builtin_clz(a));
}
constexpr int kTuRateHalf = 8;      // cbf / last position of a coded TU
constexpr int kSplitRateHalf = 12;  // the split CU's extra cbf flags
constexpr int kSplit8RateHalf = 8;  // an 8x8 node's split flag and extra cbf_luma flags

// Most probable modes (8.4.2) from the left (cand_a) and above (cand_b) PU modes (DC
// when unavailable, not intra, or above the CTB).
SK_HD void intra_mpm(int cand_a, int cand_b, int* list) {
    if (cand_a == cand_b) {
        if (cand_a < 2) {
            list[0] = 0; list[1] = 1; list[2] = 26;
        } else {
            list[0] = cand_a;
            list[1] = 2 + ((cand_a + 29) % 32);
            list[2] = 2 + ((cand_a - 2 + 1) % 32);
        }
    } else {
        list[0] = cand_a;
        list[1] = cand_b;
        list[2] = (cand_a != 0 && cand_b != 0) ? 0 : ((cand_a != 1 && cand_b != 1) ? 1 : 26);
    }
}
// Bins of a luma mode given its MPM list: prev_intra_luma_pred_flag, then (written after
// every PU's flag) mpm_idx (TR, bypass) or rem_intra_luma_pred_mode (5 bypass bins).
SK_HD int mpm_hit(int m, const int* mpm) { return m == mpm[0] ? 0 : (m == mpm[1] ? 1 : (m == mpm[2] ? 2 : -1)); }
template <class W>
SK_HD void code_mpm_rest(W& w, int m, const int* mpm) {
    const int hit = mpm_hit(m, mpm);
    if (hit >= 0) {
        if (hit == 0) w.bypass(0, 1);
        else w.bypass(hit == 1 ? 2u : 3u, 2);
        return;
    }
    int s[3] = {mpm[0], mpm[1], mpm[2]};
    if (s[0] > s[1]) { int t = s[0]; s[0] = s[1]; s[1] = t; }
    if (s[0] > s[2]) { int t = s[0]; s[0] = s[2]; s[2] = t; }
    if (s[1] > s[2]) { int t = s[1]; s[1] = s[2]; s[2] = t; }
    int rem = m;
    for (int i = 2; i >= 0; i--)
        if (rem > s[i]) rem--;
    w.bypass((uint32_t)rem, 5);
}

// ---------------------------------------------------------------------------
// Luma motion compensation (8.5.3.3.3.1): quarter-pel vectors, 8-tap filters fL
// (Table 8-12), 8-bit samples (shift1 = 0, shift2 = 6), uni-prediction weighted to 8 bits
// (shift3 = 6). Written in the separable form every implementation here uses:
//   h(r) = xFrac ? sum_i fL[xFrac][i] ref(x + i - 3, r) : ref(x, r) << 6
//   v    = yFrac ? (sum_k fL[yFrac][k] h(y + k - 3)) >> 6 : h(y)
// which equals the spec's three cases (the << 6 / >> 6 pair is exact).
SK_TABLE int8_t HEVC_LUMA_FILTER[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                          {-1, 4, -10, 58, 17, -5, 1, 0},
                                          {-1, 4, -11, 40, 40, -11, 4, -1},
                                          {0, 1, -5, 17, 58, -10, 4, -1}};
SK_HD int luma_mc_sample(const uint8_t* plane, int stride, int w, int h, int x, int y, int mvx, int mvy) {
    const int xi = x + (mvx >> 2), yi = y + (mvy >> 2), fx = mvx & 3, fy = mvy & 3;
    auto P = [&](int xx, int yy) { return (int)plane[(size_t)sk_clip(yy, 0, h - 1) * stride + sk_clip(xx, 0, w - 1)]; };
    auto H = [&](int yy) {
        if (!fx) return P(xi, yy) << 6;
        int s = 0;
        for (int i = 0; i < 8; i++) s += HEVC_LUMA_FILTER[fx][i] * P(xi + i - 3, yy);
        return s;
    };
    int v;
    if (!fy) {
        v = H(yi);
    } else {
        v = 0;
        for (int k = 0; k < 8; k++) v += HEVC_LUMA_FILTER[fy][k] * H(yi + k - 3);
        v >>= 6;
    }
    return sk_clip255((v + 32) >> 6);
}

// Chroma motion compensation (8.5.3.3.3.3) for integer or fractional luma vectors in
// quarter-pel (4:2:0: chroma fraction in 1/8), uni-prediction weighted to 8 bits.
SK_HD int chroma_filter_tap(int frac, int i) {
    // fC[frac][i] (Table 8-13): {0,64,0,0} {-2,58,10,-2} {-4,54,16,-2} {-6,46,28,-4}
    // {-4,36,36,-4} {-4,28,46,-6} {-2,16,54,-4} {-2,10,58,-2}; outer taps packed as
    // negated nibbles, inner taps as bytes.
    const int outer = (int)((0x2242644446242200ull >> (8 * frac + 4 * (i == 3))) & 15);
    const uint64_t inner0 = 0x0A101C242E363A40ull, inner1 = 0x3A362E241C100A00ull;
    if (i == 0 || i == 3) return -outer;
    return (int)(((i == 1 ? inner0 : inner1) >> (8 * frac)) & 0xff);
}
SK_HD int chroma_mc_sample(const uint8_t* plane, int stride, int w, int h, int xc, int yc, int mvx, int mvy) {
    const int xi = xc + (mvx >> 3), yi = yc + (mvy >> 3), fx = mvx & 7, fy = mvy & 7;
    auto P = [&](int x, int y) { return (int)plane[(size_t)sk_clip(y, 0, h - 1) * stride + sk_clip(x, 0, w - 1)]; };
    int v;
    if (fx == 0 && fy == 0) {
        v = P(xi, yi) << 6;
    } else if (fy == 0) {
        v = 0;
        for (int i = 0; i < 4; i++) v += chroma_filter_tap(fx, i) * P(xi + i - 1, yi);
    } else if (fx == 0) {
        v = 0;
        for (int i = 0; i < 4; i++) v += chroma_filter_tap(fy, i) * P(xi, yi + i - 1);
    } else {
        v = 0;
        for (int r = 0; r < 4; r++) {
            int t = 0;
            for (int i = 0; i < 4; i++) t += chroma_filter_tap(fx, i) * P(xi + i - 1, yi + r - 1);
            v += chroma_filter_tap(fy, r) * t;   // shift1 = 0 for 8-bit
        }
        v >>= 6;   // shift2
    }
    return sk_clip255((v + 32) >> 6);   // default weighted prediction: shift 14 - 8
}

// ---------------------------------------------------------------------------
// Merge candidates (8.5.3.2.2-4) and AMVP predictors (8.5.3.2.6-7) of a PU of a P slice
// with one reference picture (refIdx 0 everywhere, so no scaling): neighbours A0 below-left,
// A1 left, B0 above-right, B1 above, B2 above-left of the PU, `av` = available and inter
// (P slices carry inter CUs only). MVs quarter-pel.
struct NbMv {
    bool av;
    int mvx, mvy;
};
constexpr int kMaxMergeCand = 5;
SK_HD int merge_list(const NbMv& A1, const NbMv& B1, const NbMv& B0, const NbMv& A0, const NbMv& B2, int* lx, int* ly) {
    int n = 0;
    auto same = [](const NbMv& p, const NbMv& q) { return p.av && q.av && p.mvx == q.mvx && p.mvy == q.mvy; };
    const bool a1 = A1.av;
    const bool b1 = B1.av && !same(A1, B1);
    const bool b0 = B0.av && !same(B1, B0);
    const bool a0 = A0.av && !same(A1, A0);
    const bool b2 = B2.av && !same(A1, B2) && !same(B1, B2) && ((int)a1 + (int)b1 + (int)b0 + (int)a0) != 4;
    if (a1) { lx[n] = A1.mvx; ly[n] = A1.mvy; n++; }
    if (b1) { lx[n] = B1.mvx; ly[n] = B1.mvy; n++; }
    if (b0) { lx[n] = B0.mvx; ly[n] = B0.mvy; n++; }
    if (a0) { lx[n] = A0.mvx; ly[n] = A0.mvy; n++; }
    if (b2) { lx[n] = B2.mvx; ly[n] = B2.mvy; n++; }
    while (n < kMaxMergeCand) { lx[n] = 0; ly[n] = 0; n++; }   // zero candidates (refIdx 0)
    return n;
}
SK_HD void amvp_list(const NbMv& A0, const NbMv& A1, const NbMv& B0, const NbMv& B1, const NbMv& B2, int* px, int* py) {
    // A: first available of A0, A1 (same reference picture: all inter neighbours here)
    bool avA = A0.av || A1.av;
    int ax = A0.av ? A0.mvx : A1.mvx, ay = A0.av ? A0.mvy : A1.mvy;
    bool avB = false;
    int bx = 0, by = 0;
    if (B0.av) { avB = true; bx = B0.mvx; by = B0.mvy; }
    else if (B1.av) { avB = true; bx = B1.mvx; by = B1.mvy; }
    else if (B2.av) { avB = true; bx = B2.mvx; by = B2.mvy; }
    const bool is_scaled = A0.av || A1.av;   // availableA0 || availableA1
    if (!is_scaled && avB) { avA = true; ax = bx; ay = by; }
    // (!is_scaled: B re-derived with scaling allowed gives the identical vector - same POC distance)
    int n = 0;
    if (avA) { px[n] = ax; py[n] = ay; n++; }
    if (avB && !(avA && ax == bx && ay == by)) { px[n] = bx; py[n] = by; n++; }
    while (n < 2) { px[n] = 0; py[n] = 0; n++; }
}

// The five spatial neighbours of a PU (luma position (xp, yp), size pw x ph) of the CU at
// (xc, yc), size nc, part index pi, over the unit motion field: mv(ux, uy) gives a unit's
// vector; availability 6.4.2 - a neighbour inside the current CU is available only when it
// lies in PU 0 and this is PU 1 (sameCb), one outside needs z-scan availability on the CTB
// grid (UnitGrid::avail from the CU's first unit).
struct PuNb {
    NbMv A0, A1, B0, B1, B2;
};
template <class MV>
SK_HD PuNb pu_neighbours(const UnitGrid& g, const SliceMap& m, MV mv, int xc, int yc, int nc, int xp, int yp, int pw,
                         int ph, int pi) {
    auto at = [&](int xn, int yn) {
        NbMv r;
        r.av = false;
        r.mvx = r.mvy = 0;
        if (xn < 0 || yn < 0 || xn >= 16 * g.W16 || yn >= 16 * g.H16) return r;
        const bool in_cu = xn >= xc && yn >= yc && xn < xc + nc && yn < yc + nc;
        if (in_cu) r.av = pi == 1 && !(xn >= xp && yn >= yp && xn < xp + pw && yn < yp + ph);
        else r.av = g.avail(m, xc >> 4, yc >> 4, xn >> 4, yn >> 4);
        if (r.av) mv(xn >> 4, yn >> 4, &r.mvx, &r.mvy);
        return r;
    };
    PuNb n;
    n.A1 = at(xp - 1, yp + ph - 1);
    n.B1 = at(xp + pw - 1, yp - 1);
    n.B0 = at(xp + pw, yp - 1);
    n.A0 = at(xp - 1, yp + ph);
    n.B2 = at(xp - 1, yp - 1);
    return n;
}
// Merge list of a PU (8.5.3.2.3: PART_Nx2N / 2NxN part 1 drop A1 / B1, the candidate of part 0).
SK_HD void pu_merge_list(PuNb n, int part, int pi, int* lx, int* ly) {
    if (pi == 1 && part == PART_Nx2N) n.A1.av = false;
    if (pi == 1 && part == PART_2NxN) n.B1.av = false;
    merge_list(n.A1, n.B1, n.B0, n.A0, n.B2, lx, ly);
}
SK_HD void pu_amvp_list(const PuNb& n, int* px, int* py) { amvp_list(n.A0, n.A1, n.B0, n.B1, n.B2, px, py); }
// Geometry of PU pi of a CU at (xc, yc) of size nc for a Part.
SK_HD void pu_rect(int part, int pi, int xc, int yc, int nc, int* xp, int* yp, int* pw, int* ph) {
    *xp = xc + (part == PART_Nx2N && pi ? nc / 2 : 0);
    *yp = yc + (part == PART_2NxN && pi ? nc / 2 : 0);
    *pw = part == PART_Nx2N ? nc / 2 : nc;
    *ph = part == PART_2NxN ? nc / 2 : nc;
}
// EGk bypass bin count and value (9.3.3.3).
SK_HD int egk_bins(uint32_t v, int k, uint32_t* bits) {
    int n = 0;
    uint32_t out = 0;
    while (v >= (1u << k)) {
        out = (out << 1) | 1u;
        n++;
        v -= 1u << k;
        k++;
    }
    out = (out << 1);
    n++;
    out = (out << k) | v;
    n += k;
    *bits = out;
    return n;
}
SK_HD int mvd_bits_est(int d) {   // abs_mvd coding cost estimate in bins (AMVP predictor choice)
    const int a = sk_abs(d);
    if (a == 0) return 1;
    if (a == 1) return 3;
    uint32_t b;
    return 3 + egk_bins((uint32_t)(a - 2), 1, &b);
}


// Merge / AMVP choice of a PU with vector (mvx, mvy) from its candidate lists (the first
// merge candidate that equals it, else the AMVP predictor with the cheaper difference).
SK_HD void pu_choose(CuInfo& cu, int mvx, int mvy, const int* mlx, const int* mly, const int* px, const int* py) {
    int midx = -1;
    for (int i = 0; i < kMaxMergeCand && midx < 0; i++)
        if (mlx[i] == mvx && mly[i] == mvy) midx = i;
    cu.mvx = (int16_t)mvx;
    cu.mvy = (int16_t)mvy;
    if (midx >= 0) {
        cu.mode = CU_MERGE;
        cu.merge_idx = (uint8_t)midx;
        cu.mvp_idx = 0;
        cu.mvdx = cu.mvdy = 0;
    } else {
        cu.mode = CU_AMVP;
        cu.merge_idx = 0;
        const int c0 = mvd_bits_est(mvx - px[0]) + mvd_bits_est(mvy - py[0]);
        const int c1 = mvd_bits_est(mvx - px[1]) + mvd_bits_est(mvy - py[1]);
        const int k = c1 < c0 ? 1 : 0;
        cu.mvp_idx = (uint8_t)k;
        cu.mvdx = (int16_t)(mvx - px[k]);
        cu.mvdy = (int16_t)(mvy - py[k]);
    }
}

// Encoder rate estimates of CU / PU syntax (half bits): the CU32 vs four-CU16 choice
// (hevc_cpu.cpp cu32_decide and k_hevc_inter run the same rule).
SK_HD int pu_hdr_half(int mode, int merge_idx, int mvdx, int mvdy) {   // merge_flag + idx, or mvd + mvp flag
    return mode == CU_AMVP ? 6 + 2 * (mvd_bits_est(mvdx) + mvd_bits_est(mvdy)) : 2 + 2 * merge_idx;
}
SK_HD int cu16_hdr_half(const CuInfo& cu) {   // split_cu_flag, cu_skip_flag, pred mode, part, PU, root cbf
    if (cu.mode == CU_SKIP) return 4 + 2 * cu.merge_idx;
    return 8 + pu_hdr_half(cu.mode, cu.merge_idx, cu.mvdx, cu.mvdy) + (cu.mode == CU_AMVP ? 2 : 0);
}
SK_HD int cu32_hdr_half(int part, const CuInfo& pu0, const CuInfo& pu1, bool skip) {
    if (skip) return 2 + 2 * pu0.merge_idx;
    return 6 + (part == PART_2Nx2N ? 2 : 4) + pu_hdr_half(pu0.mode, pu0.merge_idx, pu0.mvdx, pu0.mvdy) +
           (part != PART_2Nx2N ? pu_hdr_half(pu1.mode, pu1.merge_idx, pu1.mvdx, pu1.mvdy) : 0);
}
// The PU split a CTB's four unit vectors allow (-1: none): all equal 2Nx2N, rows 2NxN, columns Nx2N.
SK_HD int cu32_part(const int* mx, const int* my) {
    auto eq = [&](int a, int b) { return mx[a] == mx[b] && my[a] == my[b]; };
    if (eq(0, 1) && eq(0, 2) && eq(0, 3)) return PART_2Nx2N;
    if (eq(0, 1) && eq(2, 3)) return PART_2NxN;
    if (eq(0, 2) && eq(1, 3)) return PART_Nx2N;
    return -1;
}
// The PU (0 / 1) of a CU32 that unit z lies in.
SK_HD int cu32_pu_of(int part, int z) { return part == PART_2NxN ? z >> 1 : (part == PART_Nx2N ? z & 1 : 0); }

// ---------------------------------------------------------------------------
// Syntax binarisation. residual_coding (7.3.8.11) of one TU from raster levels.
// last_sig_coeff prefix (group index) of a position and the first position of a group.
SK_HD int last_group_min(int g) { return (int)((0x310620c418820ull >> (5 * g)) & 31); }
SK_HD int last_prefix(int p) {
    if (p < 4) return p;
    int g = 4;
    while (g < 9 && p >= last_group_min(g + 1)) g++;
    return g;
}

// Four levels (one sub-block row) at an 8-byte aligned address, 16 bits each: one load.
SK_HD uint64_t load4(const int16_t* p) {
    uint64_t v;
    __builtin_memcpy(&v, __builtin_assume_aligned(p, 8), 8);
    return v;
}
// Coefficient accessors: c(i) = the level at raster index i (y * n + x) of the TU,
// c.row4(i) = the four levels at i .. i + 3 (i a multiple of 4).
struct CoefPtr {
    const int16_t* p;
    SK_HD int operator()(int i) const { return p[i]; }
    SK_HD uint64_t row4(int i) const { return load4(p + i); }
};
// The CTB's four units in z order inside the raster unit arrays (CuInfo and coefficient
// slots, `W` units per row). Only a complete CTB's view is dereferenced (CU32s are).
struct Ctb4 {
    const CuInfo* cu;      // the CTB's unit z0
    const int16_t* coef;   // its coefficient slot
    int W;
    SK_HD const CuInfo& operator[](int z) const { return cu[(z >> 1) * W + (z & 1)]; }
    SK_HD const int16_t* slot(int z) const { return coef + (size_t)((z >> 1) * W + (z & 1)) * kCoefPerCu; }
};
// The levels of a CU32's 32x32 TU (and its 16x16 chroma TUs) spread over its units' slots:
// logical index i (kT32Cb / kT32Cr offsets) -> slot of unit z = i / kCoefPerCu.
struct CoefT32 {
    Ctb4 q;
    int base;   // 0 luma, kT32Cb, kT32Cr
    SK_HD int operator()(int i) const {
        const int k = base + i;
        return q.slot(k / kCoefPerCu)[k % kCoefPerCu];
    }
    SK_HD uint64_t row4(int i) const {   // kCoefPerCu % 4 == 0: a row never straddles two slots
        const int k = base + i;
        return load4(q.slot(k / kCoefPerCu) + k % kCoefPerCu);
    }
};
// A 4x4 sub-block's levels as four packed rows.
struct Sb4 {
    uint64_t r0, r1, r2, r3;
    SK_HD bool nz() const { return (r0 | r1 | r2 | r3) != 0; }
    SK_HD int at(int i) const {   // level i (0..15): raster position, or scan position of a scan-ordered Sb4
        // masks, not a select of member addresses (which would pin the struct in scratch)
        const uint64_t m1 = 0 - (uint64_t)((i >> 2) & 1), m2 = 0 - (uint64_t)((i >> 3) & 1);
        const uint64_t lo = (r0 & ~m1) | (r1 & m1), hi = (r2 & ~m1) | (r3 & m1);
        const uint64_t v = (lo & ~m2) | (hi & m2);
        return (int16_t)(uint16_t)(v >> (16 * (i & 3)));
    }
    SK_HD void set(int i, int x) {   // i a compile-time constant after unrolling
        const uint64_t m = (uint64_t)(uint16_t)x << (16 * (i & 3));
        if (i < 4) r0 |= m; else if (i < 8) r1 |= m; else if (i < 12) r2 |= m; else r3 |= m;
    }
};
template <class C>
SK_HD Sb4 load_sb(C c, int n, int xs, int ys) {
    const int o = ys * 4 * n + xs * 4;
    return Sb4{c.row4(o), c.row4(o + n), c.row4(o + 2 * n), c.row4(o + 3 * n)};
}

// g1ctx (greater1 context state) a sub-block with a significant level leaves behind: its
// first eight significant levels in reverse scan order.
SK_HD int sb_g1(const Sb4& s, int scan) {
    int g1ctx = 1, ng1 = 0;
    for (int k = 15; k >= 0 && ng1 < 8; k--) {
        const int v = s.at(scan4_raster(scan, k));
        if (!v) continue;
        ng1++;
        if (g1ctx > 0) g1ctx = sk_abs(v) > 1 ? 0 : g1ctx + 1;
    }
    return g1ctx;
}

// residual_coding (7.3.8.11), split into the TU prologue (code_last) and one sub-block's
// syntax (code_sb); code_residual runs them over a TU in coding order.
//
// The prologue: transform_skip_flag (4x4), the last significant position (sub-block last_i,
// scan position last_n).
template <class W>
SK_HD void code_last(W& w, int log2n, int cidx, int scan, int ts, int last_i, int last_n) {
    const int sbw = 1 << (log2n - 2);
    if (log2n == 2) w.ctx(CTX_TS + (cidx ? 1 : 0), ts);   // transform_skip_flag (PPS enables it)
    const int lsr = sb_scan_raster(log2n, scan, last_i);
    int lx = (lsr % sbw) * 4 + (scan4_raster(scan, last_n) & 3);
    int ly = (lsr / sbw) * 4 + (scan4_raster(scan, last_n) >> 2);
    if (scan == SCAN_VER) { const int t = lx; lx = ly; ly = t; }   // coded swapped (7.4.9.11)
    // last_sig_coeff_x/y_prefix (TR, cMax 2*log2n - 1), then suffixes (FL, bypass)
    const int off = cidx == 0 ? 3 * (log2n - 2) + ((log2n - 1) >> 2) : 15;
    const int shift = cidx == 0 ? (log2n + 1) >> 2 : log2n - 2;
    const int cmax = 2 * log2n - 1;
    const int px = last_prefix(lx), py = last_prefix(ly);
    for (int b = 0; b < px; b++) w.ctx(CTX_LAST_X + off + (b >> shift), 1);
    if (px < cmax) w.ctx(CTX_LAST_X + off + (px >> shift), 0);
    for (int b = 0; b < py; b++) w.ctx(CTX_LAST_Y + off + (b >> shift), 1);
    if (py < cmax) w.ctx(CTX_LAST_Y + off + (py >> shift), 0);
    if (px > 3) w.bypass((uint32_t)(lx - last_group_min(px)), (px >> 1) - 1);
    if (py > 3) w.bypass((uint32_t)(ly - last_group_min(py)), (py >> 1) - 1);
}
// Last significant position of a TU: sub-block scan index (-1: no level) and position.
SK_HD int sb_last_pos(const Sb4& s, int scan) {
    for (int k = 15; k >= 0; k--)
        if (s.at(scan4_raster(scan, k))) return k;
    return -1;
}
// The syntax of sub-block i (scan order; levels s in raster order, at (xs, ys) of the
// sub-block grid) from coded_sub_block_flag to coeff_abs_level_remaining. right / below:
// the neighbours' coded_sub_block_flag; first_g1 / c1_in: whether a sub-block with a
// significant level was coded before in the TU, and the greater1 state it left (HM c1).
// The state this sub-block leaves is sb_g1's when it holds a level (else unchanged).
template <class W>
SK_HD void code_sb(W& w, const Sb4& s, int log2n, int cidx, int scan, int i, int last_i, int last_n, int xs, int ys,
                   int right, int below, bool first_g1, int c1_in) {
    bool coded = s.nz();
    bool infer_dc = false;
    if (i < last_i && i > 0) {
        w.ctx(CTX_CSBF + sk_min(1, right + below) + (cidx ? 2 : 0), coded ? 1 : 0);
        infer_dc = true;
    } else {
        coded = true;   // inferred for the DC and last sub-blocks
    }
    if (!coded) return;   // no flags beyond coded_sub_block_flag
    const int prev_csbf = right | (below << 1);
    Sb4 lev{0, 0, 0, 0};   // the sub-block's levels in scan order (registers, no local array)
#pragma unroll
    for (int k = 0; k < 16; k++) lev.set(k, s.at(scan4_raster(scan, k)));
    // sig_coeff_flag
    uint32_t sig = 0;
    const int start = (i == last_i) ? last_n - 1 : 15;
    if (i == last_i) sig |= 1u << last_n;
#pragma unroll 1
    for (int k = start; k >= 0; k--) {
        const int r = scan4_raster(scan, k);
        const int xc = xs * 4 + (r & 3), yc = ys * 4 + (r >> 2);
        const bool sg = lev.at(k) != 0;
        if (k == 0 && infer_dc) {   // inferred 1 when no other flag of the sub-block was 1
            sig |= 1u;
            break;
        }
        int sctx;
        if (log2n == 2) {   // ctxIdxMap (4x4 TUs)
            sctx = (int)((0x877886654325410ull >> (4 * ((yc << 2) + xc))) & 15);
        } else if (xc + yc == 0) {
            sctx = 0;
        } else {
            const int xp = xc & 3, yp = yc & 3;
            if (prev_csbf == 0) sctx = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
            else if (prev_csbf == 1) sctx = yp == 0 ? 2 : (yp == 1 ? 1 : 0);
            else if (prev_csbf == 2) sctx = xp == 0 ? 2 : (xp == 1 ? 1 : 0);
            else sctx = 2;
            if (cidx == 0) {
                if (xs > 0 || ys > 0) sctx += 3;
                sctx += log2n == 3 ? (scan == SCAN_DIAG ? 9 : 15) : 21;
            } else {
                sctx += log2n == 3 ? 9 : 12;
            }
        }
        w.ctx(CTX_SIG + (cidx == 0 ? sctx : 27 + sctx), sg ? 1 : 0);
        if (sg) {
            sig |= 1u << k;
            infer_dc = false;
        }
    }
    if (!sig) return;
    // greater1 / greater2
    int ctx_set = (i == 0 || cidx > 0) ? 0 : 2;
    if (!first_g1 && c1_in == 0) ctx_set++;
    int g1ctx = 1, ng1 = 0, last_g1_pos = -1;
    uint32_t g1 = 0;
#pragma unroll 1
    for (int k = 15; k >= 0; k--) {
        if (!((sig >> k) & 1)) continue;
        if (ng1 < 8) {
            const int f = sk_abs(lev.at(k)) > 1;
            w.ctx(CTX_GT1 + ctx_set * 4 + sk_min(3, g1ctx) + (cidx ? 16 : 0), f);
            ng1++;
            if (f) {
                g1 |= 1u << k;
                if (last_g1_pos < 0) last_g1_pos = k;
            }
            if (g1ctx > 0) g1ctx = f ? 0 : g1ctx + 1;
        }
    }
    int g2 = 0;
    if (last_g1_pos >= 0) {
        g2 = sk_abs(lev.at(last_g1_pos)) > 2;
        w.ctx(CTX_GT2 + ctx_set + (cidx ? 4 : 0), g2);
    }
    // signs
    {
        uint32_t bits = 0;
        int nb = 0;
#pragma unroll 1
        for (int k = 15; k >= 0; k--)
            if ((sig >> k) & 1) {
                bits = (bits << 1) | (lev.at(k) < 0 ? 1u : 0u);
                nb++;
            }
        // nb <= 16: two bypass runs at most
        w.bypass(bits, nb);
    }
    // coeff_abs_level_remaining
    int rice = 0, nsig = 0;
#pragma unroll 1
    for (int k = 15; k >= 0; k--) {
        if (!((sig >> k) & 1)) continue;
        const int a = sk_abs(lev.at(k));
        const int base = 1 + (int)((g1 >> k) & 1) + (k == last_g1_pos ? g2 : 0);
        const int thr = nsig < 8 ? (k == last_g1_pos ? 3 : 2) : 1;
        if (base == thr) {
            const uint32_t rem = (uint32_t)(a - base);
            if (rem < (3u << rice)) {
                const int len = (int)(rem >> rice);
                w.bypass((1u << (len + 1)) - 2u, len + 1);
                if (rice) w.bypass(rem & ((1u << rice) - 1u), rice);
            } else {
                uint32_t v = rem - (3u << rice);
                int len = rice;
                while (v >= (1u << len)) {
                    v -= 1u << len;
                    len++;
                }
                const int ones = 3 + len + 1 - rice;   // prefix: (ones - 1) ones then a zero
                // prefix may exceed 32 bins only for levels far beyond kMaxLevel
                int pre = ones;
                while (pre > 0) {
                    const int k2 = pre > 16 ? 16 : pre;
                    pre -= k2;
                    const uint32_t chunk = pre == 0 ? ((1u << k2) - 2u) : ((1u << k2) - 1u);
                    w.bypass(chunk, k2);
                }
                w.bypass(v, len);
            }
            if (a > 3 * (1 << rice)) rice = sk_min(rice + 1, 4);
        }
        nsig++;
    }
}

// residual_coding of one TU from raster levels - or of the sub-blocks with scan index in
// [lo, hi] only: a CU32's 32x32 and 16x16 TUs are binarised in pieces, one per unit (the
// units' bin slots are the chunks of the chunk-parallel coder). The piece that holds the
// last significant sub-block writes the prologue; a later piece starts from the greater1
// state the sub-blocks coded before it leave (that of the nearest one with a level).
// A writer with W::kWave set (k_hevc_bins) codes the sub-blocks on the lanes of a wave.
template <class W, class C>
SK_HD void code_residual_serial(W& w, C c, int log2n, int cidx, int scan, int ts, int lo, int hi);
template <class W, class C>
SK_HD void code_residual(W& w, C c, int log2n, int cidx, int scan = SCAN_DIAG, int ts = 0, int lo = 0, int hi = 63) {
    if constexpr (W::kWave) w.residual(c, log2n, cidx, scan, ts, lo, hi);
    else code_residual_serial(w, c, log2n, cidx, scan, ts, lo, hi);
}
template <class W, class C>
SK_HD void code_residual_serial(W& w, C c, int log2n, int cidx, int scan, int ts, int lo, int hi) {
    {
        const int n = 1 << log2n;
        const int sbw = n >> 2;                     // sub-blocks per row
        const int nsb = sbw * sbw;
        int last_i = -1, last_n = -1;
#pragma unroll 1
        for (int i = nsb - 1; i >= 0; i--) {
            const int sr = sb_scan_raster(log2n, scan, i);
            const Sb4 s = load_sb(c, n, sr % sbw, sr / sbw);
            if (!s.nz()) continue;
            last_i = i;
            last_n = sb_last_pos(s, scan);
            break;
        }
        if (last_i < 0) return;   // callers only code TUs with cbf = 1
        const int i0 = last_i < hi ? last_i : hi;
        if (i0 < lo) return;      // a piece above the last sub-block: nothing to code
        if (i0 == last_i) code_last(w, log2n, cidx, scan, ts, last_i, last_n);
        // coded_sub_block_flag per sub-block (raster in the sub-block grid). The right / below
        // neighbours a sub-block's contexts read come later in every scan, and nothing after
        // last_i is coded: the flags of scan positions lo .. last_i are all that is read.
        uint64_t csbf = 0;
#pragma unroll 1
        for (int i = lo; i <= last_i; i++) {
            const int sr = sb_scan_raster(log2n, scan, i);
            if (load_sb(c, n, sr % sbw, sr / sbw).nz()) csbf |= 1ull << sr;
        }
        int c1 = 1;   // greater1 state carried between sub-blocks
        bool first_g1 = true;
#pragma unroll 1
        for (int i = i0 + 1; i <= last_i && first_g1; i++) {   // a later piece: the state so far
            const int sr = sb_scan_raster(log2n, scan, i);
            const Sb4 s = load_sb(c, n, sr % sbw, sr / sbw);
            if (s.nz()) {
                c1 = sb_g1(s, scan);
                first_g1 = false;
            }
        }
#pragma unroll 1
        for (int i = i0; i >= lo; i--) {
            const int sr = sb_scan_raster(log2n, scan, i), xs = sr % sbw, ys = sr / sbw;
            const int right = (xs + 1 < sbw) ? (int)((csbf >> (sr + 1)) & 1) : 0;
            const int below = (ys + 1 < sbw) ? (int)((csbf >> (sr + sbw)) & 1) : 0;
            const Sb4 s = load_sb(c, n, xs, ys);
            code_sb(w, s, log2n, cidx, scan, i, last_i, last_n, xs, ys, right, below, first_g1, c1);
            if (s.nz()) {
                c1 = sb_g1(s, scan);
                first_g1 = false;
            }
        }
    }
}

// merge_idx: TR cMax 4, first bin context coded, bins 1..3 bypass.
template <class W>
SK_HD void code_merge_idx(W& w, int merge_idx) {
    w.ctx(CTX_MERGE_IDX, merge_idx > 0);
    if (merge_idx > 0) {
        const int rest = merge_idx - 1;
        if (rest < 3) w.bypass((1u << (rest + 1)) - 2u, rest + 1);
        else w.bypass(7u, 3);
    }
}
// prediction_unit (7.3.8.6) of a non-skipped inter PU: merge_flag, then merge_idx or
// mvd_coding (7.3.8.9) and mvp_l0_flag.
template <class W>
SK_HD void code_pu(W& w, const CuInfo& cu) {
    w.ctx(CTX_MERGE_FLAG, cu.mode == CU_MERGE);
    if (cu.mode == CU_MERGE) {
        code_merge_idx(w, cu.merge_idx);
        return;
    }
    const int ax = sk_abs(cu.mvdx), ay = sk_abs(cu.mvdy);
    w.ctx(CTX_MVD_G0, ax > 0);
    w.ctx(CTX_MVD_G0, ay > 0);
    if (ax > 0) w.ctx(CTX_MVD_G1, ax > 1);
    if (ay > 0) w.ctx(CTX_MVD_G1, ay > 1);
    if (ax > 0) {
        if (ax > 1) {
            uint32_t b;
            const int nb = egk_bins((uint32_t)(ax - 2), 1, &b);
            w.bypass(b, nb);
        }
        w.bypass(cu.mvdx < 0 ? 1u : 0u, 1);
    }
    if (ay > 0) {
        if (ay > 1) {
            uint32_t b;
            const int nb = egk_bins((uint32_t)(ay - 2), 1, &b);
            w.bypass(b, nb);
        }
        w.bypass(cu.mvdy < 0 ? 1u : 0u, 1);
    }
    w.ctx(CTX_MVP, cu.mvp_idx);
}

// transform_tree (7.3.8.8) of a 16x16 node: a CU16's root (depth 0) or a CU32's node
// (depth 1, under the root's chroma cbfs pcb / pcr): split_transform_flag at log2 4, the
// chroma cbfs, then either the 16x16 transform unit or four 8x8 nodes (each one 8x8 TU or
// four 4x4 TUs, the node's chroma 4x4 after its last). Intra scans follow each TU's mode.
template <class W>
SK_HD void code_tt16(W& w, const CuInfo& cu, const int16_t* coef, bool intra, int depth, int pcb, int pcr) {
    const int cbf_y = cu.cbf & 1, cbf_cb = (cu.cbf >> 1) & 1, cbf_cr = (cu.cbf >> 2) & 1;
    const bool split = (cu.tu >> 4) & 1;
    w.ctx(CTX_SPLIT_TF + 1, split);   // ctxInc 5 - log2 4 (depth < MaxTrafoDepth: always coded)
    if (depth == 0 || pcb) w.ctx(CTX_CBF_CHROMA + depth, cbf_cb);
    if (depth == 0 || pcr) w.ctx(CTX_CBF_CHROMA + depth, cbf_cr);
    if (!split) {
        if (intra || depth || cbf_cb || cbf_cr) w.ctx(CTX_CBF_LUMA + (depth ? 0 : 1), cbf_y);
        const int sy = intra ? intra_scan(cu.ipm[0], 4, 0) : SCAN_DIAG;
        const int sc = intra ? intra_scan(cu.ipm[0], 3, 1) : SCAN_DIAG;
        if (cbf_y) code_residual(w, CoefPtr{coef}, 4, 0, sy);
        if (cbf_cb) code_residual(w, CoefPtr{coef + kCoefCb}, 3, 1, sc);
        if (cbf_cr) code_residual(w, CoefPtr{coef + kCoefCr}, 3, 2, sc);
        return;
    }
    const int d1 = depth + 1;
    for (int q = 0; q < 4; q++) {
        const int cb = (cu.tuc >> q) & 1, cr = (cu.tuc >> (4 + q)) & 1;
        const bool split8 = (cu.tu >> q) & 1;
        const int mq = cu.ipm[4 * q];
        w.ctx(CTX_SPLIT_TF + 2, split8);   // log2 3
        if (cbf_cb) w.ctx(CTX_CBF_CHROMA + d1, cb);
        if (cbf_cr) w.ctx(CTX_CBF_CHROMA + d1, cr);
        if (!split8) {
            const int cy = (cu.ycbf >> (4 * q)) & 1;
            w.ctx(CTX_CBF_LUMA + 0, cy);
            if (cy) code_residual(w, CoefPtr{coef + 64 * q}, 3, 0, intra ? intra_scan(mq, 3, 0) : SCAN_DIAG);
        } else {
            for (int j = 0; j < 4; j++) {   // depth d1 + 1: chroma of the node after the last 4x4 (blkIdx 3)
                const int cy = (cu.ycbf >> (4 * q + j)) & 1;
                w.ctx(CTX_CBF_LUMA + 0, cy);
                if (cy)
                    code_residual(w, CoefPtr{coef + 64 * q + 16 * j}, 2, 0,
                                  intra ? intra_scan(cu.ipm[4 * q + j], 2, 0) : SCAN_DIAG, (cu.tsy >> (4 * q + j)) & 1);
            }
        }
        const int sc = intra ? intra_scan(mq, 2, 1) : SCAN_DIAG;
        if (cb) code_residual(w, CoefPtr{coef + kCoefCb + 16 * q}, 2, 1, sc, (cu.tsc >> q) & 1);
        if (cr) code_residual(w, CoefPtr{coef + kCoefCr + 16 * q}, 2, 2, sc, (cu.tsc >> (4 + q)) & 1);
    }
}

// transform_tree of intra CU8 q of a CU8-split unit (depth 0, log2 3): PART_2Nx2N codes
// split_transform_flag (one 8x8 TU or four 4x4), PART_NxN infers the split (IntraSplitFlag);
// chroma cbfs at depth 0, the CU8's chroma 4x4 TUs last. Same storage as node q of code_tt16.
template <class W>
SK_HD void code_tt8(W& w, const CuInfo& cu, const int16_t* coef, int q) {
    const int nxn = (cu.cu8 >> q) & 1;
    const int cb = (cu.tuc >> q) & 1, cr = (cu.tuc >> (4 + q)) & 1;
    const bool split8 = nxn || ((cu.tu >> q) & 1);
    const int mq = cu.ipm[4 * q];
    if (!nxn) w.ctx(CTX_SPLIT_TF + 2, split8);
    w.ctx(CTX_CBF_CHROMA + 0, cb);
    w.ctx(CTX_CBF_CHROMA + 0, cr);
    if (!split8) {
        const int cy = (cu.ycbf >> (4 * q)) & 1;
        w.ctx(CTX_CBF_LUMA + 1, cy);   // intra, depth 0
        if (cy) code_residual(w, CoefPtr{coef + 64 * q}, 3, 0, intra_scan(mq, 3, 0));
    } else {
        for (int j = 0; j < 4; j++) {
            const int cy = (cu.ycbf >> (4 * q + j)) & 1;
            w.ctx(CTX_CBF_LUMA + 0, cy);
            if (cy)
                code_residual(w, CoefPtr{coef + 64 * q + 16 * j}, 2, 0, intra_scan(cu.ipm[4 * q + j], 2, 0),
                              (cu.tsy >> (4 * q + j)) & 1);
        }
    }
    const int sc = intra_scan(mq, 2, 1);
    if (cb) code_residual(w, CoefPtr{coef + kCoefCb + 16 * q}, 2, 1, sc, (cu.tsc >> q) & 1);
    if (cr) code_residual(w, CoefPtr{coef + kCoefCr + 16 * q}, 2, 2, sc, (cu.tsc >> (4 + q)) & 1);
}

// The bin entries one unit contributes to its CTB's share of the substream (the chunk
// of the chunk-parallel coder): the CTB's split_cu_flag when it is the CTB's first unit,
// then its CU16 (split_cu_flag, CU syntax or four CU8s) - or, in a CU32, the CU header and
// tree root (z0) and the unit's node (TU split) or piece of the 32x32 / 16x16 TUs (one TU).
// SAO syntax before and end_of_slice_segment_flag after are the caller's (binarize).
struct UnitCtx {
    int z;          // z index of the unit in its CTB
    int first;      // first unit of its CTB in coding order (z0)
    int complete;   // the CTB lies inside the picture (its split_cu_flag is coded)
    int left, top;  // the left / above unit is available (z-scan, slice)
    int row0;       // the unit is in its CTB's top row (an above PU in another CTB counts as DC)
    int p_slice;
};
// MPM candidates of the PU at 4x4 block (bx, by) of the unit.
SK_HD void pu_mpm(const UnitCtx& u, const CuInfo& cu, const CuInfo* L, const CuInfo* T, int bx, int by, int* mpm) {
    const int a = bx > 0 ? cu.ipm[zorder4(bx - 1, by)]
                         : ((u.left && L->mode == CU_INTRA) ? L->ipm[zorder4(3, by)] : 1);
    const int b = by > 0 ? cu.ipm[zorder4(bx, by - 1)]
                         : ((!u.row0 && u.top && T->mode == CU_INTRA) ? T->ipm[zorder4(bx, 3)] : 1);
    intra_mpm(a, b, mpm);
}
// c32: the CTB's four units in z order with their coefficient slots (read by CU32 units).
template <class W>
SK_HD void code_unit(W& w, const UnitCtx& u, const CuInfo& cu, const CuInfo* L, const CuInfo* T, const int16_t* coef,
                     const Ctb4& c32) {
    const int skip_ctx = (u.left && L->mode == CU_SKIP) + (u.top && T->mode == CU_SKIP);
    if (u.first && u.complete) {   // CTB split_cu_flag (cqtDepth 0)
        const int ctx = (u.left && cu_depth(*L) > 0) + (u.top && cu_depth(*T) > 0);
        w.ctx(CTX_SPLIT_CU + ctx, (cu.c32 & kC32) ? 0 : 1);
    }
    if (cu.c32 & kC32) {   // ---- CU32 (inter)
        const int part = c32_part(cu);
        const bool tu32 = (cu.c32 & kC32Tu) != 0;
        int cy = 0, cb = 0, cr = 0;
        for (int k = 0; k < 4; k++) {
            cy |= c32[k].cbf & 1;
            cb |= (c32[k].cbf >> 1) & 1;
            cr |= (c32[k].cbf >> 2) & 1;
        }
        const int root = cy | cb | cr;
        const bool skip = c32[0].mode == CU_SKIP;
        if (u.z == 0) {
            if (u.p_slice) w.ctx(CTX_SKIP + skip_ctx, skip);
            if (skip) {
                code_merge_idx(w, c32[0].merge_idx);
                return;
            }
            w.ctx(CTX_PRED_MODE, 0);
            w.ctx(CTX_PART_MODE, part == PART_2Nx2N);             // "1" 2Nx2N, "01" 2NxN, "00" Nx2N
            if (part != PART_2Nx2N) w.ctx(CTX_PART_MODE1, part == PART_2NxN);
            code_pu(w, c32[0]);
            if (part != PART_2Nx2N) code_pu(w, c32[3]);            // z3 lies in PU 1 of both splits
            if (!(part == PART_2Nx2N && c32[0].mode == CU_MERGE)) w.ctx(CTX_RQT_ROOT_CBF, root);
            if (!root) return;
            w.ctx(CTX_SPLIT_TF + 0, tu32 ? 0 : 1);                 // log2 5, depth 0
            w.ctx(CTX_CBF_CHROMA + 0, cb);
            w.ctx(CTX_CBF_CHROMA + 0, cr);
            if (!tu32) {
                code_tt16(w, cu, coef, false, 1, cb, cr);
                return;
            }
            if (cb || cr) w.ctx(CTX_CBF_LUMA + 1, cy);   // else inferred 1
        }
        if (skip || !root) return;
        if (!tu32) {
            if (u.z) code_tt16(w, cu, coef, false, 1, cb, cr);
            return;
        }
        // one 32x32 TU: luma sub-blocks 63..40 | 39..16 | 15..0 + Cb 15..8 | Cb 7..0 + Cr
        const CoefT32 ty{c32, 0}, tb{c32, kT32Cb}, tr{c32, kT32Cr};
        if (u.z == 0 && cy) code_residual(w, ty, 5, 0, SCAN_DIAG, 0, 40, 63);
        if (u.z == 1 && cy) code_residual(w, ty, 5, 0, SCAN_DIAG, 0, 16, 39);
        if (u.z == 2 && cy) code_residual(w, ty, 5, 0, SCAN_DIAG, 0, 0, 15);
        if (u.z == 2 && cb) code_residual(w, tb, 4, 1, SCAN_DIAG, 0, 8, 15);
        if (u.z == 3 && cb) code_residual(w, tb, 4, 1, SCAN_DIAG, 0, 0, 7);
        if (u.z == 3 && cr) code_residual(w, tr, 4, 2, SCAN_DIAG, 0, 0, 15);
        return;
    }
    // ---- CU16: split_cu_flag at cqtDepth 1 (log2 4 > MinCb 3: coded)
    {
        const int ctx = (u.left && cu_depth(*L) > 1) + (u.top && cu_depth(*T) > 1);
        w.ctx(CTX_SPLIT_CU + ctx, (cu.cu8 >> 4) & 1);
    }
    if (cu.cu8 & 16) {   // four intra CU8s (I slices)
        for (int q = 0; q < 4; q++) {
            const int nxn = (cu.cu8 >> q) & 1, npu = nxn ? 4 : 1;
            w.ctx(CTX_PART_MODE, nxn ? 0 : 1);   // intra at MinCb: "1" 2Nx2N, "0" NxN
            for (int pass = 0; pass < 2; pass++)   // every prev_intra_luma_pred_flag first, then the rest
                for (int p = 0; p < npu; p++) {
                    const int bx = 2 * (q & 1) + (nxn ? (p & 1) : 0), by = 2 * (q >> 1) + (nxn ? (p >> 1) : 0);
                    const int md = cu.ipm[zorder4(bx, by)];
                    int mpm[3];
                    pu_mpm(u, cu, L, T, bx, by, mpm);
                    if (pass == 0) w.ctx(CTX_PREV_INTRA, mpm_hit(md, mpm) >= 0);
                    else code_mpm_rest(w, md, mpm);
                }
            w.ctx(CTX_CHROMA_PRED, 0);   // intra_chroma_pred_mode = 4 (DM)
            code_tt8(w, cu, coef, q);
        }
        return;
    }
    if (u.p_slice) w.ctx(CTX_SKIP + skip_ctx, cu.mode == CU_SKIP);
    if (cu.mode == CU_SKIP) {
        code_merge_idx(w, cu.merge_idx);
        return;
    }
    const bool intra = cu.mode == CU_INTRA;
    if (u.p_slice) w.ctx(CTX_PRED_MODE, intra ? 1 : 0);
    if (intra) {   // PART_2Nx2N (part_mode is coded for intra CUs at MinCb only)
        int mpm[3];
        pu_mpm(u, cu, L, T, 0, 0, mpm);
        w.ctx(CTX_PREV_INTRA, mpm_hit(cu.ipm[0], mpm) >= 0);
        code_mpm_rest(w, cu.ipm[0], mpm);
        w.ctx(CTX_CHROMA_PRED, 0);   // intra_chroma_pred_mode = 4 (DM)
    } else {
        w.ctx(CTX_PART_MODE, 1);     // PART_2Nx2N
        code_pu(w, cu);
        if (cu.mode != CU_MERGE) {
            w.ctx(CTX_RQT_ROOT_CBF, cu.cbf != 0);
            if (cu.cbf == 0) return;
        }
    }
    code_tt16(w, cu, coef, intra, 0, 1, 1);
}

// ---------------------------------------------------------------------------
// Deblocking (8.7.2) for this coding structure: the luma edges on the 8x8 grid that are
// transform or prediction block edges - unit boundaries (CU edges, or TU edges inside a
// CU32 split into 16x16 nodes), the inner edges of split units (8x8 nodes, CU8s), and
// inside a CU32 with one 32x32 TU only its PU edge (2NxN / Nx2N, bS from the motion) - with
// a boundary strength per 4-sample segment, and the chroma edges (bS 2 only) on the
// 8-sample chroma grid (unit boundaries between intra CUs). Edges at the picture border
// and between slices (pps_loop_filter_across_slices_enabled_flag = 0) are not filtered.
// All vertical edges of the picture first, then the horizontal ones on their output.
SK_TABLE uint8_t HEVC_BETA[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  6,  7,
                                  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 22, 24, 26, 28, 30, 32,
                                  34, 36, 38, 40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};   // Table 8-11 beta'
SK_TABLE uint8_t HEVC_TC[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,  1,  1,  1,  1,  1, 1, 1,
                                2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

// cbf_luma of the transform block covering luma sample (x, y) of the unit (0..15).
SK_HD int tu_cbf_y(const CuInfo& c, int x, int y) { return (c.ycbf >> zorder4(x >> 2, y >> 2)) & 1; }
// Boundary strength of an edge segment (8.7.2.4) between CUs p and q (the same CU for an
// inner TU edge) whose luma transform blocks on the two sides have cbf pc / qc.
SK_HD int dbk_bs(const CuInfo& p, const CuInfo& q, int pc, int qc) {
    if (p.mode == CU_INTRA || q.mode == CU_INTRA) return 2;
    if (pc | qc) return 1;   // a luma transform block with coefficients
    const int dx = p.mvx - q.mvx, dy = p.mvy - q.mvy;   // one reference picture: motion only
    return (dx >= 4 || dx <= -4 || dy >= 4 || dy <= -4) ? 1 : 0;
}

// One 4-line luma segment (8.7.2.5.3 decisions, 8.7.2.5.7 filtering). q: the q0
// sample of line 0; step: q0 -> q1 (1 across a vertical edge, the stride across a
// horizontal one); along: line 0 -> line 1.
SK_HD void dbk_luma_segment(uint8_t* q, int step, int along, int bs, int qp) {
    const int beta = HEVC_BETA[sk_clip(qp, 0, 51)];
    const int tc = HEVC_TC[sk_clip(qp + 2 * (bs - 1), 0, 53)];
    auto P = [&](int ln, int i) -> int { return q[ln * along - (i + 1) * step]; };
    auto Q = [&](int ln, int i) -> int { return q[ln * along + i * step]; };
    const int dp0 = sk_abs(P(0, 2) - 2 * P(0, 1) + P(0, 0)), dp3 = sk_abs(P(3, 2) - 2 * P(3, 1) + P(3, 0));
    const int dq0 = sk_abs(Q(0, 2) - 2 * Q(0, 1) + Q(0, 0)), dq3 = sk_abs(Q(3, 2) - 2 * Q(3, 1) + Q(3, 0));
    const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3, dp = dp0 + dp3, dq = dq0 + dq3;
    if (dpq0 + dpq3 >= beta) return;
    auto strong = [&](int ln, int dpq) {
        return 2 * dpq < (beta >> 2) && sk_abs(P(ln, 3) - P(ln, 0)) + sk_abs(Q(ln, 0) - Q(ln, 3)) < (beta >> 3) &&
               sk_abs(P(ln, 0) - Q(ln, 0)) < ((5 * tc + 1) >> 1);
    };
    const bool de2 = strong(0, dpq0) && strong(3, dpq3);
    const bool dep = dp < ((beta + (beta >> 1)) >> 3), deq = dq < ((beta + (beta >> 1)) >> 3);
    for (int ln = 0; ln < 4; ln++) {
        uint8_t* o = q + ln * along;
        const int p0 = P(ln, 0), p1 = P(ln, 1), p2 = P(ln, 2), p3 = P(ln, 3);
        const int q0 = Q(ln, 0), q1 = Q(ln, 1), q2 = Q(ln, 2), q3 = Q(ln, 3);
        if (de2) {
            const int t2 = 2 * tc;
            o[-1 * step] = (uint8_t)sk_clip((p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3, p0 - t2, p0 + t2);
            o[-2 * step] = (uint8_t)sk_clip((p2 + p1 + p0 + q0 + 2) >> 2, p1 - t2, p1 + t2);
            o[-3 * step] = (uint8_t)sk_clip((2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3, p2 - t2, p2 + t2);
            o[0] = (uint8_t)sk_clip((p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3, q0 - t2, q0 + t2);
            o[step] = (uint8_t)sk_clip((p0 + q0 + q1 + q2 + 2) >> 2, q1 - t2, q1 + t2);
            o[2 * step] = (uint8_t)sk_clip((p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3, q2 - t2, q2 + t2);
        } else {
            int d = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
            if (sk_abs(d) >= tc * 10) continue;
            d = sk_clip(d, -tc, tc);
            o[-step] = (uint8_t)sk_clip255(p0 + d);
            o[0] = (uint8_t)sk_clip255(q0 - d);
            if (dep) o[-2 * step] = (uint8_t)sk_clip255(p1 + sk_clip((((p2 + p0 + 1) >> 1) - p1 + d) >> 1, -(tc >> 1), tc >> 1));
            if (deq) o[step] = (uint8_t)sk_clip255(q1 + sk_clip((((q2 + q0 + 1) >> 1) - q1 - d) >> 1, -(tc >> 1), tc >> 1));
        }
    }
}

// One chroma line across an edge with bS 2 (8.7.2.5.5); qp: the luma QP average.
SK_HD void dbk_chroma_line(uint8_t* q, int step, int qp) {
    const int tc = HEVC_TC[sk_clip(chroma_qp(sk_clip(qp, 0, 57)) + 2, 0, 53)];
    const int p0 = q[-step], p1 = q[-2 * step], q0 = q[0], q1 = q[step];
    const int d = sk_clip((((q0 - p0) * 4) + p1 - q1 + 4) >> 3, -tc, tc);
    q[-step] = (uint8_t)sk_clip255(p0 + d);
    q[0] = (uint8_t)sk_clip255(q0 - d);
}

// The whole picture (CPU reference; k_hevc_dbk_v / k_hevc_dbk_h are the same loops in
// parallel). cus: [H16][W16] units; m: the slice layout (edges between slices stay).
// One luma segment: the vertical (vert) or horizontal edge at luma position e (a
// multiple of 8, > 0) of the picture, 4 samples long from position a along the edge.
// Returns without filtering when the edge is no transform / prediction edge or bS is 0.
SK_HD void dbk_luma_edge(uint8_t* Y, int sy, const CuInfo* cus, int W16, bool vert, int e, int a) {
    const int x = vert ? e : a, y = vert ? a : e;
    const CuInfo& q = cus[(y >> 4) * W16 + (x >> 4)];
    const CuInfo& p = vert ? cus[(y >> 4) * W16 + ((x - 1) >> 4)] : cus[((y - 1) >> 4) * W16 + (x >> 4)];
    if ((e & 8) && !(q.tu & 16)) return;   // no transform edge inside an unsplit unit
    int bs;
    if ((e & 31) == 16 && (q.c32 & kC32) && (p.c32 & kC32)) {   // inside one CU32
        if (q.c32 & kC32Tu) {   // one 32x32 TU: only the PU edge, motion only
            if (c32_part(q) != (vert ? PART_Nx2N : PART_2NxN)) return;
            bs = dbk_bs(p, q, 0, 0);
        } else {
            const int pc = vert ? tu_cbf_y(p, (x - 1) & 15, y & 15) : tu_cbf_y(p, x & 15, (y - 1) & 15);
            bs = dbk_bs(p, q, pc, tu_cbf_y(q, x & 15, y & 15));
        }
    } else {
        const int pc = vert ? tu_cbf_y(p, (x - 1) & 15, y & 15) : tu_cbf_y(p, x & 15, (y - 1) & 15);
        bs = dbk_bs(p, q, pc, tu_cbf_y(q, x & 15, y & 15));
    }
    if (bs) dbk_luma_segment(Y + (size_t)y * sy + x, vert ? 1 : sy, vert ? sy : 1, bs, (p.qp + q.qp + 1) >> 1);
}
SK_HD void deblock_picture(uint8_t* Y, uint8_t* U, uint8_t* V, int sy, int sc, const CuInfo* cus, int W16, int H16,
                           const SliceMap& m) {
    for (int x = 8; x < 16 * W16; x += 8)   // vertical edges (not between slices)
        for (int a = 0; a < 16 * H16; a += 4) {
            if (!(x & 8) && !m.same_u((x >> 4) - 1, a >> 4, x >> 4, a >> 4)) continue;
            dbk_luma_edge(Y, sy, cus, W16, true, x, a);
        }
    for (int cy = 0; cy < H16; cy++)
        for (int cx = 1; cx < W16; cx++) {
            const CuInfo &p = cus[cy * W16 + cx - 1], &q = cus[cy * W16 + cx];
            if (p.mode != CU_INTRA && q.mode != CU_INTRA) continue;   // chroma: bS 2 only
            if (!m.same_u(cx - 1, cy, cx, cy)) continue;
            const int qp = (p.qp + q.qp + 1) >> 1;
            for (int l = 0; l < 8; l++) {
                dbk_chroma_line(U + (size_t)(cy * 8 + l) * sc + cx * 8, 1, qp);
                dbk_chroma_line(V + (size_t)(cy * 8 + l) * sc + cx * 8, 1, qp);
            }
        }
    for (int y = 8; y < 16 * H16; y += 8)   // horizontal edges (not between slices)
        for (int a = 0; a < 16 * W16; a += 4) {
            if (!(y & 8) && !m.same_u(a >> 4, (y >> 4) - 1, a >> 4, y >> 4)) continue;
            dbk_luma_edge(Y, sy, cus, W16, false, y, a);
        }
    for (int cy = 1; cy < H16; cy++)
        for (int cx = 0; cx < W16; cx++) {
            const CuInfo &p = cus[(cy - 1) * W16 + cx], &q = cus[cy * W16 + cx];
            if (p.mode != CU_INTRA && q.mode != CU_INTRA) continue;
            if (!m.same_u(cx, cy - 1, cx, cy)) continue;
            const int qp = (p.qp + q.qp + 1) >> 1;
            for (int l = 0; l < 8; l++) {
                dbk_chroma_line(U + (size_t)(cy * 8) * sc + cx * 8 + l, sc, qp);
                dbk_chroma_line(V + (size_t)(cy * 8) * sc + cx * 8 + l, sc, qp);
            }
        }
}

}  // namespace hevc
}  // namespace sk
