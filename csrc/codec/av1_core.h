// AV1 (Main profile, 8-bit 4:2:0) primitives shared by the CPU reference encoder
// (av1_cpu.cpp) and the gfx950 kernels (kernels/av1_kernels.hip): block geometry,
// transforms and (de)quantisation, intra prediction, sub-pel motion compensation,
// the reference-MV stack and the syntax of blocks and coefficients written through
// a symbol sink (direct arithmetic coding on the host, token lists on the GPU).
//
// Decoder-side processes (inverse transform, dequantisation, prediction, MV stack,
// context selection) follow the normative processes of the AV1 bitstream spec
// (v1.0.0 + errata) §5.11 / §7.10-7.13 / §8.3; forward transform, quantisation and
// every mode decision are encoder choices. Conformance is checked by decoding the
// streams with dav1d (tests/test_av1_encoder.py) and comparing with the encoder's
// own reconstruction bit for bit.
//
// Coding structure (fixed by the sequence / frame headers of av1_cpu.cpp):
//   64x64 superblocks; blocks are square 8/16/32/64 (PARTITION_NONE or SPLIT only);
//   TX_MODE_LARGEST (one transform per block, reduced_tx_set: DCT_DCT or IDTX, the
//   screen-content identity transform, chosen per luma block); intra DC / V / H /
//   SMOOTH(_V/_H) / PAETH / directional, luma palettes of 2..8 colours on key frames
//   (code_palette_mode_info / code_palette_tokens), no filter-intra / CfL / chroma
//   palette / intraBC, intra edge filter off; one reference (LAST), single prediction, EIGHTTAP
//   regular filter, quarter-pel vectors (allow_high_precision_mv = 0); no order
//   hints (no temporal MVs, no skip mode); in-loop deblocking (av1_lf.h) and CDEF
//   (av1_cdef.h) on, loop restoration off.
#pragma once
#include "sk_common.h"
#include "av1_tables.h"
#include "av1_ec.h"

namespace sk::av1 {

// ---------------------------------------------------------------------------------
// Enumerations (spec values).
enum PredMode : uint8_t {
    DC_PRED = 0, V_PRED, H_PRED, D45_PRED, D135_PRED, D113_PRED, D157_PRED, D203_PRED, D67_PRED,
    SMOOTH_PRED, SMOOTH_V_PRED, SMOOTH_H_PRED, PAETH_PRED, UV_CFL_PRED,
    NEARESTMV = 13, NEARMV = 14, GLOBALMV = 15, NEWMV = 16
};
enum Partition : int { PARTITION_NONE = 0, PARTITION_HORZ = 1, PARTITION_VERT = 2, PARTITION_SPLIT = 3,
                       PARTITION_HORZ_A = 4, PARTITION_HORZ_B = 5, PARTITION_VERT_A = 6, PARTITION_VERT_B = 7,
                       PARTITION_HORZ_4 = 8, PARTITION_VERT_4 = 9 };
enum TxSize : int { TX_4X4 = 0, TX_8X8 = 1, TX_16X16 = 2, TX_32X32 = 3, TX_64X64 = 4 };
enum MvJoint : int { MV_JOINT_ZERO = 0, MV_JOINT_HNZVZ = 1, MV_JOINT_HZVNZ = 2, MV_JOINT_HNZVNZ = 3 };

constexpr int kRefCatLevel = 640;
constexpr int kMaxRefMvStack = 8;
constexpr int kMvBorder = 128;            // MV_BORDER, 1/8 pel
constexpr int kIntraFrame = 0, kLastFrame = 1;

// Block sizes are square: bsl = log2(width in 4x4 units) = Mi_Width_Log2: 8x8 -> 1 ... 64x64 -> 4.
SK_HD int bsl_px(int bsl) { return 4 << bsl; }

// Intra_Mode_Context (kf y-mode contexts)
SK_HD int intra_mode_ctx(int m) { return (int)((0x0123444430120ull >> (4 * (12 - m))) & 15); }

// ---------------------------------------------------------------------------------
// Geometry of one frame and its tiles (uniform tile spacing, §5.9.15).
struct Av1Geo {
    int W = 0, H = 0;            // frame size
    int mi_cols = 0, mi_rows = 0;
    int sb_cols = 0, sb_rows = 0;
    int tile_cols_log2 = 0, tile_rows_log2 = 0;
    int tile_cols = 0, tile_rows = 0;
    int tile_w_sb = 0, tile_h_sb = 0;
    int min_log2_tile_cols = 0, max_log2_tile_cols = 0, max_log2_tile_rows = 0, min_log2_tiles = 0;
    int c8 = 0, r8 = 0;          // 8x8 cell grid (mi_cols / 2, mi_rows / 2)
};

SK_HD int tile_log2(int blk, int target) {
    int k = 0;
    while ((blk << k) < target) k++;
    return k;
}

// Automatic tile split (log2 columns / rows) of a frame of sbc x sbr superblocks: up to
// 8 x 8 tiles; from 48 superblock columns (3072 px: 4K, 8K) 16 columns x 4 rows, the
// level-5.1 limits (MaxTileCols 16, MaxTiles 64). A key frame's tile is one workgroup of
// 16 waves stepping along anti-diagonals of 16x16 units (k_av1_intra_rec): 4K tiles of
// 16 x 36 units never hold more units on a diagonal than there are waves, where 8 x 7 tiles
// of 32 x 20 units needed a second round on 19 of their 51 steps.
SK_HD void auto_tiles(int sbc, int sbr, int* cols_log2, int* rows_log2) {
    if (sbc >= 48) {
        *cols_log2 = 4;
        *rows_log2 = tile_log2(1, sk_min(4, sbr));
        return;
    }
    *cols_log2 = tile_log2(1, sk_min(8, sbc));
    *rows_log2 = tile_log2(1, sk_min(8, sbr));
}

// want_cols_log2 / want_rows_log2: requested split, clamped to the legal range.
SK_HD void geo_init(Av1Geo& g, int W, int H, int want_cols_log2, int want_rows_log2) {
    g.W = W;
    g.H = H;
    g.mi_cols = 2 * ((W + 7) >> 3);
    g.mi_rows = 2 * ((H + 7) >> 3);
    g.c8 = g.mi_cols >> 1;
    g.r8 = g.mi_rows >> 1;
    g.sb_cols = (g.mi_cols + 15) >> 4;
    g.sb_rows = (g.mi_rows + 15) >> 4;
    const int max_tile_w_sb = 4096 >> 6, max_tile_area_sb = (4096 * 2304) >> 12;
    g.min_log2_tile_cols = tile_log2(max_tile_w_sb, g.sb_cols);
    g.max_log2_tile_cols = tile_log2(1, sk_min(g.sb_cols, 64));
    g.max_log2_tile_rows = tile_log2(1, sk_min(g.sb_rows, 64));
    g.min_log2_tiles = sk_max(g.min_log2_tile_cols, tile_log2(max_tile_area_sb, g.sb_rows * g.sb_cols));
    g.tile_cols_log2 = sk_clip(want_cols_log2, g.min_log2_tile_cols, g.max_log2_tile_cols);
    g.tile_w_sb = (g.sb_cols + (1 << g.tile_cols_log2) - 1) >> g.tile_cols_log2;
    g.tile_cols = (g.sb_cols + g.tile_w_sb - 1) / g.tile_w_sb;
    const int min_log2_rows = sk_max(g.min_log2_tiles - g.tile_cols_log2, 0);
    g.tile_rows_log2 = sk_clip(want_rows_log2, min_log2_rows, g.max_log2_tile_rows);
    g.tile_h_sb = (g.sb_rows + (1 << g.tile_rows_log2) - 1) >> g.tile_rows_log2;
    g.tile_rows = (g.sb_rows + g.tile_h_sb - 1) / g.tile_h_sb;
}

struct TileRect {
    int mi_row0, mi_row1, mi_col0, mi_col1;   // [start, end)
};
SK_HD TileRect tile_rect(const Av1Geo& g, int t) {
    const int tr = t / g.tile_cols, tc = t % g.tile_cols;
    TileRect r;
    r.mi_row0 = tr * g.tile_h_sb * 16;
    r.mi_row1 = sk_min((tr + 1) * g.tile_h_sb * 16, g.mi_rows);
    r.mi_col0 = tc * g.tile_w_sb * 16;
    r.mi_col1 = sk_min((tc + 1) * g.tile_w_sb * 16, g.mi_cols);
    return r;
}
SK_HD bool inside(const TileRect& t, int r, int c) {
    return r >= t.mi_row0 && r < t.mi_row1 && c >= t.mi_col0 && c < t.mi_col1;
}

// ---------------------------------------------------------------------------------
// Per-8x8-cell block info (every block is >= 8x8 and 8-aligned, so an 8x8 cell
// grid holds the spec's per-mi arrays MiSizes / YModes / IsInters / RefFrames /
// Mvs / Skips at 2x2-mi resolution). 12 bytes, shared by CPU and GPU buffers.
struct BlkInfo {
    uint8_t bsl;       // block size (Mi_Width_Log2), 0 = not coded yet
    uint8_t mode;      // YMode (intra 0..12, inter NEARESTMV..NEWMV)
    uint8_t uv_mode;   // UVMode (intra)
    uint8_t flags;     // bit0 is_inter, bit1 skip, bit2 merged-static (encoder), bits 4-5 RefMvIdx
    int16_t mv_row, mv_col;   // 1/8 pel (LAST), even values (no high-precision MVs)
    int16_t tx_type;   // luma transform type: TX_DCT_DCT (0) or TX_IDTX (1); inter chroma follows it
    uint8_t pal_n;     // PaletteSizeY (0: no palette; colours in the frame's palette cells)
    uint8_t pad1;
};
static_assert(sizeof(BlkInfo) == 12, "BlkInfo layout");
SK_HD bool blk_inter(const BlkInfo& b) { return (b.flags & 1) != 0; }
SK_HD bool blk_skip(const BlkInfo& b) { return (b.flags & 2) != 0; }

// ---------------------------------------------------------------------------------
// Transforms. Forward: encoder choice, an integer DCT-II scaled to 8x the
// orthonormal transform (the coefficient domain of AV1's 4/8/16-point transforms,
// fwd_shift {2,0..-2,0}). Inverse: the normative butterflies (spec §7.13.2,
// cos_bit 12) with the 2-D row/column shifts of §7.13.3.
SK_HD int cospi12(int i) {   // round(4096 * cos(i * pi / 128)), i = 0..64
    constexpr uint16_t t[65] = {4096, 4095, 4091, 4085, 4076, 4065, 4052, 4036, 4017, 3996, 3973, 3948, 3920,
                                3889, 3857, 3822, 3784, 3745, 3703, 3659, 3612, 3564, 3513, 3461, 3406, 3349,
                                3290, 3229, 3166, 3102, 3035, 2967, 2896, 2824, 2751, 2675, 2598, 2520, 2440,
                                2359, 2276, 2191, 2106, 2019, 1931, 1842, 1751, 1660, 1567, 1474, 1380, 1285,
                                1189, 1092, 995,  897,  799,  700,  601,  501,  401,  301,  201,  101,  0};
    return t[i];
}
SK_HD int32_t hbtf(int w0, int32_t a, int w1, int32_t b) {
    return (int32_t)(((int64_t)w0 * a + (int64_t)w1 * b + 2048) >> 12);
}

SK_HD void idct4(int32_t* x) {
    const int32_t a0 = x[0], a1 = x[2], a2 = x[1], a3 = x[3];
    const int32_t b0 = hbtf(cospi12(32), a0, cospi12(32), a1);
    const int32_t b1 = hbtf(cospi12(32), a0, -cospi12(32), a1);
    const int32_t b2 = hbtf(cospi12(48), a2, -cospi12(16), a3);
    const int32_t b3 = hbtf(cospi12(16), a2, cospi12(48), a3);
    x[0] = b0 + b3;
    x[1] = b1 + b2;
    x[2] = b1 - b2;
    x[3] = b0 - b3;
}

SK_HD void idct8(int32_t* x) {
    int32_t a[8] = {x[0], x[4], x[2], x[6], x[1], x[5], x[3], x[7]};
    int32_t b[8];
    // stage 2
    b[0] = a[0]; b[1] = a[1]; b[2] = a[2]; b[3] = a[3];
    b[4] = hbtf(cospi12(56), a[4], -cospi12(8), a[7]);
    b[5] = hbtf(cospi12(24), a[5], -cospi12(40), a[6]);
    b[6] = hbtf(cospi12(40), a[5], cospi12(24), a[6]);
    b[7] = hbtf(cospi12(8), a[4], cospi12(56), a[7]);
    // stage 3
    a[0] = hbtf(cospi12(32), b[0], cospi12(32), b[1]);
    a[1] = hbtf(cospi12(32), b[0], -cospi12(32), b[1]);
    a[2] = hbtf(cospi12(48), b[2], -cospi12(16), b[3]);
    a[3] = hbtf(cospi12(16), b[2], cospi12(48), b[3]);
    a[4] = b[4] + b[5];
    a[5] = b[4] - b[5];
    a[6] = -b[6] + b[7];
    a[7] = b[6] + b[7];
    // stage 4
    b[0] = a[0] + a[3];
    b[1] = a[1] + a[2];
    b[2] = a[1] - a[2];
    b[3] = a[0] - a[3];
    b[4] = a[4];
    b[5] = hbtf(-cospi12(32), a[5], cospi12(32), a[6]);
    b[6] = hbtf(cospi12(32), a[5], cospi12(32), a[6]);
    b[7] = a[7];
    // stage 5
    for (int i = 0; i < 4; i++) {
        x[i] = b[i] + b[7 - i];
        x[7 - i] = b[i] - b[7 - i];
    }
}

SK_HD void idct16(int32_t* x) {
    int32_t a[16] = {x[0], x[8], x[4], x[12], x[2], x[10], x[6], x[14],
                     x[1], x[9], x[5], x[13], x[3], x[11], x[7], x[15]};
    int32_t b[16];
    // stage 2
    for (int i = 0; i < 8; i++) b[i] = a[i];
    b[8] = hbtf(cospi12(60), a[8], -cospi12(4), a[15]);
    b[9] = hbtf(cospi12(28), a[9], -cospi12(36), a[14]);
    b[10] = hbtf(cospi12(44), a[10], -cospi12(20), a[13]);
    b[11] = hbtf(cospi12(12), a[11], -cospi12(52), a[12]);
    b[12] = hbtf(cospi12(52), a[11], cospi12(12), a[12]);
    b[13] = hbtf(cospi12(20), a[10], cospi12(44), a[13]);
    b[14] = hbtf(cospi12(36), a[9], cospi12(28), a[14]);
    b[15] = hbtf(cospi12(4), a[8], cospi12(60), a[15]);
    // stage 3
    for (int i = 0; i < 4; i++) a[i] = b[i];
    a[4] = hbtf(cospi12(56), b[4], -cospi12(8), b[7]);
    a[5] = hbtf(cospi12(24), b[5], -cospi12(40), b[6]);
    a[6] = hbtf(cospi12(40), b[5], cospi12(24), b[6]);
    a[7] = hbtf(cospi12(8), b[4], cospi12(56), b[7]);
    a[8] = b[8] + b[9];
    a[9] = b[8] - b[9];
    a[10] = -b[10] + b[11];
    a[11] = b[10] + b[11];
    a[12] = b[12] + b[13];
    a[13] = b[12] - b[13];
    a[14] = -b[14] + b[15];
    a[15] = b[14] + b[15];
    // stage 4
    b[0] = hbtf(cospi12(32), a[0], cospi12(32), a[1]);
    b[1] = hbtf(cospi12(32), a[0], -cospi12(32), a[1]);
    b[2] = hbtf(cospi12(48), a[2], -cospi12(16), a[3]);
    b[3] = hbtf(cospi12(16), a[2], cospi12(48), a[3]);
    b[4] = a[4] + a[5];
    b[5] = a[4] - a[5];
    b[6] = -a[6] + a[7];
    b[7] = a[6] + a[7];
    b[8] = a[8];
    b[9] = hbtf(-cospi12(16), a[9], cospi12(48), a[14]);
    b[10] = hbtf(-cospi12(48), a[10], -cospi12(16), a[13]);
    b[11] = a[11];
    b[12] = a[12];
    b[13] = hbtf(-cospi12(16), a[10], cospi12(48), a[13]);
    b[14] = hbtf(cospi12(48), a[9], cospi12(16), a[14]);
    b[15] = a[15];
    // stage 5
    a[0] = b[0] + b[3];
    a[1] = b[1] + b[2];
    a[2] = b[1] - b[2];
    a[3] = b[0] - b[3];
    a[4] = b[4];
    a[5] = hbtf(-cospi12(32), b[5], cospi12(32), b[6]);
    a[6] = hbtf(cospi12(32), b[5], cospi12(32), b[6]);
    a[7] = b[7];
    a[8] = b[8] + b[11];
    a[9] = b[9] + b[10];
    a[10] = b[9] - b[10];
    a[11] = b[8] - b[11];
    a[12] = -b[12] + b[15];
    a[13] = -b[13] + b[14];
    a[14] = b[13] + b[14];
    a[15] = b[12] + b[15];
    // stage 6
    for (int i = 0; i < 4; i++) {
        b[i] = a[i] + a[7 - i];
        b[7 - i] = a[i] - a[7 - i];
    }
    b[8] = a[8];
    b[9] = a[9];
    b[10] = hbtf(-cospi12(32), a[10], cospi12(32), a[13]);
    b[11] = hbtf(-cospi12(32), a[11], cospi12(32), a[12]);
    b[12] = hbtf(cospi12(32), a[11], cospi12(32), a[12]);
    b[13] = hbtf(cospi12(32), a[10], cospi12(32), a[13]);
    b[14] = a[14];
    b[15] = a[15];
    // stage 7
    for (int i = 0; i < 8; i++) {
        x[i] = b[i] + b[15 - i];
        x[15 - i] = b[i] - b[15 - i];
    }
}

SK_HD void idct_1d(int32_t* x, int log2n) {
    if (log2n == 2) idct4(x);
    else if (log2n == 3) idct8(x);
    else idct16(x);
}

// Identity transform (IDTX, the screen-content transform): inverse of spec 7.13.2.15
// for n = 4 / 8 / 16; the forward identity is 8 x the residual (the coefficient domain
// of the DCT path: 8 x orthonormal, so one quantiser serves both).
SK_HD int32_t iidentity(int32_t x, int log2n) {
    if (log2n == 2) return (int32_t)(((int64_t)x * 5793 + 2048) >> 12);
    if (log2n == 3) return x * 2;
    return (int32_t)(((int64_t)x * 11586 + 2048) >> 12);
}
enum TxType : int { TX_DCT_DCT = 0, TX_IDTX = 1 };

// 2-D inverse DCT_DCT (or IDTX) of an n x n block (n = 4, 8, 16): dequantised
// coefficients `d` (raster [row][col], row = vertical frequency) -> residual `r`.
SK_HD void inv_transform(const int32_t* d, int log2n, int32_t* r, bool idtx = false) {
    const int n = 1 << log2n;
    const int row_shift = log2n == 2 ? 0 : (log2n == 3 ? 1 : 2);
    int32_t t[16];
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < n; j++) t[j] = d[i * n + j];
        if (idtx)
            for (int j = 0; j < n; j++) t[j] = iidentity(t[j], log2n);
        else
            idct_1d(t, log2n);
        for (int j = 0; j < n; j++) {
            const int32_t v = row_shift ? (t[j] + (1 << (row_shift - 1))) >> row_shift : t[j];
            r[i * n + j] = sk_clip(v, -32768, 32767);   // colClampRange = 16 bits (8-bit video)
        }
    }
    for (int j = 0; j < n; j++) {
        for (int i = 0; i < n; i++) t[i] = r[i * n + j];
        if (idtx)
            for (int i = 0; i < n; i++) t[i] = iidentity(t[i], log2n);
        else
            idct_1d(t, log2n);
        for (int i = 0; i < n; i++) r[i * n + j] = (t[i] + 8) >> 4;
    }
}

// Orthonormal DCT-II basis in Q13: K[k][m] = round(8192 * sqrt(2/N) * c_k * cos(pi*(2m+1)*k / 2N)).
SK_HD int fdct_basis(int log2n, int k, int m) {
    const int n = 1 << log2n;
    // cos table at pi/64 resolution, Q14: cos(pi * i / 64), i = 0..64
    constexpr int16_t c64[65] = {16384, 16364, 16305, 16207, 16069, 15893, 15679, 15426, 15137, 14811, 14449,
                                 14053, 13623, 13160, 12665, 12140, 11585, 11003, 10394, 9760,  9102,  8423,
                                 7723,  7005,  6270,  5520,  4756,  3981,  3196,  2404,  1606,  804,   0,
                                 -804,  -1606, -2404, -3196, -3981, -4756, -5520, -6270, -7005, -7723, -8423,
                                 -9102, -9760, -10394, -11003, -11585, -12140, -12665, -13160, -13623, -14053,
                                 -14449, -14811, -15137, -15426, -15679, -15893, -16069, -16207, -16305, -16364,
                                 -16384};
    // angle = pi*(2m+1)*k / (2N) = pi * i / 64 with i = (2m+1)*k*(32/N); reduce modulo 128 (2 pi)
    int i = ((2 * m + 1) * k * (32 >> log2n)) & 127;
    int c = i <= 64 ? c64[i] : c64[128 - i];
    // scale: sqrt(2/N) * c_k; Q14 cos -> Q13 basis
    // sqrt(2/N): N=4 -> 0.70710678, N=8 -> 0.5, N=16 -> 0.35355339
    int64_t v = (int64_t)c * (log2n == 2 ? 11585 : (log2n == 3 ? 8192 : 5793));   // Q14
    if (k == 0) v = v * 11585 >> 14;   // c_0 = 1/sqrt(2)
    (void)n;
    return (int)((v + (1 << 14)) >> 15);   // Q14 * Q14 -> Q13
}

// Forward DCT_DCT: residual `x` (n x n raster) -> coefficients in AV1's domain
// (8 x orthonormal), raster [row][col] with row = vertical frequency.
SK_HD void fwd_transform(const int32_t* x, int log2n, int32_t* c) {
    const int n = 1 << log2n;
    int32_t t[256];
    // columns: t[k][j] = sum_m K[k][m] x[m][j], kept at 8x (Q13 -> >> 10)
    for (int k = 0; k < n; k++)
        for (int j = 0; j < n; j++) {
            int64_t s = 0;
            for (int m = 0; m < n; m++) s += (int64_t)fdct_basis(log2n, k, m) * x[m * n + j];
            t[k * n + j] = (int32_t)((s + 512) >> 10);
        }
    // rows: c[k][l] = sum_j t[k][j] K[l][j], Q13 -> >> 13
    for (int k = 0; k < n; k++)
        for (int l = 0; l < n; l++) {
            int64_t s = 0;
            for (int j = 0; j < n; j++) s += (int64_t)t[k * n + j] * fdct_basis(log2n, l, j);
            c[k * n + l] = (int32_t)((s + (s >= 0 ? 4096 : 4095)) >> 13);
        }
}

// ---------------------------------------------------------------------------------
// Quantisation. AV1 dequantisation (§7.12.3) for 8-bit, no quantiser matrices,
// dqDenom 0 (transforms up to 16x16).
SK_HD int dc_q(int qidx) { return AV1_DC_QLOOKUP[sk_clip(qidx, 0, 255)]; }
SK_HD int ac_q(int qidx) { return AV1_AC_QLOOKUP[sk_clip(qidx, 0, 255)]; }
SK_HD int32_t dequant(int level, int q) {
    const int a = level < 0 ? -level : level;
    int32_t dq = (int32_t)(((int64_t)a * q) & 0xFFFFFF);
    dq = level < 0 ? -dq : dq;
    return sk_clip(dq, -(1 << 15), (1 << 15) - 1);
}
// Encoder quantiser: dead-zone rounding (intra 1/3, inter 1/6 of a step), level capped.
SK_HD int quantize(int32_t c, int q, bool intra) {
    const int a = c < 0 ? -c : c;
    // |c| < 2^17 and q <= 1828: the numerator stays far below 2^32 (32-bit division; the
    // 64-bit one is a long software sequence on the GPU)
    const int l = (int)(((uint32_t)a * 6u + (uint32_t)((intra ? 2 : 1) * q)) / (6u * (uint32_t)q));
    const int lc = l > 4095 ? 4095 : l;
    return c < 0 ? -lc : lc;
}
// Transform-type decision (encoder choice): J = 256 x (SSE + lambda x bits) for the
// levels of one transform type, lambda = 0.136 x (ac_q / 8)^2 (x264's SSE lambda at the
// same quantiser step). dist4 = 4 x sum of squared coefficient errors (the coefficient
// domain is 8 x orthonormal: pixel SSE = coefficient SSE / 64); rate2 in half bits from
// tx_bits2 over the scan up to the end of block plus tx_eob_bits2.
SK_HD int tx_bits2(int level) {
    const int a = level < 0 ? -level : level;
    if (a == 0) return 1;
    if (a == 1) return 6;
    return 8 + 4 * (31 - __builtin_clz((unsigned)a));
}
SK_HD int tx_eob_bits2(int eob) { return eob ? 2 * (32 - __builtin_clz((unsigned)eob)) + 2 : 0; }
SK_HD long long tx_rd_cost(long long dist4, int rate2, int qa) {
    return dist4 + (((long long)qa * qa * rate2 * 70) >> 8);
}

// qindex -> coefficient CDF context (§7.20: <= 20, <= 60, <= 120, else)
SK_HD int coef_qctx(int qidx) { return qidx <= 20 ? 0 : (qidx <= 60 ? 1 : (qidx <= 120 ? 2 : 3)); }
// Frame qindex of a rate-controlled frame at fractional QP qpf (Q8, ratecontrol.h):
// AV1 has ~5 qindex steps per H.264 QP at the top of its range, so the fraction is
// realised in the frame's qindex (tab: qindex of each integer QP 0..51).
SK_HD int frame_qidx(const uint8_t* tab, int qpf) {
    const int lo = sk_clip(qpf >> 8, 0, 51), f = qpf & 255;
    if (lo >= 51) return tab[51];
    return tab[lo] + (((int)tab[lo + 1] - (int)tab[lo]) * f + 128) / 256;
}

// ---------------------------------------------------------------------------------
// Scans: the default (zig-zag) scan of an n x n DCT_DCT block, scan index -> raster position.
// kScanTransposed selects the orientation of the zig-zag (spec Default_Scan_NxN walk:
// odd anti-diagonals run down-left, even ones up-right, in raster [row][col]).
constexpr int kScanTransposed = 0;
// 4x4 | 8x8 | 16x16 scans, generated from the walk below (kept as the definition):
//   n = 1 << log2n; anti-diagonal d of length d < n ? d + 1 : 2n - 1 - d holding idx;
//   k = idx - (positions before d); row = (d & 1) ^ kScanTransposed ? row_first + k
//   : row_last - k (row_first = max(0, d - n + 1), row_last = min(d, n - 1)); pos = row * n + d - row.
// A table: the walk costs ~200 instructions per call on the GPU, where the token and
// residual kernels call it for every coefficient.
SK_TABLE uint8_t AV1_DEFAULT_SCAN[336] = {
    0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15, 0, 1, 8, 16, 9, 2, 3, 10,
    17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46,
    53, 60, 61, 54, 47, 55, 62, 63, 0, 1, 16, 32, 17, 2, 3, 18, 33, 48, 64, 49, 34, 19, 4, 5,
    20, 35, 50, 65, 80, 96, 81, 66, 51, 36, 21, 6, 7, 22, 37, 52, 67, 82, 97, 112, 128, 113, 98, 83,
    68, 53, 38, 23, 8, 9, 24, 39, 54, 69, 84, 99, 114, 129, 144, 160, 145, 130, 115, 100, 85, 70, 55, 40,
    25, 10, 11, 26, 41, 56, 71, 86, 101, 116, 131, 146, 161, 176, 192, 177, 162, 147, 132, 117, 102, 87, 72, 57,
    42, 27, 12, 13, 28, 43, 58, 73, 88, 103, 118, 133, 148, 163, 178, 193, 208, 224, 209, 194, 179, 164, 149, 134,
    119, 104, 89, 74, 59, 44, 29, 14, 15, 30, 45, 60, 75, 90, 105, 120, 135, 150, 165, 180, 195, 210, 225, 240,
    241, 226, 211, 196, 181, 166, 151, 136, 121, 106, 91, 76, 61, 46, 31, 47, 62, 77, 92, 107, 122, 137, 152, 167,
    182, 197, 212, 227, 242, 243, 228, 213, 198, 183, 168, 153, 138, 123, 108, 93, 78, 63, 79, 94, 109, 124, 139, 154,
    169, 184, 199, 214, 229, 244, 245, 230, 215, 200, 185, 170, 155, 140, 125, 110, 95, 111, 126, 141, 156, 171, 186, 201,
    216, 231, 246, 247, 232, 217, 202, 187, 172, 157, 142, 127, 143, 158, 173, 188, 203, 218, 233, 248, 249, 234, 219, 204,
    189, 174, 159, 175, 190, 205, 220, 235, 250, 251, 236, 221, 206, 191, 207, 222, 237, 252, 253, 238, 223, 239, 254, 255,
};
SK_HD int default_scan(int log2n, int idx) {
    return AV1_DEFAULT_SCAN[(log2n == 2 ? 0 : (log2n == 3 ? 16 : 80)) + idx];
}

// ---------------------------------------------------------------------------------
// Intra prediction (§7.11.2) for DC / V / H (angle delta 0) / SMOOTH* / PAETH.
// Edges: above[-1..n-1] and left[-1..n-1] per the spec's availability rules.
struct IntraEdge {
    uint8_t above[17];   // [0] = top-left, [1..n] = above row
    uint8_t left[17];    // [0] = top-left, [1..n] = left column
    bool have_above, have_left;
};

// plane: pointer to the reconstructed plane, (x, y) block origin, n block size,
// max_x / max_y: last addressable column / row of the plane (MiCols*4 >> ss) - 1.
SK_HD void intra_edges(const uint8_t* plane, int stride, int x, int y, int n, bool have_above, bool have_left,
                       int max_x, int max_y, IntraEdge& e) {
    e.have_above = have_above;
    e.have_left = have_left;
    for (int i = 0; i < n; i++) {
        if (!have_above && have_left) e.above[1 + i] = plane[(size_t)y * stride + x - 1];
        else if (!have_above) e.above[1 + i] = 127;
        else e.above[1 + i] = plane[(size_t)(y - 1) * stride + sk_min(max_x, x + i)];
        if (!have_left && have_above) e.left[1 + i] = plane[(size_t)(y - 1) * stride + x];
        else if (!have_left) e.left[1 + i] = 129;
        else e.left[1 + i] = plane[(size_t)sk_min(max_y, y + i) * stride + x - 1];
    }
    uint8_t tl;
    if (have_above && have_left) tl = plane[(size_t)(y - 1) * stride + x - 1];
    else if (have_above) tl = plane[(size_t)(y - 1) * stride + x];
    else if (have_left) tl = plane[(size_t)y * stride + x - 1];
    else tl = 128;
    e.above[0] = e.left[0] = tl;
}

SK_HD int intra_pred_px(const IntraEdge& e, int mode, int log2n, int i /*row*/, int j /*col*/) {
    const int n = 1 << log2n;
    const uint8_t* A = e.above + 1;
    const uint8_t* L = e.left + 1;
    switch (mode) {
        case V_PRED: return A[j];
        case H_PRED: return L[i];
        case SMOOTH_PRED: {
            const int wy = AV1_SM_WEIGHTS[n + i], wx = AV1_SM_WEIGHTS[n + j];
            const int s = wy * A[j] + (256 - wy) * L[n - 1] + wx * L[i] + (256 - wx) * A[n - 1];
            return (s + 256) >> 9;
        }
        case SMOOTH_V_PRED: {
            const int wy = AV1_SM_WEIGHTS[n + i];
            return (wy * A[j] + (256 - wy) * L[n - 1] + 128) >> 8;
        }
        case SMOOTH_H_PRED: {
            const int wx = AV1_SM_WEIGHTS[n + j];
            return (wx * L[i] + (256 - wx) * A[n - 1] + 128) >> 8;
        }
        case PAETH_PRED: {
            const int base = A[j] + L[i] - e.above[0];
            const int pl = sk_abs(base - L[i]), pt = sk_abs(base - A[j]), ptl = sk_abs(base - e.above[0]);
            if (pl <= pt && pl <= ptl) return L[i];
            if (pt <= ptl) return A[j];
            return e.above[0];
        }
        default: return -1;   // DC: see intra_dc
    }
}

SK_HD int intra_dc(const IntraEdge& e, int log2n) {
    const int n = 1 << log2n;
    int s = 0;
    if (e.have_above && e.have_left) {
        for (int k = 0; k < n; k++) s += e.above[1 + k] + e.left[1 + k];
        return (s + n) >> (log2n + 1);
    }
    if (e.have_above) {
        for (int k = 0; k < n; k++) s += e.above[1 + k];
        return (s + (n >> 1)) >> log2n;
    }
    if (e.have_left) {
        for (int k = 0; k < n; k++) s += e.left[1 + k];
        return (s + (n >> 1)) >> log2n;
    }
    return 128;
}

SK_HD void intra_predict(const IntraEdge& e, int mode, int log2n, uint8_t* pred) {
    const int n = 1 << log2n;
    if (mode == DC_PRED) {
        const int dc = intra_dc(e, log2n);
        for (int k = 0; k < n * n; k++) pred[k] = (uint8_t)dc;
        return;
    }
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) pred[i * n + j] = (uint8_t)intra_pred_px(e, mode, log2n, i, j);
}

SK_HD bool is_directional(int mode) { return mode >= V_PRED && mode <= D67_PRED; }

// ---------------------------------------------------------------------------------
// Inter prediction (§7.11.3.4, no scaling): EIGHTTAP regular, 4-tap variant for
// blocks 4 wide/high. mv in 1/8 luma pel (row, col); positions clamp to the
// reference frame's real size (last_x / last_y).
SK_HD int subpel_tap(int filt4, int frac, int t) {
    // Subpel_Filters[0] (regular 8-tap) and [4] (regular 4-tap), 1/16 positions
    constexpr int16_t f8[16][8] = {
        {0, 0, 0, 128, 0, 0, 0, 0},      {0, 2, -6, 126, 8, -2, 0, 0},    {0, 2, -10, 122, 18, -4, 0, 0},
        {0, 2, -12, 116, 28, -8, 2, 0},  {0, 2, -14, 110, 38, -10, 2, 0}, {0, 2, -14, 102, 48, -12, 2, 0},
        {0, 2, -16, 94, 58, -12, 2, 0},  {0, 2, -14, 84, 66, -12, 2, 0},  {0, 2, -14, 76, 76, -14, 2, 0},
        {0, 2, -12, 66, 84, -14, 2, 0},  {0, 2, -12, 58, 94, -16, 2, 0},  {0, 2, -12, 48, 102, -14, 2, 0},
        {0, 2, -10, 38, 110, -14, 2, 0}, {0, 2, -8, 28, 116, -12, 2, 0},  {0, 0, -4, 18, 122, -10, 2, 0},
        {0, 0, -2, 8, 126, -6, 2, 0}};
    constexpr int16_t f4[16][8] = {
        {0, 0, 0, 128, 0, 0, 0, 0},     {0, 0, -4, 126, 8, -2, 0, 0},   {0, 0, -8, 122, 18, -4, 0, 0},
        {0, 0, -10, 116, 28, -6, 0, 0}, {0, 0, -12, 110, 38, -8, 0, 0}, {0, 0, -12, 102, 48, -10, 0, 0},
        {0, 0, -14, 94, 58, -10, 0, 0}, {0, 0, -12, 84, 66, -10, 0, 0}, {0, 0, -12, 76, 76, -12, 0, 0},
        {0, 0, -10, 66, 84, -12, 0, 0}, {0, 0, -10, 58, 94, -14, 0, 0}, {0, 0, -10, 48, 102, -12, 0, 0},
        {0, 0, -8, 38, 110, -12, 0, 0}, {0, 0, -6, 28, 116, -10, 0, 0}, {0, 0, -4, 18, 122, -8, 0, 0},
        {0, 0, -2, 8, 126, -4, 0, 0}};
    return filt4 ? f4[frac][t] : f8[frac][t];
}

// One w x h block of one plane. (x, y): block position in the plane; ss: chroma
// subsampling shift (0 luma, 1 chroma); ref: reference plane.
SK_HD void mc_block(const uint8_t* ref, int stride, int last_x, int last_y, int x, int y, int w, int h, int ss,
                    int mv_row, int mv_col, uint8_t* pred, int pstride) {
    // positions in 1/16 sample units of this plane
    const int px16 = (x << 4) + ((2 * mv_col) >> ss);
    const int py16 = (y << 4) + ((2 * mv_row) >> ss);
    const int fx = px16 & 15, fy = py16 & 15;
    const int ix = px16 >> 4, iy = py16 >> 4;
    const int fh = w <= 4, fv = h <= 4;
    if (fx == 0 && fy == 0) {   // exact copy (the filter at position 0 is the identity)
        for (int r = 0; r < h; r++)
            for (int c = 0; c < w; c++)
                pred[r * pstride + c] = ref[(size_t)sk_clip(iy + r, 0, last_y) * stride + sk_clip(ix + c, 0, last_x)];
        return;
    }
    int16_t im[(64 + 7) * 64];
    const int ih = h + 7;
    for (int r = 0; r < ih; r++) {
        const uint8_t* row = ref + (size_t)sk_clip(iy + r - 3, 0, last_y) * stride;
        for (int c = 0; c < w; c++) {
            int s = 0;
            for (int t = 0; t < 8; t++) s += subpel_tap(fh, fx, t) * row[sk_clip(ix + c + t - 3, 0, last_x)];
            im[r * w + c] = (int16_t)((s + 4) >> 3);   // InterRound0 = 3
        }
    }
    for (int r = 0; r < h; r++)
        for (int c = 0; c < w; c++) {
            int s = 0;
            for (int t = 0; t < 8; t++) s += subpel_tap(fv, fy, t) * im[(r + t) * w + c];
            pred[r * pstride + c] = (uint8_t)sk_clip255((s + 1024) >> 11);   // InterRound1 = 11
        }
}

// ---------------------------------------------------------------------------------
// Reference-MV stack (§7.10.2, single reference LAST, no temporal candidates,
// identity global motion). The neighbour view is a function over mi positions.
struct MvStack {
    int n;                      // NumMvFound
    int new_count;              // NewMvCount
    int16_t mv[kMaxRefMvStack][2];   // RefStackMv[..][0] (row, col), clamped
    int weight[kMaxRefMvStack];
    int close_matches, total_matches;
    int newmv_ctx, refmv_ctx;   // NewMvContext, RefMvContext (ZeroMvContext = 0)
};

// Grid: BlkInfo per 8x8 cell, row stride c8.
struct BlkGrid {
    const BlkInfo* b;
    int c8;
    SK_HD const BlkInfo& at(int mi_r, int mi_c) const { return b[(mi_r >> 1) * c8 + (mi_c >> 1)]; }
};

namespace detail {
SK_HD void search_stack(MvStack& s, const BlkInfo& nb, int weight, bool& found) {
    int16_t mv[2] = {nb.mv_row, nb.mv_col};
    for (int i = 0; i < 2; i++)
        if (mv[i] & 1) mv[i] += mv[i] > 0 ? -1 : 1;   // lower_mv_precision (no high precision)
    if (nb.mode == NEWMV) s.new_count++;
    found = true;
    int idx = 0;
    for (; idx < s.n; idx++)
        if (s.mv[idx][0] == mv[0] && s.mv[idx][1] == mv[1]) break;
    if (idx < s.n) {
        s.weight[idx] += weight;
    } else if (s.n < kMaxRefMvStack) {
        s.mv[s.n][0] = mv[0];
        s.mv[s.n][1] = mv[1];
        s.weight[s.n] = weight;
        s.n++;
    }
}
SK_HD void add_candidate(MvStack& s, const BlkInfo& nb, int weight, bool& found) {
    if (!blk_inter(nb)) return;
    search_stack(s, nb, weight, found);   // RefFrames[..][0] == LAST for every inter block
}
SK_HD void scan_row(MvStack& s, const BlkGrid& g, const TileRect& t, int mi_rows, int mi_cols, int r, int c,
                    int bw4, int delta_row, bool& found) {
    int end4 = sk_min(sk_min(bw4, mi_cols - c), 16);
    int delta_col = 0;
    const bool step16 = bw4 >= 16;
    if (sk_abs(delta_row) > 1) {
        delta_row += r & 1;
        delta_col = 1 - (c & 1);
    }
    int i = 0;
    while (i < end4) {
        const int mr = r + delta_row, mc = c + delta_col + i;
        if (!inside(t, mr, mc)) break;
        const BlkInfo& nb = g.at(mr, mc);
        int len = sk_min(bw4, 1 << nb.bsl);
        if (sk_abs(delta_row) > 1) len = sk_max(2, len);
        if (step16) len = sk_max(4, len);
        add_candidate(s, nb, len * 2, found);
        i += len;
    }
    (void)mi_rows;
}
SK_HD void scan_col(MvStack& s, const BlkGrid& g, const TileRect& t, int mi_rows, int mi_cols, int r, int c,
                    int bh4, int delta_col, bool& found) {
    int end4 = sk_min(sk_min(bh4, mi_rows - r), 16);
    int delta_row = 0;
    const bool step16 = bh4 >= 16;
    if (sk_abs(delta_col) > 1) {
        delta_row = 1 - (r & 1);
        delta_col += c & 1;
    }
    int i = 0;
    while (i < end4) {
        const int mr = r + delta_row + i, mc = c + delta_col;
        if (!inside(t, mr, mc)) break;
        const BlkInfo& nb = g.at(mr, mc);
        int len = sk_min(bh4, 1 << nb.bsl);
        if (sk_abs(delta_col) > 1) len = sk_max(2, len);
        if (step16) len = sk_max(4, len);
        add_candidate(s, nb, len * 2, found);
        i += len;
    }
    (void)mi_cols;
}
}  // namespace detail

// `decoded(mr, mc)`: whether the block covering mi (mr, mc) precedes the current
// block in coding order (top-right candidate availability).
template <class Decoded>
SK_HD void find_mv_stack(MvStack& s, const BlkGrid& g, const TileRect& t, int mi_rows, int mi_cols, int r, int c,
                         int bsl, const Decoded& decoded) {
    using namespace detail;
    const int bw4 = 1 << bsl, bh4 = bw4;
    s.n = 0;
    s.new_count = 0;
    bool found = false;
    scan_row(s, g, t, mi_rows, mi_cols, r, c, bw4, -1, found);
    bool found_above = found;
    found = false;
    scan_col(s, g, t, mi_rows, mi_cols, r, c, bh4, -1, found);
    bool found_left = found;
    found = false;
    if (sk_max(bw4, bh4) <= 16) {   // top-right
        const int mr = r - 1, mc = c + bw4;
        if (inside(t, mr, mc) && decoded(mr, mc)) add_candidate(s, g.at(mr, mc), 4, found);
    }
    if (found) found_above = true;
    s.close_matches = (int)found_above + (int)found_left;
    const int num_nearest = s.n, num_new = s.new_count;
    for (int i = 0; i < num_nearest; i++) s.weight[i] += kRefCatLevel;
    found = false;
    {   // top-left
        const int mr = r - 1, mc = c - 1;
        if (inside(t, mr, mc) && decoded(mr, mc)) add_candidate(s, g.at(mr, mc), 4, found);
    }
    if (found) found_above = true;
    found = false;
    scan_row(s, g, t, mi_rows, mi_cols, r, c, bw4, -3, found);
    if (found) found_above = true;
    found = false;
    scan_col(s, g, t, mi_rows, mi_cols, r, c, bh4, -3, found);
    if (found) found_left = true;
    found = false;
    if (bh4 > 1) scan_row(s, g, t, mi_rows, mi_cols, r, c, bw4, -5, found);
    if (found) found_above = true;
    found = false;
    if (bw4 > 1) scan_col(s, g, t, mi_rows, mi_cols, r, c, bh4, -5, found);
    if (found) found_left = true;
    s.total_matches = (int)found_above + (int)found_left;
    // sorting (bubble, stable for equal weights) of [0, nearest) and [nearest, n)
    for (int pass = 0; pass < 2; pass++) {
        const int start = pass == 0 ? 0 : num_nearest;
        int end = pass == 0 ? num_nearest : s.n;
        while (end > start) {
            int new_end = start;
            for (int idx = start + 1; idx < end; idx++)
                if (s.weight[idx - 1] < s.weight[idx]) {
                    const int w = s.weight[idx - 1];
                    s.weight[idx - 1] = s.weight[idx];
                    s.weight[idx] = w;
                    for (int k = 0; k < 2; k++) {
                        const int16_t m = s.mv[idx - 1][k];
                        s.mv[idx - 1][k] = s.mv[idx][k];
                        s.mv[idx][k] = m;
                    }
                    new_end = idx;
                }
            end = new_end;
        }
    }
    if (s.n < 2) {   // extra search
        const int w4 = sk_min(sk_min(16, bw4), mi_cols - c), h4 = sk_min(sk_min(16, bh4), mi_rows - r);
        const int num4x4 = sk_min(w4, h4);
        for (int pass = 0; pass < 2 && s.n < 2; pass++) {
            int idx = 0;
            while (idx < num4x4 && s.n < 2) {
                const int mr = pass == 0 ? r - 1 : r + idx, mc = pass == 0 ? c + idx : c - 1;
                if (!inside(t, mr, mc)) break;
                const BlkInfo& nb = g.at(mr, mc);
                if (blk_inter(nb)) {   // add_extra_mv_candidate: same sign bias (single LAST)
                    const int16_t mv0 = nb.mv_row, mv1 = nb.mv_col;
                    int k = 0;
                    for (; k < s.n; k++)
                        if (s.mv[k][0] == mv0 && s.mv[k][1] == mv1) break;
                    if (k == s.n) {
                        s.mv[k][0] = mv0;
                        s.mv[k][1] = mv1;
                        s.weight[k] = 2;
                        s.n++;
                    }
                }
                idx += 1 << nb.bsl;
            }
        }
        for (int k = s.n; k < 2; k++) {   // GlobalMvs[0] = 0
            s.mv[k][0] = s.mv[k][1] = 0;
            s.weight[k] = 0;
        }
    }
    // context and clamping
    const int top = -((r * 4) * 8), bottom = ((mi_rows - bh4 - r) * 4) * 8;
    const int left = -((c * 4) * 8), right = ((mi_cols - bw4 - c) * 4) * 8;
    for (int i = 0; i < s.n; i++) {
        s.mv[i][0] = (int16_t)sk_clip(s.mv[i][0], top - (kMvBorder + bh4 * 32), bottom + kMvBorder + bh4 * 32);
        s.mv[i][1] = (int16_t)sk_clip(s.mv[i][1], left - (kMvBorder + bw4 * 32), right + kMvBorder + bw4 * 32);
    }
    if (s.close_matches == 0) {
        s.newmv_ctx = sk_min(s.total_matches, 1);
        s.refmv_ctx = s.total_matches;
    } else if (s.close_matches == 1) {
        s.newmv_ctx = 3 - sk_min(num_new, 1);
        s.refmv_ctx = 2 + s.total_matches;
    } else {
        s.newmv_ctx = 5 - sk_min(num_new, 1);
        s.refmv_ctx = 5;
    }
}

SK_HD int drl_ctx(const MvStack& s, int idx) {
    if (s.weight[idx] >= kRefCatLevel && s.weight[idx + 1] >= kRefCatLevel) return 0;
    if (s.weight[idx] >= kRefCatLevel && s.weight[idx + 1] < kRefCatLevel) return 1;
    if (s.weight[idx] < kRefCatLevel && s.weight[idx + 1] < kRefCatLevel) return 2;
    return 0;
}

// ---------------------------------------------------------------------------------
// Symbol sinks. A sink offers sym(cdf offset in CdfContext u16 units, N, value),
// bit(b) (an L(1) equiprobable bit) and lits(value, nbits).
SK_HD int cdf_off(const CdfContext& base, const uint16_t* p) { return (int)(p - (const uint16_t*)&base); }

// split_or_horz / split_or_vert: a binary CDF gathered from the (adapted) partition
// CDF of the node (spec §9.3.x psum, libaom partition_gather_{vert,horz}_alike).
// bottom_out: the bottom half lies outside the frame (SPLIT vs HORZ), else the right half.
SK_HD void gather_partition_cdf(const uint16_t* pc, bool bottom_out, uint16_t* out) {
    auto P = [&](int k) { return (int)pc[k] - (k > 0 ? (int)pc[k - 1] : 0); };
    int psum;
    if (bottom_out)
        psum = P(PARTITION_VERT) + P(PARTITION_SPLIT) + P(PARTITION_HORZ_A) + P(PARTITION_VERT_A) + P(PARTITION_VERT_B) +
               P(PARTITION_VERT_4);
    else
        psum = P(PARTITION_HORZ) + P(PARTITION_SPLIT) + P(PARTITION_HORZ_A) + P(PARTITION_HORZ_B) + P(PARTITION_VERT_A) +
               P(PARTITION_HORZ_4);
    out[0] = (uint16_t)(32768 - psum);
    out[1] = 32768;
    out[2] = 0;
}

// Direct coding: adaptive CDFs in `ctx`, coded by a SymbolCoder.
template <class Coder>
struct DirectSink {
    Coder& coder;
    CdfContext& ctx;
    SK_HD void sym(int off, int n, int v) { coder.encode_adapt((uint16_t*)&ctx + off, n, v); }
    SK_HD void bit(int b) { coder.bool_(b); }
    SK_HD void lits(uint32_t v, int nbits) { coder.literal(v, nbits); }
    SK_HD void gather(int off, bool bottom_out, int v) {
        uint16_t c[3];
        gather_partition_cdf((const uint16_t*)&ctx + off, bottom_out, c);
        coder.encode(c, 2, v);
    }
};

// Token stream (GPU): the block syntax is generated in parallel per 16x16 unit into
// token lists; one wave per tile then runs the arithmetic coder over them in order.
//   symbol   [31:30] 0 | [29:26] N-1 | [25:22] value | [21:0] CDF offset (u16 index)
//   literal  [31:30] 1 | [29:25] bits-1 | [24:0] value (L(1) bits, MSB first)
//   gather   [31:30] 2 | [29] right-half-out | [28] value | [21:0] partition CDF offset
SK_HD uint32_t tok_sym(int off, int n, int v) { return ((uint32_t)(n - 1) << 26) | ((uint32_t)v << 22) | (uint32_t)off; }
SK_HD uint32_t tok_lit(uint32_t v, int nb) { return (1u << 30) | ((uint32_t)(nb - 1) << 25) | v; }
SK_HD uint32_t tok_gather(int off, bool bottom_out, int v) {
    return (2u << 30) | ((uint32_t)(bottom_out ? 0 : 1) << 29) | ((uint32_t)v << 28) | (uint32_t)off;
}

struct TokenSink {
    uint32_t* p;
    int n, cap;
    uint32_t pend;
    int pend_n;
    SK_HD void push(uint32_t t) {
        if (n < cap) p[n] = t;
        n++;
    }
    SK_HD void flush() {
        if (pend_n) push(tok_lit(pend, pend_n));
        pend = 0;
        pend_n = 0;
    }
    SK_HD void sym(int off, int n2, int v) {
        flush();
        push(tok_sym(off, n2, v));
    }
    SK_HD void bit(int b) {
        pend = (pend << 1) | (uint32_t)(b & 1);
        if (++pend_n == 24) flush();
    }
    SK_HD void lits(uint32_t v, int nbits) {
        for (int i = nbits - 1; i >= 0; i--) bit((v >> i) & 1);
    }
    SK_HD void gather(int off, bool bottom_out, int v) {
        flush();
        push(tok_gather(off, bottom_out, v));
    }
};

// Replays one token through a coder with the tile's adaptive CDFs.
template <class Coder>
SK_HD void code_token(Coder& coder, uint16_t* cdfs, uint32_t t) {
    const uint32_t kind = t >> 30;
    if (kind == 0) {
        coder.encode_adapt(cdfs + (t & 0x3fffff), (int)((t >> 26) & 15) + 1, (int)((t >> 22) & 15));
    } else if (kind == 1) {
        coder.literal(t & 0x1ffffff, (int)((t >> 25) & 31) + 1);
    } else {
        uint16_t c[3];
        gather_partition_cdf(cdfs + (t & 0x3fffff), ((t >> 29) & 1) == 0, c);
        coder.encode(c, 2, (int)((t >> 28) & 1));
    }
}

// ---------------------------------------------------------------------------------
// Coefficient syntax (§5.11.39 coeffs) of one transform block.
// lev: quantised levels, raster [row][col]; txs: TX_4X4..TX_16X16 (square);
// ctx_skip: all_zero context; ctx_dc: dc_sign context.
// Returns cul_level | dc_category << 6 (the value the level contexts store).
struct CoefCtx {
    int txb_skip, dc_sign;
};

SK_HD int eob_pt_of(int eob) {
    if (eob <= 2) return eob;
    int l = 0;
    while ((1 << (l + 1)) <= eob - 1) l++;   // floor(log2(eob - 1))
    return l + 2;
}

// Encoder choice: tail trimming of an inter block's levels (raster lev, n x n). The
// tokens of a block run to its last nonzero level in scan order, so a lone +-1 far
// behind the others costs a run of zero coeff_base symbols - the serial work of the
// GPU's CDF adaptation (k_av1_cdf) and bits - for a small error. From the end of the
// scan, a +-1 more than kTrimGap positions after the previous nonzero level (or the
// block start) is dropped; the first level that is larger, or closer, ends the trim.
constexpr int kTrimGap = 4;
SK_HD bool trim_keep(int level, int s, int prev) { return level > 1 || level < -1 || s - prev <= kTrimGap; }
SK_HD void trim_tail(int16_t* lev, int log2n) {
    const int nn = 1 << (2 * log2n);
    int last = -1, prev = -1;
    for (int s = nn - 1; s >= 0 && last < 0; s--) {
        if (!lev[default_scan(log2n, s)]) continue;
        prev = -1;
        for (int t2 = s - 1; t2 >= 0; t2--)
            if (lev[default_scan(log2n, t2)]) {
                prev = t2;
                break;
            }
        if (trim_keep(lev[default_scan(log2n, s)], s, prev)) last = s;
    }
    for (int s = last + 1; s < nn; s++) lev[default_scan(log2n, s)] = 0;
}

template <class Sink>
SK_HD int code_coeffs(Sink& w, const CdfContext& cx, const int16_t* lev, int txs, int plane, CoefCtx cc,
                      bool is_inter, int intra_dir, int qidx, int tx_type = TX_DCT_DCT) {
    const int log2n = txs + 2, n = 1 << log2n, nn = n * n;
    const int ptype = plane > 0;
    // eob = 1 + last nonzero scan index
    int eob = 0;
    for (int c = nn - 1; c >= 0; c--)
        if (lev[default_scan(log2n, c)] != 0) {
            eob = c + 1;
            break;
        }
    w.sym(cdf_off(cx, cx.txb_skip[txs][cc.txb_skip]), 2, eob == 0);
    if (eob == 0) return 0;
    if (plane == 0 && qidx > 0) {   // transform_type: IDTX = index 0, DCT_DCT = 1 of the reduced sets
        const int sym = tx_type == TX_IDTX ? 0 : 1;
        if (is_inter) w.sym(cdf_off(cx, cx.inter_tx_set3[txs]), 2, sym);
        else w.sym(cdf_off(cx, cx.intra_tx_set2[txs][intra_dir]), 5, sym);
    }
    const int eob_multi = 2 * log2n - 4;   // log2(nn) - 4
    const int eob_pt = eob_pt_of(eob);
    switch (eob_multi) {
        case 0: w.sym(cdf_off(cx, cx.eob_pt_16[ptype][0]), 5, eob_pt - 1); break;
        case 2: w.sym(cdf_off(cx, cx.eob_pt_64[ptype][0]), 7, eob_pt - 1); break;
        default: w.sym(cdf_off(cx, cx.eob_pt_256[ptype][0]), 9, eob_pt - 1); break;
    }
    if (eob_pt >= 3) {
        const int off = eob - ((1 << (eob_pt - 2)) + 1);
        const int sh = eob_pt - 3;
        w.sym(cdf_off(cx, cx.eob_extra[txs][ptype][eob_pt - 3]), 2, (off >> sh) & 1);
        for (int i = 1; i < eob_pt - 2; i++) w.bit((off >> (sh - i)) & 1);
    }
    // base levels + ranges, reverse scan; q holds min(level, 15) as the decoder sees it
    int16_t q[256];
    for (int i = 0; i < nn; i++) q[i] = 0;
    for (int c = eob - 1; c >= 0; c--) {
        const int pos = default_scan(log2n, c);
        const int a = sk_abs(lev[pos]);
        const int row = pos >> log2n, col = pos & (n - 1);
        if (c == eob - 1) {
            const int ctx = c == 0 ? 0 : (c <= nn / 8 ? 1 : (c <= nn / 4 ? 2 : 3));
            w.sym(cdf_off(cx, cx.coeff_base_eob[txs][ptype][ctx]), 3, sk_min(a, 3) - 1);
        } else {
            int mag = 0;
            const int8_t off[5][2] = {{0, 1}, {1, 0}, {1, 1}, {0, 2}, {2, 0}};
            for (int k = 0; k < 5; k++) {
                const int rr = row + off[k][0], cc2 = col + off[k][1];
                if (rr < n && cc2 < n) mag += sk_min(q[(rr << log2n) + cc2], 3);
            }
            int ctx = sk_min((mag + 1) >> 1, 4);
            if (row == 0 && col == 0) ctx = 0;
            else {
                const int rm = sk_min(row, 4), cm = sk_min(col, 4);
                int o;
                if (txs == TX_4X4) {
                    constexpr uint8_t t4[5][5] = {{0, 1, 6, 6, 0}, {1, 6, 6, 21, 0}, {6, 6, 21, 21, 0},
                                                  {6, 21, 21, 21, 0}, {0, 0, 0, 0, 0}};
                    o = t4[rm][cm];
                } else {
                    constexpr uint8_t t8[5][5] = {{0, 1, 6, 6, 21}, {1, 6, 6, 21, 21}, {6, 6, 21, 21, 21},
                                                  {6, 21, 21, 21, 21}, {21, 21, 21, 21, 21}};
                    o = t8[rm][cm];
                }
                ctx += o;
            }
            w.sym(cdf_off(cx, cx.coeff_base[txs][ptype][ctx]), 4, sk_min(a, 3));
        }
        if (a > 2) {
            int mag = 0;
            const int8_t off[3][2] = {{0, 1}, {1, 0}, {1, 1}};
            for (int k = 0; k < 3; k++) {
                const int rr = row + off[k][0], cc2 = col + off[k][1];
                if (rr < n && cc2 < n) mag += q[(rr << log2n) + cc2];
            }
            mag = sk_min((mag + 1) >> 1, 6);
            const int ctx = pos == 0 ? mag : ((row < 2 && col < 2) ? mag + 7 : mag + 14);
            int level = 3;
            for (int idx = 0; idx < 4; idx++) {
                const int br = sk_min(a - level, 3);
                w.sym(cdf_off(cx, cx.coeff_br[sk_min(txs, TX_32X32)][ptype][ctx]), 4, br);
                level += br;
                if (br < 3) break;
            }
        }
        q[pos] = (int16_t)sk_min(a, 15);
    }
    // signs and Golomb remainders, forward scan
    int cul = 0, dcc = 0;
    for (int c = 0; c < eob; c++) {
        const int pos = default_scan(log2n, c);
        const int l = lev[pos];
        if (l == 0) continue;
        const int a = sk_abs(l);
        if (c == 0) w.sym(cdf_off(cx, cx.dc_sign[ptype][cc.dc_sign]), 2, l < 0);
        else w.bit(l < 0);
        if (a > 14) {
            const uint32_t x = (uint32_t)(a - 14);
            int len = 0;
            while ((x >> len) > 1) len++;   // len = bit length - 1
            for (int i = 0; i < len; i++) w.bit(0);
            w.bit(1);
            for (int i = len - 1; i >= 0; i--) w.bit((x >> i) & 1);
        }
        if (pos == 0) dcc = l < 0 ? 1 : 2;
        cul += a;
    }
    return sk_min(cul, 63) | (dcc << 6);
}

// ---------------------------------------------------------------------------------
// Motion vector syntax (§5.11.32 read_mv, MvCtx 0, no high precision).
template <class Sink>
SK_HD void code_mv_component(Sink& w, const CdfContext& cx, int comp, int v) {
    const uint16_t* sign = comp ? cx.mv1_sign[0] : cx.mv0_sign[0];
    const uint16_t* classes = comp ? cx.mv1_classes[0] : cx.mv0_classes[0];
    w.sym(cdf_off(cx, sign), 2, v < 0);
    const int mag = (v < 0 ? -v : v) - 1;   // ((d << 3) | (fr << 1) | hp), hp = 1
    int cls = 0;
    if (mag >= 16) {   // CLASS0_SIZE << 3 = 16
        cls = 1;
        while (mag >= (2 << (cls + 3))) cls++;
    }
    w.sym(cdf_off(cx, classes), 11, cls);
    if (cls == 0) {
        const int d = mag >> 3, fr = (mag >> 1) & 3;
        w.sym(cdf_off(cx, comp ? cx.mv1_class0[0] : cx.mv0_class0[0]), 2, d);
        w.sym(cdf_off(cx, comp ? cx.mv1_class0_fp[d] : cx.mv0_class0_fp[d]), 4, fr);
    } else {
        const int rem = mag - (2 << (cls + 2));
        const int d = rem >> 3, fr = (rem >> 1) & 3;
        for (int i = 0; i < cls; i++) w.sym(cdf_off(cx, comp ? cx.mv1_bits[i] : cx.mv0_bits[i]), 2, (d >> i) & 1);
        w.sym(cdf_off(cx, comp ? cx.mv1_fp[0] : cx.mv0_fp[0]), 4, fr);
    }
}

// diff: (row, col) in 1/8 pel, both even
template <class Sink>
SK_HD void code_mv(Sink& w, const CdfContext& cx, int drow, int dcol) {
    const int joint = (drow != 0 ? 2 : 0) | (dcol != 0 ? 1 : 0);
    w.sym(cdf_off(cx, cx.mv_joint[0]), 4, joint);
    if (drow != 0) code_mv_component(w, cx, 0, drow);
    if (dcol != 0) code_mv_component(w, cx, 1, dcol);
}

// ---------------------------------------------------------------------------------
// Frame view for the block syntax: everything the decisions left behind.
struct FrameView {
    Av1Geo geo;
    const BlkInfo* blk;          // [r8][c8]
    const int16_t* lev;          // [units][384] (unit grid = front-end MBs, stride unit_w)
    const uint8_t* lctx[3];      // level contexts (cul | dc << 6), 4x4 units per plane
    int lctx_w[3];
    int unit_w;                  // 16x16 units per row
    int qidx, key;
    int screen;                  // allow_screen_content_tools (palette syntax)
    const uint8_t* pal;          // [r8][c8][8] palette colours of each cell's block
    const uint8_t* src_y;        // source luma: the colour index map of a palette block
    int stride_y;
    MvStack* stk = nullptr;      // the reference MV stack's storage (set by the caller; GPU: this wave's LDS slot)
    SK_HD const BlkInfo& at(int r, int c) const { return blk[(r >> 1) * geo.c8 + (c >> 1)]; }
    SK_HD const uint8_t* pal_at(int r, int c) const { return pal + ((size_t)(r >> 1) * geo.c8 + (c >> 1)) * 8; }
    // levels of the block at mi (r, c) of size bsl in plane p (raster [row][col])
    SK_HD const int16_t* levels(int r, int c, int bsl, int p) const {
        const int16_t* u = lev + ((size_t)(r >> 2) * unit_w + (c >> 2)) * 384;
        if (bsl >= 2) return u + (p == 0 ? 0 : (p == 1 ? 256 : 320));
        const int k = ((r >> 1) & 1) * 2 + ((c >> 1) & 1);
        return u + (p == 0 ? 64 * k : (p == 1 ? 256 + 16 * k : 320 + 16 * k));
    }
    // selects without indexing lctx / lctx_w by a run-time plane: an indexed member array
    // keeps the whole view in GPU scratch memory
    SK_HD uint8_t lc(int p, int x4, int y4) const {
        const uint8_t* b = p == 0 ? lctx[0] : (p == 1 ? lctx[1] : lctx[2]);
        return b[(size_t)y4 * (p == 0 ? lctx_w[0] : lctx_w[1]) + x4];
    }
};

// above / left level contexts of a tx block (plane units of 4 samples), tile-bounded:
// AboveLevelContext is cleared at the tile start, LeftLevelContext at every SB row start
SK_HD CoefCtx coef_ctx(const FrameView& v, const TileRect& t, int plane, int x4, int y4, int n4) {
    const int ss = plane ? 1 : 0;
    const int row0 = t.mi_row0 >> ss, col0 = t.mi_col0 >> ss;
    const int max_x4 = v.geo.mi_cols >> ss, max_y4 = v.geo.mi_rows >> ss;
    int above = 0, left = 0, dcs = 0;
    if (y4 - 1 >= row0)
        for (int k = 0; k < n4; k++)
            if (x4 + k < max_x4) {
                const int q = v.lc(plane, x4 + k, y4 - 1);
                above |= q;
                dcs += (q >> 6) == 1 ? -1 : ((q >> 6) == 2 ? 1 : 0);
            }
    if (x4 - 1 >= col0)
        for (int k = 0; k < n4; k++)
            if (y4 + k < max_y4) {
                const int q = v.lc(plane, x4 - 1, y4 + k);
                left |= q;
                dcs += (q >> 6) == 1 ? -1 : ((q >> 6) == 2 ? 1 : 0);
            }
    CoefCtx cc;
    cc.txb_skip = plane == 0 ? 0 : 7 + (above != 0) + (left != 0);
    cc.dc_sign = dcs < 0 ? 1 : (dcs > 0 ? 2 : 0);
    return cc;
}

// ---------------------------------------------------------------------------------
// Palette (screen content tools; §5.11.46 palette_mode_info, §5.11.49 palette_tokens,
// §7.11.4 get_palette_cache / get_palette_color_context), luma only, on key frames.
// Encoder choice (av1_cpu.cpp intra_block = k_av1_intra_rec): a fully visible block
// whose source luma takes 2..8 distinct values can be coded as that exact palette, with
// no luma residual, when palette_rate2's cost is below the transform path's J.
constexpr int kPalMax = 8;
SK_HD int ceil_log2(int x) {
    if (x < 2) return 0;
    int i = 1, p = 2;
    while (p < x) {
        i++;
        p <<= 1;
    }
    return i;
}

// PaletteCache: the sorted union of the above (only inside the same 64-row superblock
// row) and left blocks' palettes, duplicates dropped. Returns its size.
SK_HD int palette_cache(const FrameView& v, const TileRect& t, int r, int c, uint8_t* cache) {
    const int an = inside(t, r - 1, c) && (r & 15) ? v.at(r - 1, c).pal_n : 0;
    const int ln = inside(t, r, c - 1) ? v.at(r, c - 1).pal_n : 0;
    const uint8_t* ac = an ? v.pal_at(r - 1, c) : nullptr;
    const uint8_t* lc = ln ? v.pal_at(r, c - 1) : nullptr;
    int ai = 0, li = 0, n = 0;
    while (ai < an && li < ln) {
        const int a = ac[ai], l = lc[li];
        if (l < a) {
            if (n == 0 || l != cache[n - 1]) cache[n++] = (uint8_t)l;
            li++;
        } else {
            if (n == 0 || a != cache[n - 1]) cache[n++] = (uint8_t)a;
            ai++;
            if (l == a) li++;
        }
    }
    for (; ai < an; ai++)
        if (n == 0 || ac[ai] != cache[n - 1]) cache[n++] = ac[ai];
    for (; li < ln; li++)
        if (n == 0 || lc[li] != cache[n - 1]) cache[n++] = lc[li];
    return n;
}

// ColorOrder and ColorContextHash -> context of the index at (i, j) of a colour map
// (pitch n); *order gets the colours by neighbour score as nibbles (colour of rank r in
// bits 4r..4r+3). Scores (<= 5) and the order live in packed registers: no arrays the GPU
// would index dynamically (scratch memory).
SK_HD int palette_color_context(const uint8_t* map, int n, int i, int j, int k, uint32_t* order) {
    uint32_t sc = 0, ord = 0x76543210u;   // nibble q: score / colour of rank q
    if (j > 0) sc += 2u << (4 * map[i * n + j - 1]);
    if (i > 0 && j > 0) sc += 1u << (4 * map[(i - 1) * n + j - 1]);
    if (i > 0) sc += 2u << (4 * map[(i - 1) * n + j]);
    auto nib = [](uint32_t w, int q) { return (int)((w >> (4 * q)) & 15u); };
    for (int q = 0; q < 3; q++) {
        int best = nib(sc, q), bi = q;
        for (int x = q + 1; x < k; x++)
            if (nib(sc, x) > best) {
                best = nib(sc, x);
                bi = x;
            }
        if (bi != q) {   // move rank bi to rank q, ranks q..bi-1 down one
            const uint32_t lo = (1u << (4 * q)) - 1u, mid = ((1u << (4 * bi)) - 1u) & ~lo;
            const uint32_t hi = bi == 7 ? 0u : ~((1u << (4 * (bi + 1))) - 1u);
            const uint32_t o = (uint32_t)nib(ord, bi);
            sc = (sc & (lo | hi)) | ((sc & mid) << 4) | ((uint32_t)best << (4 * q));
            ord = (ord & (lo | hi)) | ((ord & mid) << 4) | (o << (4 * q));
        }
    }
    *order = ord;
    const int hash = nib(sc, 0) + 2 * nib(sc, 1) + 2 * nib(sc, 2);
    return hash == 2 ? 0 : (hash == 5 ? 4 : (hash == 6 ? 3 : (hash == 7 ? 2 : (hash == 8 ? 1 : -1))));
}
// Rank of colour x in a packed order.
SK_HD int palette_rank(uint32_t order, int k, int x) {
    int rank = 0;
    for (int q = 0; q < k; q++) rank = (int)((order >> (4 * q)) & 15u) == x ? q : rank;
    return rank;
}

// Index of each sample of a palette block (raster, pitch n): its source value's position
// in the block's colours.
SK_HD int palette_index(const uint8_t* col, int k, int v) {
    int x = 0;
    for (int q = 0; q < k; q++) x = col[q] == v ? q : x;
    return x;
}

// ns(n) (§4.10.10) value x
template <class Sink>
SK_HD void code_ns(Sink& w, int n, int x) {
    int wb = 0;
    while ((1 << wb) <= n) wb++;
    const int m = (1 << wb) - n;
    if (x < m) {
        w.lits((uint32_t)x, wb - 1);
    } else {
        w.lits((uint32_t)((x + m) >> 1), wb - 1);
        w.bit((x + m) & 1);
    }
}

// palette_mode_info of a key-frame intra block (luma palette; has_palette_uv = 0)
template <class Sink>
SK_HD void code_palette_mode_info(Sink& w, const CdfContext& cx, const FrameView& v, const TileRect& t, int r, int c,
                                  int bsl, const BlkInfo& b) {
    const int bctx = 2 * bsl - 2;   // Mi_Width_Log2 + Mi_Height_Log2 - 2 (square blocks)
    const int k = b.pal_n;
    if (b.mode == DC_PRED) {
        const int ctx = (inside(t, r - 1, c) && v.at(r - 1, c).pal_n > 0) + (inside(t, r, c - 1) && v.at(r, c - 1).pal_n > 0);
        w.sym(cdf_off(cx, cx.palette_y_mode[bctx][ctx]), 2, k > 0);
        if (k > 0) {
            w.sym(cdf_off(cx, cx.palette_y_size[bctx]), 7, k - 2);
            const uint8_t* col = v.pal_at(r, c);
            uint8_t cache[2 * kPalMax];
            const int cn = palette_cache(v, t, r, c, cache);
            uint32_t from_cache = 0;   // bit q: colour q comes from the cache
            int idx = 0;
            for (int i = 0; i < cn && idx < k; i++) {
                int hit = -1;
                for (int q = 0; q < k; q++) hit = col[q] == cache[i] ? q : hit;
                w.bit(hit >= 0);
                if (hit >= 0) {
                    from_cache |= 1u << hit;
                    idx++;
                }
            }
            // the remaining colours ascending: the first as 8 bits, then deltas - 1 in
            // paletteBits bits (5 + palette_num_extra_bits, shrinking with the range left)
            int lit[kPalMax], m = 0;
            for (int q = 0; q < k; q++)
                if (!((from_cache >> q) & 1)) lit[m++] = col[q];
            if (m > 0) w.lits((uint32_t)lit[0], 8);
            if (m > 1) {
                int need = 0;
                for (int q = 1; q < m; q++) need = sk_max(need, ceil_log2(lit[q] - lit[q - 1]));
                const int extra = sk_max(need - 5, 0);
                w.lits((uint32_t)extra, 2);
                int bits = 5 + extra;
                for (int q = 1; q < m; q++) {
                    w.lits((uint32_t)(lit[q] - lit[q - 1] - 1), bits);
                    bits = sk_min(bits, ceil_log2(255 - lit[q]));
                }
            }
        }
    }
    if (b.uv_mode == DC_PRED) w.sym(cdf_off(cx, cx.palette_uv_mode[k > 0]), 2, 0);
}

// palette_tokens: the colour index map, first index as ns(k), then every other sample on
// anti-diagonals (top-right to bottom-left) as its rank in the neighbour colour order.
template <class Sink>
SK_HD void code_palette_tokens(Sink& w, const CdfContext& cx, const FrameView& v, int r, int c, int bsl, int k) {
    const int n = 4 << bsl;
    const uint8_t* col = v.pal_at(r, c);
    uint8_t map[256];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++)
            map[i * n + j] = (uint8_t)palette_index(col, k, v.src_y[(size_t)(r * 4 + i) * v.stride_y + c * 4 + j]);
    code_ns(w, k, map[0]);
    for (int d = 1; d < 2 * n - 1; d++)
        for (int j = sk_min(d, n - 1); j >= sk_max(0, d - n + 1); j--) {
            const int i = d - j;
            uint32_t order;
            const int ctx = palette_color_context(map, n, i, j, k, &order);
            w.sym(cdf_off(cx, cx.palette_y_color[k - 2][ctx]), k, palette_rank(order, k, map[i * n + j]));
        }
}

// Encoder: the distinct luma values (ascending) of the n x n block at src when there are
// 2..kPalMax of them (returns the count, else 0).
SK_HD int palette_colors(const uint8_t* src, int stride, int n, uint8_t* col) {
    uint32_t seen[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            const int v = src[(size_t)i * stride + j];
            seen[v >> 5] |= 1u << (v & 31);
        }
    int k = 0;
    for (int w = 0; w < 8; w++) k += __builtin_popcount(seen[w]);
    if (k < 2 || k > kPalMax) return 0;
    int q = 0;
    for (int v = 0; v < 256; v++)
        if ((seen[v >> 5] >> (v & 31)) & 1) col[q++] = (uint8_t)v;
    return k;
}

// Encoder: estimated rate (half bits) of coding an n x n block as its k-colour palette
// (map: raster indices, pitch n) - header, then per sample 0.5 bit when it repeats its
// left or top neighbour's index, else 1 + log2(k) bits. (i, j) one sample; the block's
// total is palette_rate2_head + the sum of palette_rate2_px over its samples.
SK_HD int palette_rate2_head(int k) { return 2 * (1 + 3 + 8 + 2 + 5 * (k - 1)); }
SK_HD int palette_rate2_px(const uint8_t* map, int n, int i, int j, int k) {
    const int x = map[i * n + j];
    if (i == 0 && j == 0) return 2 * ceil_log2(k);
    const bool rep = (j > 0 && map[i * n + j - 1] == x) || (i > 0 && map[(i - 1) * n + j] == x);
    return rep ? 1 : 2 + 2 * ceil_log2(k);
}

// Is the block containing mi (mr, mc) before the block at (r, c) in coding order?
// (raster superblocks, recursive quad-split Z order inside each 64x64 superblock)
SK_HD uint32_t zorder16(int r, int c) {
    uint32_t m = 0;
    for (int b = 3; b >= 0; b--) m = (m << 2) | (uint32_t)(((r >> b) & 1) << 1) | (uint32_t)((c >> b) & 1);
    return m;
}
SK_HD bool decoded_before(int mr, int mc, int r, int c) {
    const int sr = mr >> 4, sc = mc >> 4, cr = r >> 4, cc = c >> 4;
    if (sr != cr) return sr < cr;
    if (sc != cc) return sc < cc;
    return zorder16(mr & 15, mc & 15) < zorder16(r & 15, c & 15);
}
struct DecodedBefore {
    int r, c;
    SK_HD bool operator()(int mr, int mc) const { return decoded_before(mr, mc, r, c); }
};

// Mode info + residual of one block (§5.11.5 decode_block).
template <class Sink>
SK_HD void code_block(Sink& w, const CdfContext& cx, const FrameView& v, const TileRect& t, int r, int c, int bsl) {
    const BlkInfo& b = v.at(r, c);
    const bool au = inside(t, r - 1, c), al = inside(t, r, c - 1);
    const int sctx = (au ? (int)blk_skip(v.at(r - 1, c)) : 0) + (al ? (int)blk_skip(v.at(r, c - 1)) : 0);
    w.sym(cdf_off(cx, cx.skip[sctx]), 2, blk_skip(b));
    if (v.key) {
        const int am = au ? v.at(r - 1, c).mode : DC_PRED, lm = al ? v.at(r, c - 1).mode : DC_PRED;
        w.sym(cdf_off(cx, cx.kf_y_mode[intra_mode_ctx(am)][intra_mode_ctx(lm)]), 13, b.mode);
        if (is_directional(b.mode)) w.sym(cdf_off(cx, cx.angle_delta[b.mode - V_PRED]), 7, 3);
        if (bsl <= 3) w.sym(cdf_off(cx, cx.uv_mode_cfl_allowed[b.mode]), 14, b.uv_mode);
        else w.sym(cdf_off(cx, cx.uv_mode_cfl_not_allowed[b.mode]), 13, b.uv_mode);
        if (is_directional(b.uv_mode)) w.sym(cdf_off(cx, cx.angle_delta[b.uv_mode - V_PRED]), 7, 3);
        if (v.screen) code_palette_mode_info(w, cx, v, t, r, c, bsl, b);
    } else {
        // is_inter: every block of an inter frame is inter, so no neighbour is intra (ctx 0)
        w.sym(cdf_off(cx, cx.intra_inter[0]), 2, 1);
        const int nref = (au ? 1 : 0) + (al ? 1 : 0);
        const int rctx = nref == 0 ? 1 : 2;
        w.sym(cdf_off(cx, cx.single_ref[rctx][0]), 2, 0);   // single_ref_p1: forward
        w.sym(cdf_off(cx, cx.single_ref[rctx][2]), 2, 0);   // p3: LAST / LAST2
        w.sym(cdf_off(cx, cx.single_ref[rctx][3]), 2, 0);   // p4: LAST
        MvStack& s = *v.stk;   // caller's (GPU: LDS; a per-lane array indexed at run time lives in scratch)
        const BlkGrid grid{v.blk, v.geo.c8};
        find_mv_stack(s, grid, t, v.geo.mi_rows, v.geo.mi_cols, r, c, bsl, DecodedBefore{r, c});
        const int mode = b.mode, idx = (b.flags >> 4) & 3;
        w.sym(cdf_off(cx, cx.newmv[s.newmv_ctx]), 2, mode != NEWMV);
        if (mode != NEWMV) {
            w.sym(cdf_off(cx, cx.zeromv[0]), 2, mode != GLOBALMV);
            if (mode != GLOBALMV) w.sym(cdf_off(cx, cx.refmv[s.refmv_ctx]), 2, mode != NEARESTMV);
        }
        if (mode == NEWMV) {
            for (int k = 0; k < 2; k++)
                if (s.n > k + 1) {
                    w.sym(cdf_off(cx, cx.drl[drl_ctx(s, k)]), 2, idx != k);
                    if (idx == k) break;
                }
        } else if (mode == NEARMV) {
            for (int k = 1; k < 3; k++)
                if (s.n > k + 1) {
                    w.sym(cdf_off(cx, cx.drl[drl_ctx(s, k)]), 2, idx != k);
                    if (idx == k) break;
                }
        }
        if (mode == NEWMV) {
            const int pos = s.n <= 1 ? 0 : idx;
            code_mv(w, cx, b.mv_row - s.mv[pos][0], b.mv_col - s.mv[pos][1]);
        }
    }
    if (b.pal_n) code_palette_tokens(w, cx, v, r, c, bsl, b.pal_n);
    if (blk_skip(b)) return;
    code_coeffs(w, cx, v.levels(r, c, bsl, 0), bsl, 0, coef_ctx(v, t, 0, c, r, 1 << bsl), blk_inter(b), b.mode, v.qidx,
                b.tx_type);
    for (int p = 1; p < 3; p++)
        code_coeffs(w, cx, v.levels(r, c, bsl, p), bsl - 1, p, coef_ctx(v, t, p, c >> 1, r >> 1, (1 << bsl) >> 1),
                    blk_inter(b), b.mode, v.qidx);
}

// Partition symbol of the node (r, c, bsl), NONE or SPLIT (gathered bool at edges).
template <class Sink>
SK_HD bool code_partition_symbol(Sink& w, const CdfContext& cx, const FrameView& v, const TileRect& t, int r, int c,
                                 int bsl) {
    const int half = (1 << bsl) >> 1;
    const bool has_rows = r + half < v.geo.mi_rows, has_cols = c + half < v.geo.mi_cols;
    const bool none = v.at(r, c).bsl == bsl && has_rows && has_cols;
    const bool au = inside(t, r - 1, c), al = inside(t, r, c - 1);
    const int actx = au && v.at(r - 1, c).bsl < bsl, lctx2 = al && v.at(r, c - 1).bsl < bsl;
    const int ctx = lctx2 * 2 + actx;
    const uint16_t* pc = bsl == 1 ? cx.partition_w8[ctx]
                         : bsl == 2 ? cx.partition_w16[ctx]
                         : bsl == 3 ? cx.partition_w32[ctx]
                                    : cx.partition_w64[ctx];
    if (has_rows && has_cols) w.sym(cdf_off(cx, pc), bsl == 1 ? 4 : 10, none ? PARTITION_NONE : PARTITION_SPLIT);
    else if (has_cols) w.gather(cdf_off(cx, pc), true, 1);
    else if (has_rows) w.gather(cdf_off(cx, pc), false, 1);
    return none;
}

// Everything the 16x16 unit (ux, uy) contributes to its tile, in coding order: the
// partition symbols of the 64 / 32 nodes it opens, then its own block(s); a unit
// inside a larger (merged) block contributes nothing. Units in Z order within
// raster superblocks reproduce decode_partition's order exactly.
template <class Sink>
SK_HD void code_unit(Sink& w, const CdfContext& cx, const FrameView& v, const TileRect& t, int ux, int uy) {
    const int r = uy * 4, c = ux * 4;
    if (r >= v.geo.mi_rows || c >= v.geo.mi_cols) return;
    const int own = v.at(r, c).bsl;
    for (int L = 4; L >= 3; L--) {
        const int m = (1 << L) - 1;
        if ((r & m) || (c & m)) {
            if (own >= L) return;   // inside a merged block coded by its origin unit
            continue;
        }
        if (code_partition_symbol(w, cx, v, t, r, c, L)) {
            code_block(w, cx, v, t, r, c, L);
            return;
        }
    }
    if (code_partition_symbol(w, cx, v, t, r, c, 2)) {
        code_block(w, cx, v, t, r, c, 2);
        return;
    }
    for (int q = 0; q < 4; q++) {
        const int rr = r + (q >> 1) * 2, cc = c + (q & 1) * 2;
        if (rr >= v.geo.mi_rows || cc >= v.geo.mi_cols) continue;
        code_partition_symbol(w, cx, v, t, rr, cc, 1);
        code_block(w, cx, v, t, rr, cc, 1);
    }
}

// Units of a tile in coding order: index i -> (ux, uy). Returns false past the end.
SK_HD bool tile_unit(const Av1Geo& g, const TileRect& t, int i, int* ux, int* uy) {
    const int sbw = (t.mi_col1 - t.mi_col0 + 15) >> 4;
    const int sb = i >> 4, k = i & 15;
    const int sr = sb / sbw, sc = sb % sbw;
    const int ury = (k >> 3 & 1) << 1 | (k >> 1 & 1), urx = (k >> 2 & 1) << 1 | (k & 1);
    *uy = ((t.mi_row0 >> 4) + sr) * 4 + ury;
    *ux = ((t.mi_col0 >> 4) + sc) * 4 + urx;
    return (t.mi_row0 >> 4) + sr < ((t.mi_row1 + 15) >> 4);
}
SK_HD int tile_units(const TileRect& t) {
    return 16 * ((t.mi_col1 - t.mi_col0 + 15) >> 4) * ((t.mi_row1 - t.mi_row0 + 15) >> 4);
}

}  // namespace sk::av1
