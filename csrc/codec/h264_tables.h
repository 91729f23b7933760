// H.264 (ITU-T Rec. H.264 | ISO/IEC 14496-10) constant tables used by the CAVLC
// Constrained-Baseline encoder. Values are the normative VLC / scaling tables of
// the standard (clauses 8.5 and 9.2). Tests check every VLC table for the
// prefix-free property and Kraft completeness (tests/test_h264_tables.py).
#pragma once
#include "sk_common.h"

// ---- coeff_token (Table 9-5) ----------------------------------------------
// index [vlc][TotalCoeff * 4 + TrailingOnes]; vlc 0: 0<=nC<2, 1: 2<=nC<4,
// 2: 4<=nC<8, 3: nC>=8 (6-bit fixed length).
SK_TABLE uint8_t H264_COEFF_TOKEN_LEN[4][68] = {
    {1, 0, 0, 0, 6, 2, 0, 0, 8, 6, 3, 0, 9, 8, 7, 5, 10, 9, 8, 6, 11, 10, 9, 7, 13, 11, 10, 8,
     13, 13, 11, 9, 13, 13, 13, 10, 14, 14, 13, 11, 14, 14, 14, 13, 15, 15, 14, 14, 15, 15,
     15, 14, 16, 15, 15, 15, 16, 16, 16, 15, 16, 16, 16, 16, 16, 16, 16, 16},
    {2, 0, 0, 0, 6, 2, 0, 0, 6, 5, 3, 0, 7, 6, 6, 4, 8, 6, 6, 4, 8, 7, 7, 5, 9, 8, 8, 6,
     11, 9, 9, 6, 11, 11, 11, 7, 12, 11, 11, 9, 12, 12, 12, 11, 12, 12, 12, 11, 13, 13,
     13, 12, 13, 13, 13, 13, 13, 14, 13, 13, 14, 14, 14, 13, 14, 14, 14, 14},
    {4, 0, 0, 0, 6, 4, 0, 0, 6, 5, 4, 0, 6, 5, 5, 4, 7, 5, 5, 4, 7, 5, 5, 4, 7, 6, 6, 4,
     7, 6, 6, 4, 8, 7, 7, 5, 8, 8, 7, 6, 9, 8, 8, 7, 9, 9, 8, 8, 9, 9, 9, 8, 10, 9, 9, 9,
     10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10, 10},
    {6, 0, 0, 0, 6, 6, 0, 0, 6, 6, 6, 0, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
     6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6,
     6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6},
};
SK_TABLE uint8_t H264_COEFF_TOKEN_CODE[4][68] = {
    {1, 0, 0, 0, 5, 1, 0, 0, 7, 4, 1, 0, 7, 6, 5, 3, 7, 6, 5, 3, 7, 6, 5, 4, 15, 6, 5, 4,
     11, 14, 5, 4, 8, 10, 13, 4, 15, 14, 9, 4, 11, 10, 13, 12, 15, 14, 9, 12, 11, 10, 13, 8,
     15, 1, 9, 12, 11, 14, 13, 8, 7, 10, 9, 12, 4, 6, 5, 8},
    {3, 0, 0, 0, 11, 2, 0, 0, 7, 7, 3, 0, 7, 10, 9, 5, 7, 6, 5, 4, 4, 6, 5, 6, 7, 6, 5, 8,
     15, 6, 5, 4, 11, 14, 13, 4, 15, 10, 9, 4, 11, 14, 13, 12, 8, 10, 9, 8, 15, 14, 13, 12,
     11, 10, 9, 12, 7, 11, 6, 8, 9, 8, 10, 1, 7, 6, 5, 4},
    {15, 0, 0, 0, 15, 14, 0, 0, 11, 15, 13, 0, 8, 12, 14, 12, 15, 10, 11, 11, 11, 8, 9, 10,
     9, 14, 13, 9, 8, 10, 9, 8, 15, 14, 13, 13, 11, 14, 10, 12, 15, 10, 13, 12, 11, 14, 9, 12,
     8, 10, 13, 8, 13, 7, 9, 12, 9, 12, 11, 10, 5, 8, 7, 6, 1, 4, 3, 2},
    {3, 0, 0, 0, 0, 1, 0, 0, 4, 5, 6, 0, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
     21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42,
     43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63},
};
// Chroma DC (nC == -1), index [TotalCoeff * 4 + TrailingOnes], TotalCoeff <= 4.
SK_TABLE uint8_t H264_CDC_COEFF_TOKEN_LEN[20] = {2, 0, 0, 0, 6, 1, 0, 0, 6, 6, 3, 0,
                                                 6, 7, 7, 6, 6, 8, 8, 7};
SK_TABLE uint8_t H264_CDC_COEFF_TOKEN_CODE[20] = {1, 0, 0, 0, 7, 1, 0, 0, 4, 6, 1, 0,
                                                  3, 3, 2, 5, 2, 3, 2, 0};
// Maximum coeff_token length over the four luma tables (for the MB-size bound).
SK_TABLE uint8_t H264_COEFF_TOKEN_MAXLEN[68] = {
    6, 0, 0, 0, 6, 6, 0, 0, 8, 6, 6, 0, 9, 8, 7, 6, 10, 9, 8, 6, 11, 10, 9, 7, 13, 11, 10, 8,
    13, 13, 11, 9, 13, 13, 13, 10, 14, 14, 13, 11, 14, 14, 14, 13, 15, 15, 14, 14, 15, 15,
    15, 14, 16, 15, 15, 15, 16, 16, 16, 15, 16, 16, 16, 16, 16, 16, 16, 16};

// Longest coeff_token (any nC table, any TrailingOnes) per TotalCoeff, and longest
// total_zeros code per TotalCoeff (derived from the tables above; used only for
// conservative size bounds).
SK_TABLE uint8_t H264_CT_MAX_TC[17] = {6, 6, 8, 9, 10, 11, 13, 13, 13, 14, 14, 15, 15, 16, 16, 16, 16};
SK_TABLE uint8_t H264_TZ_MAX_TC[16] = {0, 9, 6, 6, 5, 5, 6, 6, 6, 6, 5, 4, 4, 3, 2, 1};

// ---- total_zeros (Tables 9-7, 9-8), index [TotalCoeff-1][total_zeros] -------
SK_TABLE uint8_t H264_TOTAL_ZEROS_LEN[15][16] = {
    {1, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 9},
    {3, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 6, 6, 6, 6},
    {4, 3, 3, 3, 4, 4, 3, 3, 4, 5, 5, 6, 5, 6},
    {5, 3, 4, 4, 3, 3, 3, 4, 3, 4, 5, 5, 5},
    {4, 4, 4, 3, 3, 3, 3, 3, 4, 5, 4, 5},
    {6, 5, 3, 3, 3, 3, 3, 3, 4, 3, 6},
    {6, 5, 3, 3, 3, 2, 3, 4, 3, 6},
    {6, 4, 5, 3, 2, 2, 3, 3, 6},
    {6, 6, 4, 2, 2, 3, 2, 5},
    {5, 5, 3, 2, 2, 2, 4},
    {4, 4, 3, 3, 1, 3},
    {4, 4, 2, 1, 3},
    {3, 3, 1, 2},
    {2, 2, 1},
    {1, 1},
};
SK_TABLE uint8_t H264_TOTAL_ZEROS_CODE[15][16] = {
    {1, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 3, 2, 1},
    {7, 6, 5, 4, 3, 5, 4, 3, 2, 3, 2, 3, 2, 1, 0},
    {5, 7, 6, 5, 4, 3, 4, 3, 2, 3, 2, 1, 1, 0},
    {3, 7, 5, 4, 6, 5, 4, 3, 3, 2, 2, 1, 0},
    {5, 4, 3, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 7, 6, 5, 4, 3, 2, 1, 1, 0},
    {1, 1, 5, 4, 3, 3, 2, 1, 1, 0},
    {1, 1, 1, 3, 3, 2, 2, 1, 0},
    {1, 0, 1, 3, 2, 1, 1, 1},
    {1, 0, 1, 3, 2, 1, 1},
    {0, 1, 1, 2, 1, 3},
    {0, 1, 1, 1, 1},
    {0, 1, 1, 1},
    {0, 1, 1},
    {0, 1},
};
// Chroma DC 2x2 total_zeros (Table 9-9a), index [TotalCoeff-1][total_zeros].
SK_TABLE uint8_t H264_CDC_TOTAL_ZEROS_LEN[3][4] = {{1, 2, 3, 3}, {1, 2, 2, 0}, {1, 1, 0, 0}};
SK_TABLE uint8_t H264_CDC_TOTAL_ZEROS_CODE[3][4] = {{1, 1, 1, 0}, {1, 1, 0, 0}, {1, 0, 0, 0}};

// ---- run_before (Table 9-10), index [min(zerosLeft,7)-1][run_before] --------
SK_TABLE uint8_t H264_RUN_BEFORE_LEN[7][16] = {
    {1, 1},
    {1, 2, 2},
    {2, 2, 2, 2},
    {2, 2, 2, 3, 3},
    {2, 2, 3, 3, 3, 3},
    {2, 3, 3, 3, 3, 3, 3},
    {3, 3, 3, 3, 3, 3, 3, 4, 5, 6, 7, 8, 9, 10, 11},
};
SK_TABLE uint8_t H264_RUN_BEFORE_CODE[7][16] = {
    {1, 0},
    {1, 1, 0},
    {3, 2, 1, 0},
    {3, 2, 1, 1, 0},
    {3, 2, 3, 2, 1, 0},
    {3, 0, 1, 3, 2, 5, 4},
    {7, 6, 5, 4, 3, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1},
};

// ---- scans / block geometry --------------------------------------------------
// Frame zig-zag: scan index -> raster index (row*4 + col) inside a 4x4 block.
SK_TABLE uint8_t H264_ZIGZAG4x4[16] = {0, 1, 4, 8, 5, 2, 3, 6, 9, 12, 13, 10, 7, 11, 14, 15};
// raster index -> scan index (inverse of the zig-zag)
SK_TABLE uint8_t H264_INV_ZIGZAG4x4[16] = {0, 1, 5, 6, 2, 4, 7, 12, 3, 8, 11, 13, 9, 10, 14, 15};
// luma4x4BlkIdx -> (x, y) in 4x4-block units inside the macroblock.
SK_TABLE uint8_t H264_BLK_X[16] = {0, 1, 0, 1, 2, 3, 2, 3, 0, 1, 0, 1, 2, 3, 2, 3};
SK_TABLE uint8_t H264_BLK_Y[16] = {0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3};
// (y*4 + x) -> luma4x4BlkIdx
SK_TABLE uint8_t H264_BLK_FROM_XY[16] = {0, 1, 4, 5, 2, 3, 6, 7, 8, 9, 12, 13, 10, 11, 14, 15};

// Arithmetic forms of the small per-position tables above (no memory access on
// the GPU; lane-dependent table indices would otherwise become vector loads).
SK_HD int zigzag4x4(int k) { return (int)((0xfeb7adc963258410ULL >> (4 * k)) & 15); }
SK_HD int inv_zigzag4x4(int r) { return (int)((0xfea9db83c7426510ULL >> (4 * r)) & 15); }
SK_HD int blk_x(int b) { return (b & 1) | (((b >> 2) & 1) << 1); }
SK_HD int blk_y(int b) { return ((b >> 1) & 1) | (((b >> 3) & 1) << 1); }
SK_HD int blk_from_xy(int x, int y) { return (x & 1) | ((y & 1) << 1) | ((x >> 1) << 2) | ((y >> 1) << 3); }

// ---- quantisation ------------------------------------------------------------
// Forward quant multipliers MF[qp%6][class]; class 0: (even,even) positions,
// 1: (odd,odd), 2: mixed.
SK_TABLE int32_t H264_QUANT_MF[6][3] = {{13107, 5243, 8066}, {11916, 4660, 7490},
                                        {10082, 4194, 6554}, {9362, 3647, 5825},
                                        {8192, 3355, 5243},  {7282, 2893, 4559}};
// normAdjust4x4 v[qp%6][class] (LevelScale4x4 = 16 * v with flat weights).
SK_TABLE int32_t H264_DEQUANT_V[6][3] = {{10, 16, 13}, {11, 18, 14}, {13, 20, 16},
                                         {14, 23, 18}, {16, 25, 20}, {18, 29, 23}};
// position class of raster index r inside a 4x4 block
SK_TABLE uint8_t H264_POS_CLASS[16] = {0, 2, 0, 2, 2, 1, 2, 1, 0, 2, 0, 2, 2, 1, 2, 1};
// QPc as a function of qPi (Table 8-15), qPi in [0, 51]
SK_TABLE uint8_t H264_CHROMA_QP[52] = {
    0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17,
    18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 29, 30, 31, 32, 32, 33,
    34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39};

// ---- coded_block_pattern me(v) mapping (Table 9-4, ChromaArrayType 1/2) -------
// cbp (0..47) -> codeNum
SK_TABLE uint8_t H264_CBP_TO_CODE_INTRA[48] = {
    3,  29, 30, 17, 31, 18, 37, 8,  32, 38, 19, 9,  20, 10, 11, 2,
    16, 33, 34, 21, 35, 22, 39, 4,  36, 40, 23, 5,  24, 6,  7,  1,
    41, 42, 43, 25, 44, 26, 46, 12, 45, 47, 27, 13, 28, 14, 15, 0};
SK_TABLE uint8_t H264_CBP_TO_CODE_INTER[48] = {
    0,  2,  3,  7,  4,  8,  17, 13, 5,  18, 9,  14, 10, 15, 16, 11,
    1,  32, 33, 36, 34, 37, 44, 40, 35, 45, 38, 41, 39, 42, 43, 19,
    6,  24, 25, 20, 26, 21, 46, 28, 27, 47, 22, 29, 23, 30, 31, 12};

// ---- VLC tables as one POD block: copied into LDS by the GPU kernels so that
// per-lane (divergent) lookups are LDS reads, not dependent global loads.
struct CavlcTables {
    uint8_t ct_len[4][68], ct_code[4][68];
    uint8_t cdc_len[20], cdc_code[20];
    uint8_t tz_len[15][16], tz_code[15][16];
    uint8_t cdc_tz_len[3][4], cdc_tz_code[3][4];
    uint8_t rb_len[7][16], rb_code[7][16];
    uint8_t ct_maxlen[68];
    uint8_t ct_max_tc[17], tz_max_tc[16];
    uint8_t pad[11];
};

SK_HD void cavlc_tables_copy_range(CavlcTables& t, int begin, int step) {
    uint8_t* d = reinterpret_cast<uint8_t*>(&t);
    for (int i = begin; i < (int)sizeof(CavlcTables); i += step) {
        uint8_t v = 0;
        int k = i;
#define SK_CP(arr)                                                   \
    if (k >= 0 && k < (int)sizeof(arr)) v = (&arr[0][0])[k];         \
    k -= (int)sizeof(arr);
#define SK_CP1(arr)                                                  \
    if (k >= 0 && k < (int)sizeof(arr)) v = arr[k];                  \
    k -= (int)sizeof(arr);
        SK_CP(H264_COEFF_TOKEN_LEN) SK_CP(H264_COEFF_TOKEN_CODE) SK_CP1(H264_CDC_COEFF_TOKEN_LEN)
        SK_CP1(H264_CDC_COEFF_TOKEN_CODE) SK_CP(H264_TOTAL_ZEROS_LEN) SK_CP(H264_TOTAL_ZEROS_CODE)
        SK_CP(H264_CDC_TOTAL_ZEROS_LEN) SK_CP(H264_CDC_TOTAL_ZEROS_CODE) SK_CP(H264_RUN_BEFORE_LEN)
        SK_CP(H264_RUN_BEFORE_CODE) SK_CP1(H264_COEFF_TOKEN_MAXLEN)
        SK_CP1(H264_CT_MAX_TC) SK_CP1(H264_TZ_MAX_TC)
#undef SK_CP
#undef SK_CP1
        d[i] = v;
    }
}
