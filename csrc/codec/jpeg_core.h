// Baseline JPEG (ITU-T T.81) stripe encoder core, shared by the CPU reference
// and the gfx950 kernels (csrc/kernels/jpeg_kernels.hip): JFIF full-range
// BT.601 colour, 4:2:0 MCUs, deterministic integer FDCT, IJG quality scaling of
// the Annex K tables, Annex K.3 Huffman tables. Every stripe is a complete JPEG
// image (SOI..EOI) as the browser client decodes each 0x03 stripe on its own
// (selkies-core.js:2155-2174, 2908-2923).
#pragma once
#include "sk_common.h"

namespace sk {
namespace jpeg {

SK_TABLE uint8_t JPEG_ZIGZAG[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
// Annex K.1 quantisation tables (natural order)
SK_TABLE uint8_t JPEG_STD_LUMA_Q[64] = {
    16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
    14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
    18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
SK_TABLE uint8_t JPEG_STD_CHROMA_Q[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99,
    99, 99, 47, 66, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// Annex K.3 Huffman tables: BITS (16 counts) and HUFFVAL
SK_TABLE uint8_t JPEG_DC_LUMA_BITS[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
SK_TABLE uint8_t JPEG_DC_CHROMA_BITS[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
SK_TABLE uint8_t JPEG_DC_VALS[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
SK_TABLE uint8_t JPEG_AC_LUMA_BITS[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
SK_TABLE uint8_t JPEG_AC_LUMA_VALS[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
    0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};
SK_TABLE uint8_t JPEG_AC_CHROMA_BITS[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
SK_TABLE uint8_t JPEG_AC_CHROMA_VALS[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
    0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
    0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
    0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa};

// Integer FDCT basis: round(4096 * c(u) * cos((2x+1) u pi / 16)), c(0)=1/sqrt(8), else 1/2.
SK_TABLE int16_t JPEG_DCT_C[8][8] = {
    {1448, 1448, 1448, 1448, 1448, 1448, 1448, 1448},
    {2009, 1703, 1138, 400, -400, -1138, -1703, -2009},
    {1892, 784, -784, -1892, -1892, -784, 784, 1892},
    {1703, -400, -2009, -1138, 1138, 2009, 400, -1703},
    {1448, -1448, -1448, 1448, 1448, -1448, -1448, 1448},
    {1138, -2009, 400, 1703, -1703, -400, 2009, -1138},
    {784, -1892, 1892, -784, -784, 1892, -1892, 784},
    {400, -1138, 1703, -2009, 2009, -1703, 1138, -400}};

// Derived per-quality tables, built on the host and copied into device memory /
// LDS by the kernels.
struct JpegTables {
    uint16_t q[2][64];            // natural-order quantisers (luma, chroma)
    uint16_t dc_code[2][12];      // DC Huffman codes (luma, chroma)
    uint8_t dc_len[2][12];
    uint16_t ac_code[2][256];     // AC Huffman codes by RS symbol
    uint8_t ac_len[2][256];
};

inline void build_huff(const uint8_t* bits, const uint8_t* vals, int nvals, uint16_t* code_out,
                       uint8_t* len_out) {
    int k = 0, code = 0;
    for (int l = 1; l <= 16; l++) {
        for (int i = 0; i < bits[l - 1]; i++) {
            if (k < nvals) {
                code_out[vals[k]] = (uint16_t)code;
                len_out[vals[k]] = (uint8_t)l;
            }
            k++;
            code++;
        }
        code <<= 1;
    }
}

inline int quality_scale(int quality) {
    if (quality < 1) quality = 1;
    if (quality > 100) quality = 100;
    return quality < 50 ? 5000 / quality : 200 - 2 * quality;
}

inline void build_tables(int quality, JpegTables& t) {
    int s = quality_scale(quality);
    for (int i = 0; i < 64; i++) {
        int a = (JPEG_STD_LUMA_Q[i] * s + 50) / 100, b = (JPEG_STD_CHROMA_Q[i] * s + 50) / 100;
        t.q[0][i] = (uint16_t)(a < 1 ? 1 : (a > 255 ? 255 : a));
        t.q[1][i] = (uint16_t)(b < 1 ? 1 : (b > 255 ? 255 : b));
    }
    for (int c = 0; c < 2; c++) {
        for (int i = 0; i < 256; i++) { t.ac_code[c][i] = 0; t.ac_len[c][i] = 0; }
        for (int i = 0; i < 12; i++) { t.dc_code[c][i] = 0; t.dc_len[c][i] = 0; }
    }
    build_huff(JPEG_DC_LUMA_BITS, JPEG_DC_VALS, 12, t.dc_code[0], t.dc_len[0]);
    build_huff(JPEG_DC_CHROMA_BITS, JPEG_DC_VALS, 12, t.dc_code[1], t.dc_len[1]);
    build_huff(JPEG_AC_LUMA_BITS, JPEG_AC_LUMA_VALS, 162, t.ac_code[0], t.ac_len[0]);
    build_huff(JPEG_AC_CHROMA_BITS, JPEG_AC_CHROMA_VALS, 162, t.ac_code[1], t.ac_len[1]);
}

// JFIF full-range BT.601 (what every JPEG decoder assumes)
SK_HD void rgb_to_ycc(int r, int g, int b, int* y, int* cb, int* cr) {
    *y = (77 * r + 150 * g + 29 * b + 128) >> 8;
    *cb = ((-43 * r - 85 * g + 128 * b + 128) >> 8) + 128;
    *cr = ((128 * r - 107 * g - 21 * b + 128) >> 8) + 128;
}

// level = round(acc / 2^18 / q): acc carries the 4096^2 basis scale minus the
// 2^6 inter-pass descale.
SK_HD int jpeg_quant(int acc, int q) {
    int64_t den = (int64_t)q << 18;
    int64_t num = (int64_t)acc;
    return (int)(num >= 0 ? (num + den / 2) / den : -((-num + den / 2) / den));
}

// Forward DCT + quantisation of one 8x8 block (natural-order input samples
// 0..255); writes levels in zig-zag order. Deterministic integer arithmetic.
SK_HD void fdct_quant(const uint8_t* px, int stride, const uint16_t* q, int16_t* out_zz) {
    int t[64], f[64];
    for (int y = 0; y < 8; y++)
        for (int u = 0; u < 8; u++) {
            int acc = 0;
            for (int x = 0; x < 8; x++) acc += ((int)px[y * stride + x] - 128) * JPEG_DCT_C[u][x];
            t[y * 8 + u] = (acc + 32) >> 6;
        }
    for (int v = 0; v < 8; v++)
        for (int u = 0; u < 8; u++) {
            int acc = 0;
            for (int y = 0; y < 8; y++) acc += JPEG_DCT_C[v][y] * t[y * 8 + u];
            f[v * 8 + u] = jpeg_quant(acc, q[v * 8 + u]);
        }
    for (int k = 0; k < 64; k++) out_zz[k] = (int16_t)f[JPEG_ZIGZAG[k]];
}

SK_HD int jpeg_category(int v) {
    int a = v < 0 ? -v : v;
    int n = 0;
    while (a) { n++; a >>= 1; }
    return n;
}
SK_HD uint32_t jpeg_value_bits(int v, int cat) {
    return (uint32_t)(v >= 0 ? v : v + (1 << cat) - 1) & ((1u << cat) - 1u);
}

// Huffman-codes one block (zig-zag levels, DC difference `dc_diff`) with table
// set `c` (0 luma, 1 chroma).
template <class W>
SK_HD void huff_block(W& w, const int16_t* zz, int dc_diff, const JpegTables& t, int c) {
    int cat = jpeg_category(dc_diff);
    w.put(t.dc_code[c][cat], t.dc_len[c][cat]);
    if (cat) w.put(jpeg_value_bits(dc_diff, cat), cat);
    int run = 0;
    for (int k = 1; k < 64; k++) {
        int v = zz[k];
        if (v == 0) { run++; continue; }
        while (run > 15) {
            w.put(t.ac_code[c][0xF0], t.ac_len[c][0xF0]);
            run -= 16;
        }
        int ac = jpeg_category(v);
        int rs = (run << 4) | ac;
        w.put(t.ac_code[c][rs], t.ac_len[c][rs]);
        w.put(jpeg_value_bits(v, ac), ac);
        run = 0;
    }
    if (run > 0) w.put(t.ac_code[c][0x00], t.ac_len[c][0x00]);  // EOB
}

}  // namespace jpeg
}  // namespace sk
