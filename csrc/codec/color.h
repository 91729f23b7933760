// BGRx -> YCbCr 4:2:0 conversion (BT.709, limited or full range), integer
// arithmetic shared by the CPU path and the K1 HIP kernel.
#pragma once
#include <string.h>
#include "sk_common.h"

namespace sk {

// Converts one 2x2 quad. p0/p1 point at the first pixel of the upper / lower row
// (4 bytes per pixel, B G R X). Writes y[0..3] (raster), *cb, *cr.
SK_HD void bgrx_quad_to_yuv(const uint8_t* p0a, const uint8_t* p0b, const uint8_t* p1a,
                            const uint8_t* p1b, int full_range, uint8_t* y, uint8_t* cb,
                            uint8_t* cr) {
    const uint8_t* px[4] = {p0a, p0b, p1a, p1b};
    int rs = 0, gs = 0, bs = 0;
    for (int i = 0; i < 4; i++) {
        int b = px[i][0], g = px[i][1], r = px[i][2];
        rs += r;
        gs += g;
        bs += b;
        int yy = full_range ? ((54 * r + 183 * g + 19 * b + 128) >> 8)
                            : (((47 * r + 157 * g + 16 * b + 128) >> 8) + 16);
        y[i] = (uint8_t)sk_clip255(yy);
    }
    int u, v;
    if (full_range) {
        u = ((-29 * rs - 99 * gs + 128 * bs + 512) >> 10) + 128;
        v = ((128 * rs - 116 * gs - 12 * bs + 512) >> 10) + 128;
    } else {
        u = ((-26 * rs - 86 * gs + 112 * bs + 512) >> 10) + 128;
        v = ((112 * rs - 102 * gs - 10 * bs + 512) >> 10) + 128;
    }
    *cb = (uint8_t)sk_clip255(u);
    *cr = (uint8_t)sk_clip255(v);
}

// K2 resampling (fused into K1): bilinear, pixel centres aligned, 8-bit weights,
// edge clamped; integer only, so the CPU reference and the kernel agree exactly.
// step_x / step_y = source / destination size in 16.16 fixed point.
struct ScaleParams {
    int32_t src_w, src_h, step_x, step_y;
};
SK_HD ScaleParams scale_params(int src_w, int src_h, int dst_w, int dst_h) {
    ScaleParams s;
    s.src_w = src_w;
    s.src_h = src_h;
    s.step_x = (int32_t)(((int64_t)src_w << 16) / dst_w);
    s.step_y = (int32_t)(((int64_t)src_h << 16) / dst_h);
    return s;
}
// Source position (16.16) of destination coordinate d: (d + 0.5) * step - 0.5, clamped at 0.
SK_HD int32_t scale_pos(int d, int32_t step) {
    const int32_t p = (int32_t)((((int64_t)(2 * d + 1) * step) >> 1) - 0x8000);
    return p < 0 ? 0 : p;
}
SK_HD uint32_t bilerp4(uint32_t a, uint32_t b, int w) {   // per byte: (a * (256 - w) + b * w) / 256, 8.8 kept
    uint32_t out = 0;
    for (int c = 0; c < 4; c++) {
        const uint32_t x = (a >> (8 * c)) & 255, y = (b >> (8 * c)) & 255;
        out |= ((x * (256 - w) + y * w + 128) >> 8) << (8 * c);
    }
    return out;
}
SK_HD uint32_t scale_fetch(const uint8_t* bgrx, int stride, const ScaleParams& s, int x, int y) {
    const int32_t px = scale_pos(x, s.step_x), py = scale_pos(y, s.step_y);
    int x0 = px >> 16, y0 = py >> 16;
    x0 = x0 < s.src_w - 1 ? x0 : s.src_w - 1;
    y0 = y0 < s.src_h - 1 ? y0 : s.src_h - 1;
    const int x1 = x0 + 1 < s.src_w ? x0 + 1 : s.src_w - 1, y1 = y0 + 1 < s.src_h ? y0 + 1 : s.src_h - 1;
    const int wx = (px >> 8) & 255, wy = (py >> 8) & 255;
    const uint8_t* r0 = bgrx + (size_t)y0 * stride;
    const uint8_t* r1 = bgrx + (size_t)y1 * stride;
    uint32_t p00, p01, p10, p11;
    memcpy(&p00, r0 + 4 * x0, 4);
    memcpy(&p01, r0 + 4 * x1, 4);
    memcpy(&p10, r1 + 4 * x0, 4);
    memcpy(&p11, r1 + 4 * x1, 4);
    return bilerp4(bilerp4(p00, p01, wx), bilerp4(p10, p11, wx), wy);
}

}  // namespace sk
