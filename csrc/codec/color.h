// BGRx -> YCbCr 4:2:0 conversion (BT.709, limited or full range), integer
// arithmetic shared by the CPU path and the K1 HIP kernel.
#pragma once
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

}  // namespace sk
