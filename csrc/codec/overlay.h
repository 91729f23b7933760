// K12 watermark / K13 cursor composite, fused into the colour conversion (K1) of both
// backends: the captured frame is never written; each sampled BGRx pixel is blended
// with up to two premultiplied-BGRA overlay images on its way into the YUV planes.
// Integer blend identical to the CPU composite it replaces (capture.cpp):
//   d = s + (d * (255 - a) + 127) / 255   per colour channel, skipped where a == 0.
#pragma once
#include <stdint.h>
#include "sk_common.h"

namespace sk {

constexpr int kOverlaySlots = 2;      // 0 = watermark, 1 = cursor
constexpr int kOverlayMaxDim = 512;   // image buffers are kOverlayMaxDim^2 x 4 bytes

// Placement of one overlay for one frame. tdx/tdy > 0 repeat the image with that
// period from (x, y) to the right and downwards (tiled watermark).
struct OverlayParams {
    int32_t on, x, y, tdx, tdy, w, h, pad;
};

SK_HD uint32_t overlay_blend(uint32_t p, const uint8_t* s) {
    const uint32_t a = s[3];
    if (!a) return p;
    uint32_t out = p & 0xff000000u;
    for (int c = 0; c < 3; c++) {
        const uint32_t d = (p >> (8 * c)) & 255u;
        out |= (uint32_t)(uint8_t)(s[c] + (d * (255u - a) + 127u) / 255u) << (8 * c);
    }
    return out;
}

// Pixel (x, y) of the picture after the overlays of `op` (images `img[slot]`).
SK_HD uint32_t overlay_px(uint32_t p, int x, int y, const OverlayParams* op, const uint8_t* const* img) {
    for (int k = 0; k < kOverlaySlots; k++) {
        const OverlayParams& o = op[k];
        if (!o.on) continue;
        int dx = x - o.x, dy = y - o.y;
        if (dx < 0 || dy < 0) continue;
        if (o.tdx > 0) dx %= o.tdx;
        if (o.tdy > 0) dy %= o.tdy;
        if (dx >= o.w || dy >= o.h) continue;
        p = overlay_blend(p, img[k] + ((size_t)dy * o.w + dx) * 4);
    }
    return p;
}

}  // namespace sk
