// Small kernels the runtime itself launches (not part of any codec pipeline).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sk {
// Adds 1 to one byte in each of `pages` 4 KiB pages of `buf` (a minimal dispatch
// that reads and writes device memory; used by warm_copy_engines()).
void launch_touch_pages(uint8_t* buf, int pages, hipStream_t s);
}  // namespace sk

namespace sk {
// BGRx / BGRA -> I420 (codec/color.h bgrx_quad_to_yuv: the encoders' K1 arithmetic), one
// thread per 2x2 quad; odd widths / heights repeat the last column / row.
// nv12: u receives the interleaved UV plane (Cb, Cr byte pairs).
void launch_bgrx_i420(const uint8_t* bgrx, int stride, int w, int h, int full_range, uint8_t* y, int ys,
                      uint8_t* u, int us, uint8_t* v, int vs, hipStream_t s, int nv12 = 0);
}  // namespace sk
