#include "runtime_kernels.h"
#include "../codec/color.h"

namespace sk {

__global__ void k_touch_pages(uint8_t* buf, int pages) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < pages) buf[(size_t)i * 4096] += 1;
}

void launch_touch_pages(uint8_t* buf, int pages, hipStream_t s) {
    hipLaunchKernelGGL(k_touch_pages, dim3((pages + 255) / 256), dim3(256), 0, s, buf, pages);
}

// nv12: u is the interleaved UV plane (Cb at 2 qx, Cr at 2 qx + 1), v unused.
__global__ __launch_bounds__(256) void k_bgrx_i420(const uint8_t* __restrict__ bgrx, int stride, int w, int h,
                                                   int full, uint8_t* __restrict__ y, int ys, uint8_t* __restrict__ u,
                                                   int us, uint8_t* __restrict__ v, int vs, int nv12) {
    const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    const int qx = blockIdx.x * 256 + threadIdx.x, qy = blockIdx.y;
    if (qx >= cw || qy >= ch) return;
    const int x0 = 2 * qx, x1 = min(x0 + 1, w - 1), y0 = 2 * qy, y1 = min(y0 + 1, h - 1);
    const uint8_t* r0 = bgrx + (size_t)y0 * stride;
    const uint8_t* r1 = bgrx + (size_t)y1 * stride;
    uint8_t yy[4], cb, cr;
    bgrx_quad_to_yuv(r0 + 4 * x0, r0 + 4 * x1, r1 + 4 * x0, r1 + 4 * x1, full, yy, &cb, &cr);
    y[(size_t)y0 * ys + x0] = yy[0];
    if (x1 != x0) y[(size_t)y0 * ys + x1] = yy[1];
    if (y1 != y0) {
        y[(size_t)y1 * ys + x0] = yy[2];
        if (x1 != x0) y[(size_t)y1 * ys + x1] = yy[3];
    }
    if (nv12) {
        u[(size_t)qy * us + 2 * qx] = cb;
        u[(size_t)qy * us + 2 * qx + 1] = cr;
    } else {
        u[(size_t)qy * us + qx] = cb;
        v[(size_t)qy * vs + qx] = cr;
    }
}

void launch_bgrx_i420(const uint8_t* bgrx, int stride, int w, int h, int full_range, uint8_t* y, int ys,
                      uint8_t* u, int us, uint8_t* v, int vs, hipStream_t s, int nv12) {
    const int cw = (w + 1) >> 1, ch = (h + 1) >> 1;
    hipLaunchKernelGGL(k_bgrx_i420, dim3((cw + 255) / 256, ch), dim3(256), 0, s, bgrx, stride, w, h, full_range, y,
                       ys, u, us, v, vs, nv12);
}

}  // namespace sk
