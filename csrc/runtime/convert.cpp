// Standalone BGRx -> I420 converter (sk_convert_*): the encoders' K1 colour arithmetic
// (codec/color.h) as its own object, for the GStreamer hipconvert element
// (csrc/gst/gsthip.c) and any caller that wants 4:2:0 planes without encoding.
// HIP path: pageable host frame -> device (async copy on the converter's stream),
// k_bgrx_i420, three planes back; CPU path: the same arithmetic on the host.
#include "sk_api.h"
#include "encoder_iface.h"
#include "../codec/color.h"
#include "../kernels/runtime_kernels.h"
#include <hip/hip_runtime.h>
#include <string>

namespace sk {
namespace {

struct Converter {
    int w = 0, h = 0, full = 0, backend = 0, device = 0;
    hipStream_t stream = nullptr;
    uint8_t* d_in = nullptr;   // w * 4 bytes per row
    uint8_t* d_out = nullptr;  // Y (w x h) + U + V ((w+1)/2 x (h+1)/2)
    ~Converter() {
        if (backend) {
            hipSetDevice(device);
            if (d_in) hipFree(d_in);
            if (d_out) hipFree(d_out);
            if (stream) hipStreamDestroy(stream);
        }
    }
};

bool ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    set_last_error(std::string("convert: ") + what + ": " + hipGetErrorString(e));
    return false;
}

}  // namespace
}  // namespace sk

using namespace sk;

extern "C" {

void* sk_convert_create(int w, int h, int full_range, int backend, int device) {
    if (w < 2 || h < 2) {
        set_last_error("convert: size below 2x2");
        return nullptr;
    }
    Converter* c = new Converter;
    c->w = w;
    c->h = h;
    c->full = full_range ? 1 : 0;
    c->backend = backend ? 1 : 0;
    c->device = device;
    if (c->backend) {
        const int cw = (w + 1) / 2, ch = (h + 1) / 2;
        if (!ok(hipSetDevice(device), "hipSetDevice") ||
            !ok(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "stream") ||
            !ok(hipMalloc(&c->d_in, (size_t)w * 4 * h), "hipMalloc") ||
            !ok(hipMalloc(&c->d_out, (size_t)w * h + 2 * (size_t)cw * ch), "hipMalloc")) {
            delete c;
            return nullptr;
        }
    }
    return c;
}

int sk_convert_run(void* conv, const uint8_t* bgrx, int32_t stride, uint8_t* y, int32_t ys, uint8_t* u, int32_t us,
                   uint8_t* v, int32_t vs) {
    Converter* c = static_cast<Converter*>(conv);
    if (!c || !bgrx || !y || !u || !v) return -1;
    const int w = c->w, h = c->h, cw = (w + 1) / 2, ch = (h + 1) / 2;
    if (!c->backend) {
        for (int qy = 0; qy < ch; qy++) {
            const int y0 = 2 * qy, y1 = y0 + 1 < h ? y0 + 1 : h - 1;
            const uint8_t* r0 = bgrx + (size_t)y0 * stride;
            const uint8_t* r1 = bgrx + (size_t)y1 * stride;
            for (int qx = 0; qx < cw; qx++) {
                const int x0 = 2 * qx, x1 = x0 + 1 < w ? x0 + 1 : w - 1;
                uint8_t q[4];
                bgrx_quad_to_yuv(r0 + 4 * x0, r0 + 4 * x1, r1 + 4 * x0, r1 + 4 * x1, c->full, q, &u[(size_t)qy * us + qx],
                                 &v[(size_t)qy * vs + qx]);
                y[(size_t)y0 * ys + x0] = q[0];
                if (x1 != x0) y[(size_t)y0 * ys + x1] = q[1];
                if (y1 != y0) {
                    y[(size_t)y1 * ys + x0] = q[2];
                    if (x1 != x0) y[(size_t)y1 * ys + x1] = q[3];
                }
            }
        }
        return 0;
    }
    if (!ok(hipSetDevice(c->device), "hipSetDevice")) return -1;
    uint8_t* dy = c->d_out;
    uint8_t* du = dy + (size_t)w * h;
    uint8_t* dv = du + (size_t)cw * ch;
    if (!ok(hipMemcpy2DAsync(c->d_in, (size_t)w * 4, bgrx, (size_t)stride, (size_t)w * 4, h, hipMemcpyHostToDevice,
                             c->stream), "upload"))
        return -1;
    launch_bgrx_i420(c->d_in, w * 4, w, h, c->full, dy, w, du, cw, dv, cw, c->stream);
    if (!ok(hipMemcpy2DAsync(y, (size_t)ys, dy, (size_t)w, (size_t)w, h, hipMemcpyDeviceToHost, c->stream), "Y") ||
        !ok(hipMemcpy2DAsync(u, (size_t)us, du, (size_t)cw, (size_t)cw, ch, hipMemcpyDeviceToHost, c->stream), "U") ||
        !ok(hipMemcpy2DAsync(v, (size_t)vs, dv, (size_t)cw, (size_t)cw, ch, hipMemcpyDeviceToHost, c->stream), "V"))
        return -1;
    return ok(hipStreamSynchronize(c->stream), "sync") ? 0 : -1;
}

void sk_convert_destroy(void* conv) { delete static_cast<Converter*>(conv); }

}  // extern "C"
