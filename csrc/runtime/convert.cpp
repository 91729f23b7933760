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
#include <string.h>
#include <string>
#include <vector>

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

// General form for the GStreamer elements: source BGRx in host or device memory, I420
// (fmt 1) or NV12 (fmt 2, u = interleaved UV plane) into host or device planes. Device
// pointers belong to the converter's device. The HIP path reads a device source in place
// and writes device planes in place (no host round trip: hipupload ! hipconvert !
// video/x-raw(memory:HIPMemory) ! hiph264enc keeps the frame on the GPU).
int sk_convert_run_ex(void* conv, const uint8_t* bgrx, int32_t stride, int32_t src_on_device, int32_t fmt,
                      uint8_t* y, int32_t ys, uint8_t* u, int32_t us, uint8_t* v, int32_t vs,
                      int32_t dst_on_device) {
    Converter* c = static_cast<Converter*>(conv);
    if (!c || !bgrx || !y || !u || (fmt == 1 && !v) || (fmt != 1 && fmt != 2)) {
        set_last_error("convert: bad arguments");
        return -1;
    }
    const int w = c->w, h = c->h, cw = (w + 1) / 2, ch = (h + 1) / 2;
    const bool nv12 = fmt == 2;
    if (!c->backend) {
        // CPU: stage device memory through the host, then the reference arithmetic
        std::vector<uint8_t> hin, hout;
        const uint8_t* src = bgrx;
        int sstride = stride;
        if (src_on_device) {
            hin.resize((size_t)w * 4 * h);
            if (!ok(hipMemcpy2D(hin.data(), (size_t)w * 4, bgrx, (size_t)stride, (size_t)w * 4, h,
                                hipMemcpyDeviceToHost), "download"))
                return -1;
            src = hin.data();
            sstride = w * 4;
        }
        hout.resize((size_t)w * h + 2 * (size_t)cw * ch);
        uint8_t* hy = hout.data();
        uint8_t* hu = hy + (size_t)w * h;
        uint8_t* hv = hu + (size_t)cw * ch;
        if (sk_convert_run(conv, src, sstride, hy, w, hu, cw, hv, cw) < 0) return -1;
        std::vector<uint8_t> uv;
        if (nv12) {
            uv.resize((size_t)2 * cw * ch);
            for (size_t i = 0; i < (size_t)cw * ch; i++) {
                uv[2 * i] = hu[i];
                uv[2 * i + 1] = hv[i];
            }
        }
        // host destinations with plain row copies (no HIP runtime needed on CPU-only hosts)
        auto put = [&](uint8_t* d, int dst, const uint8_t* sp, int sst, int bw, int bh, const char* what) {
            if (dst_on_device)
                return ok(hipMemcpy2D(d, (size_t)dst, sp, (size_t)sst, (size_t)bw, bh, hipMemcpyHostToDevice), what);
            for (int r = 0; r < bh; r++) memcpy(d + (size_t)r * dst, sp + (size_t)r * sst, (size_t)bw);
            return true;
        };
        bool good = put(y, ys, hy, w, w, h, "Y");
        if (nv12) good = good && put(u, us, uv.data(), 2 * cw, 2 * cw, ch, "UV");
        else good = good && put(u, us, hu, cw, cw, ch, "U") && put(v, vs, hv, cw, cw, ch, "V");
        return good ? 0 : -1;
    }
    if (!ok(hipSetDevice(c->device), "hipSetDevice")) return -1;
    const uint8_t* din = bgrx;
    int dstride = stride;
    if (!src_on_device) {
        if (!ok(hipMemcpy2DAsync(c->d_in, (size_t)w * 4, bgrx, (size_t)stride, (size_t)w * 4, h,
                                 hipMemcpyHostToDevice, c->stream), "upload"))
            return -1;
        din = c->d_in;
        dstride = w * 4;
    }
    uint8_t* dy = dst_on_device ? y : c->d_out;
    uint8_t* du = dst_on_device ? u : c->d_out + (size_t)w * h;
    uint8_t* dv = dst_on_device ? v : c->d_out + (size_t)w * h + (size_t)cw * ch;
    const int yst = dst_on_device ? ys : w, ust = dst_on_device ? us : (nv12 ? 2 * cw : cw),
              vst = dst_on_device ? vs : cw;
    launch_bgrx_i420(din, dstride, w, h, c->full, dy, yst, du, ust, dv, vst, c->stream, nv12 ? 1 : 0);
    if (!dst_on_device) {
        bool good = ok(hipMemcpy2DAsync(y, (size_t)ys, dy, (size_t)w, (size_t)w, h, hipMemcpyDeviceToHost, c->stream),
                       "Y");
        if (nv12) {
            good = good && ok(hipMemcpy2DAsync(u, (size_t)us, du, (size_t)2 * cw, (size_t)2 * cw, ch,
                                               hipMemcpyDeviceToHost, c->stream), "UV");
        } else {
            good = good &&
                   ok(hipMemcpy2DAsync(u, (size_t)us, du, (size_t)cw, (size_t)cw, ch, hipMemcpyDeviceToHost, c->stream),
                      "U") &&
                   ok(hipMemcpy2DAsync(v, (size_t)vs, dv, (size_t)cw, (size_t)cw, ch, hipMemcpyDeviceToHost, c->stream),
                      "V");
        }
        if (!good) return -1;
    }
    return ok(hipStreamSynchronize(c->stream), "sync") ? 0 : -1;
}

void sk_convert_destroy(void* conv) { delete static_cast<Converter*>(conv); }

}  // extern "C"
