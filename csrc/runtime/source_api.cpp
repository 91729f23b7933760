// C ABI for the GStreamer elements (csrc/gst/gsthip.c): frame sources (hipximagesrc)
// and device memory (the "HIPMemory" GstAllocator). The plugin links only this ABI, so
// every HIP call of the elements runs inside libselkies_native.so.
//
//   sk_source_*  X11 MIT-SHM region grabber with XDamage rows (capture/x11_source.cpp,
//                the reference's ximagesrc, legacy/gstwebrtc_app.py:210-255) or the
//                synthetic desktop (headless hosts, capture/synthetic_source.cpp)
//   sk_dev_*     hipMalloc'd frames and copies between them and the host
#include "sk_api.h"
#include "encoder_iface.h"
#include "../capture/frame_source.h"
#include <hip/hip_runtime.h>
#include <string>
#include <vector>

namespace sk {
namespace {

struct Source {
    std::unique_ptr<FrameSource> src;
    int w = 0, h = 0;
    std::vector<int> rows;
};

bool hip_ok(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    set_last_error(std::string(what) + ": " + hipGetErrorString(e));
    return false;
}

}  // namespace
}  // namespace sk

using namespace sk;

extern "C" {

void* sk_source_open(int32_t kind, const char* display, int32_t x, int32_t y, int32_t w, int32_t h,
                     int32_t show_pointer, uint32_t seed) {
    if (w < 16 || h < 16) {
        set_last_error("source: size below 16x16");
        return nullptr;
    }
    Source* s = new Source;
    s->w = w;
    s->h = h;
    std::string err;
    if (kind == 0) {
        s->src = make_x11_source(display, x, y, w, h, show_pointer != 0, &err);
    } else if (kind >= 1 && kind <= 3) {
        s->src = make_synthetic_source(w, h, kind - 1, seed);
    } else {
        err = "source: kind must be 0 (x11), 1 (synthetic motion), 2 (synthetic desktop) or 3 (noise)";
    }
    if (!s->src) {
        set_last_error(err.empty() ? "source: open failed" : err);
        delete s;
        return nullptr;
    }
    return s;
}

const uint8_t* sk_source_grab(void* src, int32_t* stride, int32_t* rows, int32_t cap, int32_t* nrows) {
    Source* s = static_cast<Source*>(src);
    if (!s) return nullptr;
    int st = 0;
    const uint8_t* p = s->src->grab(&st);
    if (!p) {
        set_last_error("source: grab failed");
        return nullptr;
    }
    if (stride) *stride = st;
    if (nrows) {
        s->rows.clear();
        if (s->src->damage(&s->rows)) {
            const int n = (int)s->rows.size() / 2;
            for (int i = 0; i < n && i < cap && rows; i++) {
                rows[2 * i] = s->rows[2 * i];
                rows[2 * i + 1] = s->rows[2 * i + 1];
            }
            *nrows = n;
        } else {
            *nrows = -1;   // unknown: the whole frame counts as changed
        }
    }
    return p;
}

const char* sk_source_name(void* src) {
    Source* s = static_cast<Source*>(src);
    return s ? s->src->name() : "";
}

void sk_source_close(void* src) { delete static_cast<Source*>(src); }

void* sk_dev_alloc(int32_t device, int64_t bytes) {
    void* p = nullptr;
    if (!hip_ok(hipSetDevice(device), "hipSetDevice") || !hip_ok(hipMalloc(&p, (size_t)bytes), "hipMalloc"))
        return nullptr;
    return p;
}

void sk_dev_free(int32_t device, void* p) {
    if (!p) return;
    hipSetDevice(device);
    hipFree(p);
}

int sk_dev_copy(int32_t device, void* dst, const void* src, int64_t bytes, int32_t kind) {
    static const hipMemcpyKind kinds[4] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice,
                                           hipMemcpyDefault};
    if (kind < 0 || kind > 3) {
        set_last_error("sk_dev_copy: kind must be 0..3");
        return -1;
    }
    if (!hip_ok(hipSetDevice(device), "hipSetDevice")) return -1;
    // A device-to-device hipMemcpy may return before the copy lands, and the encoders'
    // streams are non-blocking (no implicit ordering with the null stream): wait for it,
    // so the caller can hand `dst` to any stream.
    return hip_ok(hipMemcpy(dst, src, (size_t)bytes, kinds[kind]), "hipMemcpy") &&
                   hip_ok(hipStreamSynchronize(nullptr), "hipStreamSynchronize") ? 0 : -1;
}

int sk_dev_copy2d(int32_t device, void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                  int64_t height, int32_t kind) {
    static const hipMemcpyKind kinds[4] = {hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice,
                                           hipMemcpyDefault};
    if (kind < 0 || kind > 3) {
        set_last_error("sk_dev_copy2d: kind must be 0..3");
        return -1;
    }
    if (!hip_ok(hipSetDevice(device), "hipSetDevice")) return -1;
    return hip_ok(hipMemcpy2D(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width, (size_t)height, kinds[kind]),
                  "hipMemcpy2D") && hip_ok(hipStreamSynchronize(nullptr), "hipStreamSynchronize") ? 0 : -1;
}

}  // extern "C"
