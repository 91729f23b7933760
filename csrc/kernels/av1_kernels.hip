// AV1 tile entropy coding on the GPU: one wave per tile runs the multi-symbol
// arithmetic coder of codec/av1_ec.h (the same SymbolCoder, device-side sink) over
// the tile's symbol list with the tile's own adaptive CDFs in LDS, then resolves
// the carries and writes the tile's bytes. AV1 tiles are independently decodable
// (separate CDF state and coder per tile), which is where the parallelism comes
// from; within a tile the coder is serial, like CABAC rows in hevc_kernels.hip.
// Byte-identical to the host SymbolEncoder (tests/test_av1_entropy.py, gpu-marked).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <vector>

#include "../codec/av1_ec.h"

namespace sk::av1 {

constexpr int kMaxCtx = 64;          // contexts per tile in LDS (17 x u16 each)

struct DevSink {
    uint16_t* p;
    int n;
    __device__ void push(uint16_t x) { p[n++] = x; }
};

// sym word: kind << 30 | ctx << 20 | value (kind 0 symbol, 1 bool, 2 literal of ctx bits)
__global__ __launch_bounds__(64) void k_av1_ec_tiles(const uint32_t* syms, const int32_t* sym_off,
                                                      const int32_t* sym_n, const uint16_t* cdf_init,
                                                      const int32_t* nsym, int n_ctx, int adapt,
                                                      uint16_t* chunks, uint8_t* out, int32_t* out_size) {
    __shared__ uint16_t cdf[kMaxCtx * 17];
    const int t = blockIdx.x;
    for (int i = threadIdx.x; i < n_ctx * 17; i += 64) cdf[i] = cdf_init[i];
    __syncthreads();
    if (threadIdx.x != 0) return;
    const int off = sym_off[t], n = sym_n[t];
    DevSink sink{chunks + 2 * (size_t)off + 8 * (size_t)t, 0};
    SymbolCoder<DevSink> coder(sink);
    for (int i = 0; i < n; i++) {
        const uint32_t w = syms[off + i];
        const int kind = (int)(w >> 30), c = (int)((w >> 20) & 1023u), v = (int)(w & 0xfffffu);
        if (kind == 1) {
            coder.bool_(v);
        } else if (kind == 2) {
            coder.literal((uint32_t)v, c);
        } else if (adapt) {
            coder.encode_adapt(cdf + c * 17, nsym[c], v);
        } else {
            coder.encode(cdf + c * 17, nsym[c], v);
        }
    }
    coder.finish();
    carry_bytes(sink.p, sink.n, out + 2 * (size_t)off + 8 * (size_t)t);
    out_size[t] = sink.n;
}

}  // namespace sk::av1

extern "C" {

// Test entry: codes `tiles` independent symbol lists on the GPU (device 0) and
// copies each tile's bytes to out + 2 * sym_off[t] + 8 * t, sizes to out_size.
// Returns 0, or < 0 on a HIP error / too many contexts.
int sk_av1_ec_encode_tiles_hip(const uint32_t* syms, const int32_t* sym_off, const int32_t* sym_n, int tiles,
                               const uint16_t* cdfs, const int32_t* nsym, int n_ctx, int adapt, uint8_t* out,
                               int32_t* out_size) {
    if (n_ctx > sk::av1::kMaxCtx || tiles <= 0) return -1;
    int total = 0;
    for (int t = 0; t < tiles; t++) {
        if (sym_off[t] < 0 || sym_n[t] < 0) return -1;
        total = sym_off[t] + sym_n[t] > total ? sym_off[t] + sym_n[t] : total;
    }
    for (int c = 0; c < n_ctx; c++) if (nsym[c] < 2 || nsym[c] > 16) return -1;
    for (int i = 0; i < total; i++) {   // the kernel indexes LDS by these: validate on the host
        const uint32_t w = syms[i];
        const int kind = (int)(w >> 30), c = (int)((w >> 20) & 1023u), v = (int)(w & 0xfffffu);
        if (kind == 0 && (c >= n_ctx || v >= nsym[c])) return -1;
        if (kind == 2 && (c < 1 || c > 20)) return -1;
        if (kind == 3) return -1;
    }
    const size_t out_cap = 2 * (size_t)total + 8 * (size_t)tiles;
    uint32_t* d_syms = nullptr;
    int32_t *d_off = nullptr, *d_n = nullptr, *d_nsym = nullptr, *d_size = nullptr;
    uint16_t *d_cdf = nullptr, *d_chunks = nullptr;
    uint8_t* d_out = nullptr;
    int rc = 0;
    auto ok = [&](hipError_t e) { if (e != hipSuccess && rc == 0) rc = -2; return rc == 0; };
    if (ok(hipMalloc(&d_syms, sizeof(uint32_t) * (total > 0 ? total : 1))) &&
        ok(hipMalloc(&d_off, sizeof(int32_t) * tiles)) && ok(hipMalloc(&d_n, sizeof(int32_t) * tiles)) &&
        ok(hipMalloc(&d_nsym, sizeof(int32_t) * n_ctx)) && ok(hipMalloc(&d_size, sizeof(int32_t) * tiles)) &&
        ok(hipMalloc(&d_cdf, sizeof(uint16_t) * 17 * n_ctx)) &&
        ok(hipMalloc(&d_chunks, sizeof(uint16_t) * out_cap)) && ok(hipMalloc(&d_out, out_cap)) &&
        ok(hipMemcpy(d_syms, syms, sizeof(uint32_t) * total, hipMemcpyHostToDevice)) &&
        ok(hipMemcpy(d_off, sym_off, sizeof(int32_t) * tiles, hipMemcpyHostToDevice)) &&
        ok(hipMemcpy(d_n, sym_n, sizeof(int32_t) * tiles, hipMemcpyHostToDevice)) &&
        ok(hipMemcpy(d_nsym, nsym, sizeof(int32_t) * n_ctx, hipMemcpyHostToDevice)) &&
        ok(hipMemcpy(d_cdf, cdfs, sizeof(uint16_t) * 17 * n_ctx, hipMemcpyHostToDevice))) {
        hipLaunchKernelGGL(sk::av1::k_av1_ec_tiles, dim3(tiles), dim3(64), 0, 0, d_syms, d_off, d_n, d_cdf, d_nsym,
                           n_ctx, adapt, d_chunks, d_out, d_size);
        if (ok(hipGetLastError()) && ok(hipDeviceSynchronize())) {
            ok(hipMemcpy(out, d_out, out_cap, hipMemcpyDeviceToHost));
            ok(hipMemcpy(out_size, d_size, sizeof(int32_t) * tiles, hipMemcpyDeviceToHost));
        }
    }
    hipFree(d_syms); hipFree(d_off); hipFree(d_n); hipFree(d_nsym); hipFree(d_size);
    hipFree(d_cdf); hipFree(d_chunks); hipFree(d_out);
    return rc;
}

}  // extern "C"
