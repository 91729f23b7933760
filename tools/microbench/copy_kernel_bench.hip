// Microbenchmark: cost of the first kernel after an H2D frame upload.
// Build: hipcc --offload-arch=gfx950 -O3 -o copy_kernel_bench copy_kernel_bench.hip
// Prints per-variant median microseconds (hipEvent timing).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <algorithm>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void k_cmp(const uint4* a, const uint4* b, int words_per_row, int rows_per_wg, int* flag) {
    bool d = false;
    int r0 = blockIdx.x * rows_per_wg;
    for (int r = r0; r < r0 + rows_per_wg; r++)
        for (int i = threadIdx.x; i < words_per_row; i += blockDim.x) {
            uint4 x = a[(size_t)r * words_per_row + i], y = b[(size_t)r * words_per_row + i];
            d |= ((x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w)) != 0u;
        }
    if (__syncthreads_or(d) && threadIdx.x == 0) flag[blockIdx.x & 15] = 1;
}

__global__ void k_nop(int* f) { if (threadIdx.x == 0 && blockIdx.x == 0) f[31] += 1; }

static float median(std::vector<float> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; }

int main() {
    const int W = 1920, H = 1088, rowb = W * 4, wpr = rowb / 16;
    const size_t bytes = (size_t)rowb * H;
    uint8_t *host, *a, *b;
    int* flag;
    CK(hipHostMalloc(&host, bytes, hipHostMallocDefault));
    for (size_t i = 0; i < bytes; i++) host[i] = (uint8_t)(i * 2654435761u >> 24);
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&flag, 256));
    CK(hipMemset(b, 1, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2)); CK(hipEventCreate(&e3));
    for (int rows_per_wg : {1, 4, 16}) {
        const int nwg = H / rows_per_wg;
        std::vector<float> tk, tc, tk_after, tk_after_nop;
        for (int it = 0; it < 60; it++) {
            // (1) kernel alone
            CK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(k_cmp, dim3(nwg), dim3(256), 0, s, (const uint4*)a, (const uint4*)b, wpr, rows_per_wg, flag);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t; CK(hipEventElapsedTime(&t, e0, e1)); if (it >= 10) tk.push_back(t * 1000);
            // (2) copy then kernel
            CK(hipEventRecord(e0, s));
            CK(hipMemcpyAsync(a, host, bytes, hipMemcpyHostToDevice, s));
            CK(hipEventRecord(e1, s));
            hipLaunchKernelGGL(k_cmp, dim3(nwg), dim3(256), 0, s, (const uint4*)a, (const uint4*)b, wpr, rows_per_wg, flag);
            CK(hipEventRecord(e2, s));
            CK(hipEventSynchronize(e2));
            float tcopy, tker; CK(hipEventElapsedTime(&tcopy, e0, e1)); CK(hipEventElapsedTime(&tker, e1, e2));
            if (it >= 10) { tc.push_back(tcopy * 1000); tk_after.push_back(tker * 1000); }
            // (3) copy, nop kernel, then kernel
            CK(hipMemcpyAsync(a, host, bytes, hipMemcpyHostToDevice, s));
            hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s, flag);
            CK(hipEventRecord(e1, s));
            hipLaunchKernelGGL(k_cmp, dim3(nwg), dim3(256), 0, s, (const uint4*)a, (const uint4*)b, wpr, rows_per_wg, flag);
            CK(hipEventRecord(e2, s));
            CK(hipEventSynchronize(e2));
            CK(hipEventElapsedTime(&tker, e1, e2));
            if (it >= 10) tk_after_nop.push_back(tker * 1000);
        }
        printf("rows/wg=%2d wgs=%4d | kernel alone %7.1f us | H2D %7.1f us (%.1f GB/s) | kernel after copy %7.1f us | "
               "kernel after copy+nop %7.1f us\n", rows_per_wg, nwg, median(tk), median(tc),
               bytes / (median(tc) * 1e3), median(tk_after), median(tk_after_nop));
    }
    return 0;
}
