#include "runtime_kernels.h"

namespace sk {

__global__ void k_touch_pages(uint8_t* buf, int pages) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < pages) buf[(size_t)i * 4096] += 1;
}

void launch_touch_pages(uint8_t* buf, int pages, hipStream_t s) {
    hipLaunchKernelGGL(k_touch_pages, dim3((pages + 255) / 256), dim3(256), 0, s, buf, pages);
}

}  // namespace sk
