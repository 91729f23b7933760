// Small kernels the runtime itself launches (not part of any codec pipeline).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sk {
// Adds 1 to one byte in each of `pages` 4 KiB pages of `buf` (a minimal dispatch
// that reads and writes device memory; used by warm_copy_engines()).
void launch_touch_pages(uint8_t* buf, int pages, hipStream_t s);
}  // namespace sk
