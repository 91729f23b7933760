// Shared host/device helpers for the selkies-mi355x native codec core.
//
// Every function tagged SK_HD is compiled twice: once for the host (the CPU
// reference encoder, used for `use_cpu` and as the bit-exact golden model in
// tests) and once for gfx950 (the HIP kernels). Integer-only math keeps the two
// builds bit-identical.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define SK_HD __host__ __device__ __forceinline__
#else
#define SK_HD inline
#endif

// Constant tables: device pass puts them in __constant__, host pass in .rodata.
#if defined(__HIP_DEVICE_COMPILE__)
#define SK_TABLE __constant__ static const
#else
#define SK_TABLE static const
#endif

SK_HD int sk_min(int a, int b) { return a < b ? a : b; }
SK_HD int sk_max(int a, int b) { return a > b ? a : b; }
SK_HD int sk_clip(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
SK_HD int sk_clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
SK_HD int sk_abs(int v) { return v < 0 ? -v : v; }
SK_HD int sk_median(int a, int b, int c) {
    int mx = sk_max(a, sk_max(b, c));
    int mn = sk_min(a, sk_min(b, c));
    return a + b + c - mx - mn;
}

// Number of bits of the Exp-Golomb ue(v) code for `v` (v >= 0).
SK_HD int sk_ue_bits(uint32_t v) {
    uint32_t x = v + 1;
    int n = 0;
    while (x >> n) n++;  // n = floor(log2(x)) + 1
    return 2 * n - 1;
}
SK_HD uint32_t sk_se_to_ue(int v) { return v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v); }
SK_HD int sk_se_bits(int v) { return sk_ue_bits(sk_se_to_ue(v)); }
