// gfx950 kernels of the JPEG stripe encoder (pixelflux output_mode 0).
//
//   k_damage  per-stripe BGRx compare against the previous frame (all 4 bytes,
//             like the CPU memcmp; 16-byte loads, one plain store per workgroup)
//   k_blocks  evaluates the per-stripe send / paint-over plan (same function as
//             the CPU backend) in every workgroup, so a frame needs no
//             cross-workgroup sync and a single host sync;
//             then one 64-lane wave per 8x8 block: BGRx -> Y / 2x2-averaged Cb,Cr,
//             separable integer FDCT through LDS (lane = coefficient), exact
//             rounding quantisation (32-bit division), zig-zag permute via LDS,
//             AC Huffman bit count with a ballot of non-zero lanes (run length =
//             distance to the previous set bit, no serial scan)
//   k_scan    one workgroup per stripe: DC prediction in coding order, per-block
//             bit totals, block-wide prefix sum -> bit offset of every block;
//             clears the stripe's bit buffer
//   k_write   one wave per block again: every lane builds its own symbol string
//             (ZRLs + code + amplitude, DC on lane 0, EOB on lane 63), a wave
//             prefix sum places it, ds_or assembles the block in LDS and the wave
//             stores whole words (global atomics only on the two edge words)
//   k_ffcount / k_stuff  4 KiB tiles: per-tile 0xFF counts, then every tile
//             workgroup stuffs (0xFF -> 0xFF 0x00, 1-bit padding, EOI on the last
//             tile) into LDS and streams it to host-mapped memory with 16-byte
//             stores
//
// Bit-exact with the CPU reference (jpeg_cpu.cpp); the host prepends the
// JFIF header (it only depends on quality and stripe height).
#include "jpeg_gpu.h"

namespace sk {
namespace jpeg {
namespace gpu {

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_sum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
           __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

__device__ __forceinline__ int wave_incl_scan(int v) {
    int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o);
        if (l >= o) v += t;
    }
    return v;
}

// Exclusive block-wide scan for blockDim = 64 * NW; returns the block total in *total.
template <int NW>
__device__ __forceinline__ int block_excl_scan(int v, int* wave_tot, int* total) {
    const int w = threadIdx.x >> 6, l = lane_id();
    int inc = wave_incl_scan(v);
    if (l == 63) wave_tot[w] = inc;
    __syncthreads();
    if (w == 0) {
        int t = l < NW ? wave_tot[l] : 0;
        int ti = wave_incl_scan(t);
        if (l < NW) wave_tot[l] = ti - t;
        if (l == NW - 1) wave_tot[NW] = ti;
    }
    __syncthreads();
    int r = wave_tot[w] + inc - v;
    *total = wave_tot[NW];
    __syncthreads();
    return r;
}

__device__ __forceinline__ int category(int v) {
    unsigned a = (unsigned)(v < 0 ? -v : v);
    return a ? 32 - __clz(a) : 0;
}

__device__ __forceinline__ int stripe_mcu_rows(const JpegArgs& a, int s) {
    int h = a.H - s * a.stripe_h;
    h = h < a.stripe_h ? h : a.stripe_h;
    return (h + 15) >> 4;
}

// XCD-aware bijective remap of a linear workgroup id (8 XCDs, round-robin).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    int q = nwg / 8, r = nwg % 8;
    int xcd = orig % 8;
    int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + orig / 8;
}

__device__ __forceinline__ void load_tables(const JpegTables* src, JpegTables* dst) {
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(dst);
    for (int i = threadIdx.x; i < (int)(sizeof(JpegTables) / 4); i += blockDim.x) d[i] = s[i];
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_damage(JpegArgs a) {
    const int s = blockIdx.y;
    if (s == 0 && blockIdx.x == 0 && threadIdx.x == 0) *a.key_now = *a.key_seq;  // one PCIe read per frame
    const int y0 = s * a.stripe_h;
    int h = a.H - y0;
    h = h < a.stripe_h ? h : a.stripe_h;
    bool diff = false;
    const bool vec = (a.stride % 16) == 0 && (a.W % 4) == 0;
    for (int r = blockIdx.x; r < h; r += gridDim.x) {
        const size_t row = (size_t)(y0 + r) * a.stride;
        if (vec) {
            const uint4* c = reinterpret_cast<const uint4*>(a.cur + row);
            const uint4* p = reinterpret_cast<const uint4*>(a.prev + row);
            for (int i = threadIdx.x; i < a.W / 4; i += blockDim.x) {
                uint4 x = c[i], y = p[i];
                diff |= ((x.x ^ y.x) | (x.y ^ y.y) | (x.z ^ y.z) | (x.w ^ y.w)) != 0u;
            }
        } else {
            const uint32_t* c = reinterpret_cast<const uint32_t*>(a.cur + row);
            const uint32_t* p = reinterpret_cast<const uint32_t*>(a.prev + row);
            for (int i = threadIdx.x; i < a.W; i += blockDim.x) diff |= c[i] != p[i];
        }
    }
    // one plain store per workgroup; visibility to k_blocks comes from the kernel boundary
    if (__syncthreads_or(diff) && threadIdx.x == 0) a.dirty_in[s] = 1;
}

// Stripe plan for this frame, evaluated identically by every workgroup of the
// stripe (same inputs); workgroup 0 publishes the result.
__device__ __forceinline__ int plan_stripe(const JpegArgs& a, int s, bool publish) {
    JpegStripeState S = a.state_in[s];
    const int key = *a.key_now;
    if (S.key_seq != key) {
        S.need_send = 1;
        S.key_seq = key;
    }
    const int act = jpeg_plan_stripe(S, a.dirty_in[s] != 0, a.use_paint_over, a.paint_over_trigger);
    if (publish) {
        a.state_out[s] = S;
        a.action[s] = act;
        a.host_action[s] = act;
        if (act < 0) a.host_size[s] = 0;
        a.dirty_out[s] = 0;  // next frame's k_damage target
    }
    return act;
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_blocks(JpegArgs a) {
    __shared__ int sC[64];
    __shared__ int sInv[64];
    __shared__ JpegTables sT;
    __shared__ int sPix[4][64];
    __shared__ int sTmp[4][64];
    __shared__ int sZz[4][64];
    const int s = blockIdx.y;
    const int act = plan_stripe(a, s, blockIdx.x == 0 && threadIdx.x == 0);
    if (act < 0) return;
    const int tid = threadIdx.x;
    if (tid < 64) {
        sC[tid] = JPEG_DCT_C[tid >> 3][tid & 7];
        sInv[JPEG_ZIGZAG[tid]] = tid;
    }
    load_tables(&a.tabs[act], &sT);
    __syncthreads();
    const int w = tid >> 6, l = lane_id();
    const int nblk = stripe_mcu_rows(a, s) * a.mcu_w * 6;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int mcu = wg * 4 + w;  // one MCU (6 blocks) per wave: tables loaded once per 24 blocks
    if (mcu * 6 >= nblk) return;  // whole wave leaves; no block barrier follows
    for (int b = 0; b < 6; b++) {
    const int blk = mcu * 6 + b;
    const int my = mcu / a.mcu_w, mx = mcu - my * a.mcu_w;
    const int y0 = s * a.stripe_h;
    const int yy = l >> 3, xx = l & 7;
    int val;
    if (b < 4) {
        int py = sk_min(y0 + my * 16 + (b >> 1) * 8 + yy, a.H - 1);
        int px = sk_min(mx * 16 + (b & 1) * 8 + xx, a.W - 1);
        uint32_t p = *reinterpret_cast<const uint32_t*>(a.cur + (size_t)py * a.stride + 4 * px);
        int Y, cb, cr;
        rgb_to_ycc((p >> 16) & 255, (p >> 8) & 255, p & 255, &Y, &cb, &cr);
        val = sk_clip255(Y);
    } else {
        int qy = my * 8 + yy, qx = mx * 8 + xx;
        int rs = 0, gs = 0, bs = 0;
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int i = 0; i < 2; i++) {
                int py = sk_min(y0 + 2 * qy + j, a.H - 1), px = sk_min(2 * qx + i, a.W - 1);
                uint32_t p = *reinterpret_cast<const uint32_t*>(a.cur + (size_t)py * a.stride + 4 * px);
                rs += (p >> 16) & 255;
                gs += (p >> 8) & 255;
                bs += p & 255;
            }
        int Y, cb, cr;
        rgb_to_ycc((rs + 2) >> 2, (gs + 2) >> 2, (bs + 2) >> 2, &Y, &cb, &cr);
        val = sk_clip255(b == 4 ? cb : cr);
    }
    sPix[w][l] = val - 128;
    wave_sync();
    {   // row pass: lane (y, u)
        const int y = l >> 3, u = l & 7;
        int acc = 0;
#pragma unroll
        for (int x = 0; x < 8; x++) acc += sPix[w][y * 8 + x] * sC[u * 8 + x];
        sTmp[w][y * 8 + u] = (acc + 32) >> 6;
    }
    wave_sync();
    const int c = b < 4 ? 0 : 1;
    {   // column pass: lane (v, u) -> quantise -> zig-zag position
        const int v = l >> 3, u = l & 7;
        int acc = 0;
#pragma unroll
        for (int y = 0; y < 8; y++) acc += sC[v * 8 + y] * sTmp[w][y * 8 + u];
        const unsigned den = (unsigned)sT.q[c][l] << 18;
        const unsigned n = (unsigned)(acc < 0 ? -acc : acc);
        const int lv = (int)((n + (den >> 1)) / den);
        sZz[w][sInv[l]] = acc < 0 ? -lv : lv;
    }
    wave_sync();
    const int zz = sZz[w][l];
    const size_t gblk = (size_t)s * a.blocks_per_stripe + blk;
    a.coef[gblk * 64 + l] = (int16_t)zz;
    // AC bit count: run = distance to the previous non-zero AC lane
    const unsigned long long mask = __ballot(l > 0 && zz != 0);
    int bits = 0;
    if (l > 0 && zz != 0) {
        unsigned long long below = mask & ((1ull << l) - 1ull);
        int prev = below ? 63 - __clzll(below) : 0;
        int run = l - prev - 1;
        int cat = category(zz);
        bits = (run >> 4) * sT.ac_len[c][0xF0] + sT.ac_len[c][((run & 15) << 4) | cat] + cat;
    }
    if (l == 63 && !((mask >> 63) & 1ull)) bits += sT.ac_len[c][0x00];
    const int total = wave_sum(bits);
    if (l == 0) {
        a.ac_bits[gblk] = total;
        a.dc[gblk] = (int16_t)zz;
    }
    }
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_scan(JpegArgs a) {
    __shared__ int wave_tot[17];
    __shared__ int sh_total;
    const int s = blockIdx.x, tid = threadIdx.x;
    const int act = a.action[s];
    if (act < 0) {
        if (tid == 0) a.stripe_bits[s] = 0;
        return;
    }
    const JpegTables& T = a.tabs[act];
    const int nblk = stripe_mcu_rows(a, s) * a.mcu_w * 6;
    const size_t base = (size_t)s * a.blocks_per_stripe;
    const int per = (nblk + 1023) / 1024;
    const int b0 = sk_min(nblk, tid * per), b1 = sk_min(nblk, b0 + per);
    int local = 0;
    for (int blk = b0; blk < b1; blk++) {
        const int mcu = blk / 6, b = blk - mcu * 6;
        int pred = -1;
        if (b >= 1 && b <= 3) pred = blk - 1;
        else if (b == 0) pred = mcu > 0 ? blk - 3 : -1;
        else pred = mcu > 0 ? blk - 6 : -1;
        const int diff = a.dc[base + blk] - (pred >= 0 ? a.dc[base + pred] : 0);
        a.dcdiff[base + blk] = (int16_t)diff;
        const int c = b < 4 ? 0 : 1;
        const int cat = category(diff);
        const int tot = a.ac_bits[base + blk] + T.dc_len[c][cat] + cat;
        a.ac_bits[base + blk] = tot;
        local += tot;
    }
    int total;
    int off = block_excl_scan<16>(local, wave_tot, &total);
    for (int blk = b0; blk < b1; blk++) {
        a.blk_off[base + blk] = off;
        off += a.ac_bits[base + blk];
    }
    if (tid == 0) {
        a.stripe_bits[s] = total;
        sh_total = total;
    }
    __syncthreads();
    uint32_t* buf = a.bits + (size_t)s * a.bits_slot_words;
    const int words = sk_min(a.bits_slot_words, (sh_total >> 5) + 2);
    for (int i = tid; i < words; i += 1024) buf[i] = 0;
}

// ---------------------------------------------------------------------------
__device__ __forceinline__ void put_bits(uint32_t* buf, int pos, unsigned long long acc, int n) {
    if (n <= 0) return;
    const unsigned long long v = acc << (64 - n);
    const int wi = pos >> 5, o = pos & 31;
    const uint32_t hi = (uint32_t)(v >> 32), lo = (uint32_t)v;
    const uint32_t x0 = hi >> o;
    const uint32_t x1 = o ? (hi << (32 - o)) | (lo >> o) : lo;
    const uint32_t x2 = o ? lo << (32 - o) : 0u;
    if (x0) atomicOr(&buf[wi], x0);
    if (n + o > 32 && x1) atomicOr(&buf[wi + 1], x1);
    if (n + o > 64 && x2) atomicOr(&buf[wi + 2], x2);
}

__global__ __launch_bounds__(256) void k_write(JpegArgs a) {
    __shared__ JpegTables sT;
    __shared__ uint32_t sBits[4][kBlockWords];
    const int s = blockIdx.y;
    const int act = a.action[s];
    if (act < 0) return;
    load_tables(&a.tabs[act], &sT);
    __syncthreads();
    const int w = threadIdx.x >> 6, l = lane_id();
    const int nblk = stripe_mcu_rows(a, s) * a.mcu_w * 6;
    const int wg = xcd_remap(blockIdx.x, gridDim.x);
    const int mcu = wg * 4 + w;
    if (mcu * 6 >= nblk) return;
    for (int b = 0; b < 6; b++) {
    const int blk = mcu * 6 + b;
    const int c = b < 4 ? 0 : 1;
    const size_t gblk = (size_t)s * a.blocks_per_stripe + blk;
    const int zz = a.coef[gblk * 64 + l];
    wave_sync();  // previous block's LDS words have been stored
    if (l < kBlockWords) sBits[w][l] = 0u;
    const unsigned long long mask = __ballot(l > 0 && zz != 0);
    unsigned long long acc = 0;
    int n = 0;
    if (l == 0) {
        const int diff = a.dcdiff[gblk];
        const int cat = category(diff);
        acc = sT.dc_code[c][cat];
        n = sT.dc_len[c][cat];
        if (cat) {
            acc = (acc << cat) | jpeg_value_bits(diff, cat);
            n += cat;
        }
    } else if (zz != 0) {
        unsigned long long below = mask & ((1ull << l) - 1ull);
        int prev = below ? 63 - __clzll(below) : 0;
        int run = l - prev - 1;
        const int lz = sT.ac_len[c][0xF0];
        for (; run > 15; run -= 16) {
            acc = (acc << lz) | sT.ac_code[c][0xF0];
            n += lz;
        }
        const int cat = category(zz);
        const int rs = (run << 4) | cat;
        acc = (acc << sT.ac_len[c][rs]) | sT.ac_code[c][rs];
        n += sT.ac_len[c][rs];
        acc = (acc << cat) | jpeg_value_bits(zz, cat);
        n += cat;
    }
    if (l == 63 && !((mask >> 63) & 1ull)) {
        acc = (acc << sT.ac_len[c][0]) | sT.ac_code[c][0];
        n += sT.ac_len[c][0];
    }
    const int off = a.blk_off[gblk];
    const int bit0 = off & 31;
    const int incl = wave_incl_scan(n);
    const int total = __builtin_amdgcn_readlane(incl, 63);
    wave_sync();
    put_bits(sBits[w], bit0 + incl - n, acc, n);  // ds_or_b32 into the wave's LDS block buffer
    wave_sync();
    const int nwords = (bit0 + total + 31) >> 5;
    if (l < nwords) {
        uint32_t* dst = a.bits + (size_t)s * a.bits_slot_words + (off >> 5);
        const uint32_t v = sBits[w][l];
        if (l == 0 || l == nwords - 1) {
            if (v) atomicOr(&dst[l], v);  // edge words are shared with the neighbour blocks
        } else {
            dst[l] = v;
        }
    }
    }
}

// ---------------------------------------------------------------------------
// Byte i of a stripe's entropy segment with the final partial byte padded by 1s.
__device__ __forceinline__ uint8_t seg_byte(uint32_t word, int j, int i, int n, int rem) {
    uint8_t v = (uint8_t)(word >> (24 - 8 * j));
    if (i == n - 1 && rem) v |= (uint8_t)((1u << (8 - rem)) - 1u);
    return v;
}

__global__ __launch_bounds__(256) void k_ffcount(JpegArgs a) {
    __shared__ int red[4];
    const int s = blockIdx.y, t = blockIdx.x;
    if (a.action[s] < 0) return;
    const int nbits = a.stripe_bits[s];
    const int n = (nbits + 7) >> 3, rem = nbits & 7;
    const int t0 = t * kTileBytes;
    if (t0 >= n) return;
    const uint32_t* buf = a.bits + (size_t)s * a.bits_slot_words;
    const int i0 = t0 + threadIdx.x * 16;
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int iq = i0 + 4 * q;
        if (iq >= n) break;
        const uint32_t word = buf[iq >> 2];
#pragma unroll
        for (int j = 0; j < 4; j++) cnt += (iq + j < n) && seg_byte(word, j, iq + j, n, rem) == 0xFF;
    }
    cnt = wave_sum(cnt);
    if (lane_id() == 0) red[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) a.tile_ff[s * a.max_tiles + t] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void k_stuff(JpegArgs a) {
    __shared__ int wave_tot[5];
    __shared__ int sh_prefix;
    __shared__ uint8_t sOut[2 * kTileBytes + 16];
    const int s = blockIdx.y, t = blockIdx.x, tid = threadIdx.x;
    if (a.action[s] < 0) return;
    const int nbits = a.stripe_bits[s];
    const int n = (nbits + 7) >> 3, rem = nbits & 7;
    const int t0 = t * kTileBytes;
    if (t0 >= n) return;
    if (tid < 64) {  // 0xFF count of all earlier tiles of this stripe
        int p = 0;
        for (int k = tid; k < t; k += 64) p += a.tile_ff[s * a.max_tiles + k];
        p = wave_sum(p);
        if (tid == 0) sh_prefix = p;
    }
    const uint32_t* buf = a.bits + (size_t)s * a.bits_slot_words;
    const int i0 = t0 + tid * 16;
    uint8_t by[16];
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int iq = i0 + 4 * q;
        const uint32_t word = iq < n ? buf[iq >> 2] : 0u;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            by[4 * q + j] = seg_byte(word, j, iq + j, n, rem);
            cnt += (iq + j < n) && by[4 * q + j] == 0xFF;
        }
    }
    int tile_ff;
    const int ex = block_excl_scan<4>(cnt, wave_tot, &tile_ff);
    int o = tid * 16 + ex;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        if (i0 + k < n) {
            sOut[o++] = by[k];
            if (by[k] == 0xFF) sOut[o++] = 0x00;
        }
    }
    const int in_len = min(n - t0, kTileBytes);
    const bool last = t0 + kTileBytes >= n;
    int len = in_len + tile_ff;
    if (last && tid == 0) {
        sOut[len] = 0xFF;
        sOut[len + 1] = 0xD9;
    }
    __syncthreads();
    if (last) len += 2;
    const int g0 = t0 + sh_prefix;  // output position inside the stripe slot
    uint8_t* dst = a.host_out + (size_t)s * a.out_slot;
    const int head = min(len, (16 - (g0 & 15)) & 15);
    if (tid < head) dst[g0 + tid] = sOut[tid];
    const int nvec = (len - head) >> 4;
    for (int v = tid; v < nvec; v += 256) {
        const uint8_t* p = sOut + head + 16 * v;
        uint4 x;
        x.x = p[0] | (p[1] << 8) | (p[2] << 16) | ((uint32_t)p[3] << 24);
        x.y = p[4] | (p[5] << 8) | (p[6] << 16) | ((uint32_t)p[7] << 24);
        x.z = p[8] | (p[9] << 8) | (p[10] << 16) | ((uint32_t)p[11] << 24);
        x.w = p[12] | (p[13] << 8) | (p[14] << 16) | ((uint32_t)p[15] << 24);
        *reinterpret_cast<uint4*>(dst + g0 + head + 16 * v) = x;
    }
    const int tail0 = head + 16 * nvec;
    if (tid < len - tail0) dst[g0 + tail0 + tid] = sOut[tail0 + tid];
    if (last && tid == 0) a.host_size[s] = n + sh_prefix + tile_ff + 2;
}

// ---------------------------------------------------------------------------
void launch_frame(const JpegArgs& a, hipStream_t st) {
    const int wgs = (a.blocks_per_stripe + 23) / 24;  // 4 waves x 1 MCU
    hipLaunchKernelGGL(k_damage, dim3(a.stripe_h, a.num_stripes), dim3(256), 0, st, a);  // 1 row / WG
    hipLaunchKernelGGL(k_blocks, dim3(wgs, a.num_stripes), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_scan, dim3(a.num_stripes), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(k_write, dim3(wgs, a.num_stripes), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_ffcount, dim3(a.max_tiles, a.num_stripes), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_stuff, dim3(a.max_tiles, a.num_stripes), dim3(256), 0, st, a);
}

}  // namespace gpu
}  // namespace jpeg
}  // namespace sk
