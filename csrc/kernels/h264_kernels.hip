// gfx950 (CDNA4) kernels of the H.264 stripe encoder.
//
// Mapping (one 64-lane wavefront per macroblock):
//   luma   lane l -> 4x4 block b = l>>2 (luma4x4BlkIdx), row r = l&3, 4 pixels per lane
//   chroma lane l -> comp = (l>>4)&1, block = (l>>2)&3, row = l&3 (lanes 32..63 mirror 0..31)
// The 4x4 integer transforms run in-lane horizontally and across the 4 lanes of a
// quad vertically with DPP quad-permutes (no LDS round trip).
//
// Stages (all bit-exact with the CPU reference csrc/codec/h264_cpu.cpp):
//   k_convert_damage  K1+K3  BGRx -> NV12-planar YUV 4:2:0 + per-MB damage bits
//   k_me_mfma         K4a    exhaustive +-16 search: int8 MFMA cross-correlation (SSD)
//   k_motion_search   K4     candidate + diamond integer search, v_sad_u8
//   k_decide                 per-slice scene-cut decision
//   k_code_inter      K6     MC, transform, quant/decimation, QP escalation, recon
//   k_code_intra      K5+K6  Intra16x16 wavefront (one wave per MB row, lag 2)
//   k_cavlc           K8     per-MB CAVLC: lanes code residual blocks in parallel,
//                            bit offsets by wave prefix-sum, LDS atomicOr packing
//   k_slice_scan, k_mb_concat, k_ep_*   K9  slice header + MB offsets, MB bit
//                            concatenation, tile-parallel emulation prevention
//                            straight into host-mapped packet slots
//   k_commit                 MV-field update (+ plain reference copy when K7 is off)
//   k_deblock_prep, k_deblock  K7  in-loop deblocking rec -> ref (LDS-ring wavefront)
#include "h264_gpu.h"
#include "../codec/color.h"
#include "../codec/h264_mb.h"

namespace sk {
namespace h264 {
namespace gpu {

// ---------------------------------------------------------------------------
// wave helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Full-wave sum with DPP (quad swaps + row rotations) and 4 readlanes; every
// lane must be active. Result is wave-uniform.
__device__ __forceinline__ int wave_sum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    v += __builtin_amdgcn_mov_dpp(v, 0x124, 0xF, 0xF, false);  // row_ror:4
    v += __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);  // row_ror:8
    return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) +
           __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
}

// K5 sub-slices (h264_encoder.h intra_split): does slice t code as sub-slices, and how
// many NALs does it produce this frame (0: not coded).
__device__ __forceinline__ bool split_i(const FrameArgs& a, const SliceTask& t) {
    return a.nal_per_slice > 1 && intra_split(t, a.mb_w, a.deblock, a.intra4x4);
}
__device__ __forceinline__ int slice_nals(const FrameArgs& a, const SliceTask& t) {
    if (t.final_action == ACT_NONE) return 0;
    return split_i(a, t) ? intra_sub_count(t.num_rows * a.mb_w) : 1;
}
// RBSP of NAL j of slice s
__device__ __forceinline__ uint32_t* nal_rbsp(const FrameArgs& a, int s, int j) {
    return a.rbsp + (size_t)s * a.rbsp_slot_words + (size_t)j * a.sub_rbsp_words;
}

__device__ __forceinline__ int wave_incl_scan_max(int v) {
    int l = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o);
        if (l >= o) v = max(v, t);
    }
    return v;
}

// inclusive prefix sum across the wave
__device__ __forceinline__ int wave_incl_scan(int v) {
    int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int t = __shfl_up(v, o);
        if (l >= o) v += t;
    }
    return v;
}

// Copies the precomputed CAVLC tables (device memory) into LDS with dword loads.
__device__ __forceinline__ void load_cavlc_tables(CavlcTables& dst, const CavlcTables* src) {
    static_assert(sizeof(CavlcTables) % 4 == 0, "dword copy");
    const uint32_t* s = reinterpret_cast<const uint32_t*>(src);
    uint32_t* d = reinterpret_cast<uint32_t*>(&dst);
    for (int i = threadIdx.x; i < (int)(sizeof(CavlcTables) / 4); i += blockDim.x) d[i] = s[i];
}

// Exclusive block-wide scan for blockDim = 64 * NW; the block total goes to *total.
template <int NW>
__device__ __forceinline__ int block_excl_scan(int v, int* wave_tot, int* total) {
    const int w = threadIdx.x >> 6, l = lane_id();
    const int inc = wave_incl_scan(v);
    if (l == 63) wave_tot[w] = inc;
    __syncthreads();
    if (w == 0) {
        const int t = l < NW ? wave_tot[l] : 0;
        const int ti = wave_incl_scan(t);
        if (l < NW) wave_tot[l] = ti - t;
        if (l == NW - 1) wave_tot[NW] = ti;
    }
    __syncthreads();
    const int r = wave_tot[w] + inc - v;
    *total = wave_tot[NW];
    __syncthreads();
    return r;
}

template <int K>
__device__ __forceinline__ int quad_bcast(int v) {
    return __builtin_amdgcn_mov_dpp(v, K * 0x55, 0xF, 0xF, false);
}

// XCD-aware bijective block remap (8 XCDs, round-robin dispatch): consecutive
// logical blocks land on the same XCD so neighbouring macroblocks share L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
    int q = nwg / 8, r = nwg % 8;
    int xcd = orig % 8;
    int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + orig / 8;
}

// Forward core transform of one 4x4 block: each lane of the quad holds row r.
__device__ __forceinline__ void fwd4_quad(const int* x, int r, int* w) {
    int t[4];
    {
        int s03 = x[0] + x[3], d03 = x[0] - x[3], s12 = x[1] + x[2], d12 = x[1] - x[2];
        t[0] = s03 + s12;
        t[1] = 2 * d03 + d12;
        t[2] = s03 - s12;
        t[3] = d03 - 2 * d12;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int a = quad_bcast<0>(t[j]), b = quad_bcast<1>(t[j]), c = quad_bcast<2>(t[j]),
            d = quad_bcast<3>(t[j]);
        int s03 = a + d, d03 = a - d, s12 = b + c, d12 = b - c;
        int o0 = s03 + s12, o1 = 2 * d03 + d12, o2 = s03 - s12, o3 = d03 - 2 * d12;
        w[j] = r == 0 ? o0 : (r == 1 ? o1 : (r == 2 ? o2 : o3));
    }
}

// Inverse transform (8.5.12.2): rows in-lane, columns across the quad.
__device__ __forceinline__ void inv4_quad(const int* d, int r, int* res) {
    int f[4];
    {
        int e0 = d[0] + d[2], e1 = d[0] - d[2], e2 = (d[1] >> 1) - d[3], e3 = d[1] + (d[3] >> 1);
        f[0] = e0 + e3;
        f[1] = e1 + e2;
        f[2] = e1 - e2;
        f[3] = e0 - e3;
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        int f0 = quad_bcast<0>(f[j]), f1 = quad_bcast<1>(f[j]), f2 = quad_bcast<2>(f[j]),
            f3 = quad_bcast<3>(f[j]);
        int g0 = f0 + f2, g1 = f0 - f2, g2 = (f1 >> 1) - f3, g3 = f1 + (f3 >> 1);
        int o0 = g0 + g3, o1 = g1 + g2, o2 = g1 - g2, o3 = g0 - g3;
        int o = r == 0 ? o0 : (r == 1 ? o1 : (r == 2 ? o2 : o3));
        res[j] = (o + 32) >> 6;
    }
}

// Diagnostic stamp: wave 0 of block SK_STAMP_BLOCK records s_memtime at numbered points.
#ifndef SK_STAMP_BLOCK
#define SK_STAMP_BLOCK 0
#endif
#ifndef SK_STAMP_STEP0
#define SK_STAMP_STEP0 0   // first recorded step (64 steps are kept)
#endif
#ifdef SK_STAMPS
__device__ __forceinline__ void stamp(unsigned long long* dbg, int step, int point) {
    __builtin_amdgcn_sched_barrier(0);
    unsigned long long t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    if (dbg && blockIdx.x == SK_STAMP_BLOCK && threadIdx.x == 0 && (unsigned)(step - SK_STAMP_STEP0) < 64u)
        dbg[(step - SK_STAMP_STEP0) * 16 + point] = t;
}
#define STAMP(step, pt) stamp(a.dbg, step, pt)
#define STAMP_S(dbg, step, pt) stamp(dbg, step, pt)
#else
#define STAMP(step, pt)
#define STAMP_S(dbg, step, pt)
#endif

// Big-endian-in-word bit writer on a shared/global u32 buffer (atomicOr, so
// several lanes may write disjoint bit ranges concurrently).
struct AtomicBitWriter {
    uint32_t* buf;
    uint32_t pos;
    __device__ void put(uint32_t code, int len) {
        if (len <= 0) return;
        if (len < 32) code &= (1u << len) - 1u;
        uint32_t wi = pos >> 5, sh = pos & 31;
        if (sh + len <= 32) {
            atomicOr(&buf[wi], code << (32 - sh - len));
        } else {
            atomicOr(&buf[wi], code >> (sh + len - 32));
            atomicOr(&buf[wi + 1], code << (64 - sh - len));
        }
        pos += len;
    }
};

// Per-lane staging writer (the lane owns `buf`, zeroed): plain LDS read-modify-writes.
// Bits past `cap` are only counted (ovf): that lane then writes its block again at
// the final offset.
struct StageBitWriter {
    uint32_t* buf;
    uint32_t pos;
    uint32_t cap;
    bool ovf;
    __device__ void put(uint32_t code, int len) {
        if (len <= 0) return;
        if (pos + (uint32_t)len > cap) { ovf = true; pos += len; return; }
        if (len < 32) code &= (1u << len) - 1u;
        uint32_t wi = pos >> 5, sh = pos & 31;
        if (sh + len <= 32) {
            buf[wi] |= code << (32 - sh - len);
        } else {
            buf[wi] |= code >> (sh + len - 32);
            buf[wi + 1] |= code << (64 - sh - len);
        }
        pos += len;
    }
};

// ---------------------------------------------------------------------------
// K1 + K3: colour conversion and damage detection.
// Workgroup = 256 threads = one MB row segment of 16 MBs (256 x 16 pixels);
// thread = 8 x 2 pixels (4 chroma quads) with 16-byte BGRx loads. Per-MB dirty
// flags go to mb_dirty; the stripe flag is one plain store per workgroup into
// host-mapped memory (no same-line atomics, no device->host copy).
__device__ __forceinline__ uint32_t bgrx_px(const uint8_t* row, int x, int W) {
    return *reinterpret_cast<const uint32_t*>(row + 4 * sk_min(x, W - 1));
}

__global__ __launch_bounds__(256) void k_convert_damage(FrameArgs a) {
    __shared__ int mbd[16];
    const int t = threadIdx.x;
    if (t < 16) mbd[t] = 0;
    __syncthreads();
    const int item = t & 31, qr = t >> 5;          // 32 items across (8 px each), 8 quad rows
    const int mby = blockIdx.y, mbx0 = blockIdx.x * 16;
    const int x0 = mbx0 * 16 + item * 8;            // first pixel column of this item
    const int qy = mby * 8 + qr;
    bool diff = false;
    if (x0 < a.stride_y) {
        const int y0 = min(2 * qy, a.H - 1), y1 = min(2 * qy + 1, a.H - 1);
        const uint8_t* r0 = a.bgrx + (size_t)y0 * a.bgrx_stride;
        const uint8_t* r1 = a.bgrx + (size_t)y1 * a.bgrx_stride;
        uint32_t p0[8], p1[8];
        if (a.scaled) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int x = sk_min(x0 + i, a.W - 1);
                p0[i] = scale_fetch(a.bgrx, a.bgrx_stride, a.scale, x, y0);
                p1[i] = scale_fetch(a.bgrx, a.bgrx_stride, a.scale, x, y1);
            }
        } else if (x0 + 7 < a.W && (a.bgrx_stride & 15) == 0) {
            const uint4 a0 = *reinterpret_cast<const uint4*>(r0 + 4 * x0);
            const uint4 a1 = *reinterpret_cast<const uint4*>(r0 + 4 * x0 + 16);
            const uint4 b0 = *reinterpret_cast<const uint4*>(r1 + 4 * x0);
            const uint4 b1 = *reinterpret_cast<const uint4*>(r1 + 4 * x0 + 16);
            p0[0] = a0.x; p0[1] = a0.y; p0[2] = a0.z; p0[3] = a0.w;
            p0[4] = a1.x; p0[5] = a1.y; p0[6] = a1.z; p0[7] = a1.w;
            p1[0] = b0.x; p1[1] = b0.y; p1[2] = b0.z; p1[3] = b0.w;
            p1[4] = b1.x; p1[5] = b1.y; p1[6] = b1.z; p1[7] = b1.w;
        } else {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                p0[i] = bgrx_px(r0, x0 + i, a.W);
                p1[i] = bgrx_px(r1, x0 + i, a.W);
            }
        }
        {   // K12 watermark / K13 cursor, in picture coordinates (edge padding repeats x = W-1)
            const OverlayParams o0 = a.ov[0], o1 = a.ov[1];
            if (o0.on | o1.on) {
                const OverlayParams op[kOverlaySlots] = {o0, o1};
#pragma unroll
                for (int i = 0; i < 8; i++) {
                    const int x = sk_min(x0 + i, a.W - 1);
                    p0[i] = overlay_px(p0[i], x, y0, op, a.ov_img);
                    p1[i] = overlay_px(p1[i], x, y1, op, a.ov_img);
                }
            }
        }
        uint32_t ya[2] = {0, 0}, yb[2] = {0, 0}, cbw = 0, crw = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            uint8_t y[4], cb, cr;
            bgrx_quad_to_yuv((const uint8_t*)&p0[2 * q], (const uint8_t*)&p0[2 * q + 1], (const uint8_t*)&p1[2 * q],
                             (const uint8_t*)&p1[2 * q + 1], a.full_range, y, &cb, &cr);
            const int sh = 16 * (q & 1);
            ya[q >> 1] |= (uint32_t)(y[0] | (y[1] << 8)) << sh;
            yb[q >> 1] |= (uint32_t)(y[2] | (y[3] << 8)) << sh;
            cbw |= (uint32_t)cb << (8 * q);
            crw |= (uint32_t)cr << (8 * q);
        }
        const size_t oy = (size_t)(2 * qy) * a.stride_y + x0;
        const size_t oc = (size_t)qy * a.stride_c + x0 / 2;
        const uint2 pa = *reinterpret_cast<const uint2*>(a.prev.y + oy);
        const uint2 pb = *reinterpret_cast<const uint2*>(a.prev.y + oy + a.stride_y);
        const uint32_t pu = *reinterpret_cast<const uint32_t*>(a.prev.u + oc);
        const uint32_t pv = *reinterpret_cast<const uint32_t*>(a.prev.v + oc);
        diff = (pa.x != ya[0]) | (pa.y != ya[1]) | (pb.x != yb[0]) | (pb.y != yb[1]) | (pu != cbw) | (pv != crw);
        *reinterpret_cast<uint2*>(a.src.y + oy) = make_uint2(ya[0], ya[1]);
        *reinterpret_cast<uint2*>(a.src.y + oy + a.stride_y) = make_uint2(yb[0], yb[1]);
        *reinterpret_cast<uint32_t*>(a.src.u + oc) = cbw;
        *reinterpret_cast<uint32_t*>(a.src.v + oc) = crw;
    }
    if (diff || a.plan_ctl[1] == 0) mbd[item >> 1] = 1;   // 2 items per MB; first frame: all dirty
    __syncthreads();
    if (t < 16) {
        const int mbx = mbx0 + t;
        if (mbx < a.mb_w) a.mb_dirty[mby * a.mb_w + mbx] = (uint8_t)mbd[t];
    }
    if (__syncthreads_or(t < 16 && mbd[t] && mbx0 + t < a.mb_w) && t == 0)
        a.stripe_dirty[mby / a.rows_per_slice] = 1;
}

// K3 for planar 4:2:0 input (GStreamer NV12 / I420, h264_frame.h YuvInput): the staged
// planes are copied into the source planes with the edge padding of yuv_sample and
// compared with the previous source, in the thread layout of k_convert_damage (thread
// = 8 x 2 luma samples and their 4 x 1 chroma samples of each plane).
__global__ __launch_bounds__(256) void k_yuv_damage(FrameArgs a) {
    __shared__ int mbd[16];
    const int t = threadIdx.x;
    if (t < 16) mbd[t] = 0;
    __syncthreads();
    const int item = t & 31, qr = t >> 5;
    const int mby = blockIdx.y, mbx0 = blockIdx.x * 16;
    const int x0 = mbx0 * 16 + item * 8;
    const int qy = mby * 8 + qr;
    bool diff = false;
    if (x0 < a.stride_y) {
        const int W = a.W, H = a.H, cw = (W + 1) >> 1, ch = (H + 1) >> 1;
        const uint8_t* py = a.yuv;
        const uint8_t* pc = a.yuv + (size_t)W * H;
        const int y0 = min(2 * qy, H - 1), y1 = min(2 * qy + 1, H - 1), cy = min(qy, ch - 1);
        uint32_t ya[2] = {0, 0}, yb[2] = {0, 0}, cbw = 0, crw = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int x = min(x0 + i, W - 1);
            ya[i >> 2] |= (uint32_t)py[(size_t)y0 * W + x] << (8 * (i & 3));
            yb[i >> 2] |= (uint32_t)py[(size_t)y1 * W + x] << (8 * (i & 3));
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int cx = min((x0 >> 1) + q, cw - 1);
            uint32_t u, v;
            if (a.yuv_fmt == 2) {   // NV12: UV interleaved
                const uint8_t* r = pc + (size_t)cy * (2 * cw) + 2 * cx;
                u = r[0];
                v = r[1];
            } else {                // I420
                u = pc[(size_t)cy * cw + cx];
                v = pc[(size_t)cw * ch + (size_t)cy * cw + cx];
            }
            cbw |= u << (8 * q);
            crw |= v << (8 * q);
        }
        const size_t oy = (size_t)(2 * qy) * a.stride_y + x0;
        const size_t oc = (size_t)qy * a.stride_c + x0 / 2;
        const uint2 pa = *reinterpret_cast<const uint2*>(a.prev.y + oy);
        const uint2 pb = *reinterpret_cast<const uint2*>(a.prev.y + oy + a.stride_y);
        const uint32_t pu = *reinterpret_cast<const uint32_t*>(a.prev.u + oc);
        const uint32_t pv = *reinterpret_cast<const uint32_t*>(a.prev.v + oc);
        diff = (pa.x != ya[0]) | (pa.y != ya[1]) | (pb.x != yb[0]) | (pb.y != yb[1]) | (pu != cbw) | (pv != crw);
        *reinterpret_cast<uint2*>(a.src.y + oy) = make_uint2(ya[0], ya[1]);
        *reinterpret_cast<uint2*>(a.src.y + oy + a.stride_y) = make_uint2(yb[0], yb[1]);
        *reinterpret_cast<uint32_t*>(a.src.u + oc) = cbw;
        *reinterpret_cast<uint32_t*>(a.src.v + oc) = crw;
    }
    if (diff || a.plan_ctl[1] == 0) mbd[item >> 1] = 1;
    __syncthreads();
    if (t < 16) {
        const int mbx = mbx0 + t;
        if (mbx < a.mb_w) a.mb_dirty[mby * a.mb_w + mbx] = (uint8_t)mbd[t];
    }
    if (__syncthreads_or(t < 16 && mbd[t] && mbx0 + t < a.mb_w) && t == 0)
        a.stripe_dirty[mby / a.rows_per_slice] = 1;
}

// ---------------------------------------------------------------------------
// K4: integer motion search (one wave per MB).
__device__ __forceinline__ uint32_t load_ref4(const uint8_t* row, int x, int stride) {
    if (x >= 0 && x + 3 <= stride - 1) {
        int xa = x & ~3, sh = x & 3;
        uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + xa);
        if (sh == 0) return w0;
        uint32_t w1 = *reinterpret_cast<const uint32_t*>(row + xa + 4);
        return __builtin_amdgcn_alignbyte(w1, w0, sh);
    }
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) v |= (uint32_t)row[sk_clip(x + i, 0, stride - 1)] << (8 * i);
    return v;
}

__device__ __forceinline__ int me_sad(const FrameArgs& a, const uint8_t* refy, uint32_t sw, int mbx,
                                      int mby, int dx, int dy, int ylo, int yhi) {
    int l = lane_id();
    int row = l >> 2, col4 = (l & 3) * 4;
    int sy = sk_clip(mby * 16 + row + dy, ylo, yhi);
    uint32_t rw = load_ref4(refy + (size_t)sy * a.stride_y, mbx * 16 + col4 + dx, a.stride_y);
    return wave_sum((int)__builtin_amdgcn_sad_u8(sw, rw, 0u));
}

// Reference window cached in LDS for the diamond refinement: +-kWin pixels
// around the best predictor, 32 rows x 36 bytes (the extra word serves the
// aligned-pair read of the last unaligned column). Window bytes are produced
// by load_ref4, so every SAD is identical to the global-memory path.
constexpr int kWin = 8;
constexpr int kWinWords = 10;  // words per LDS row (40 B)

// This lane's 4-pixel share of win_sad (<= 1020, so two candidates pack into one
// 32-bit wave sum: 64 x 1020 < 65536).
__device__ __forceinline__ uint32_t win_sad_lane(const uint32_t* win, uint32_t sw, int ox, int oy) {
    const int l = lane_id();
    const int row = l >> 2, col4 = (l & 3) * 4;
    const int bc = col4 + ox + kWin;
    const uint32_t* w = win + (row + oy + kWin) * kWinWords + (bc >> 2);
    const int sh = bc & 3;
    const uint32_t rw = sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
    return __builtin_amdgcn_sad_u8(sw, rw, 0u);
}

__device__ __forceinline__ int win_sad(const uint32_t* win, uint32_t sw, int ox, int oy) {
    const int l = lane_id();
    const int row = l >> 2, col4 = (l & 3) * 4;
    const int bc = col4 + ox + kWin;              // byte column inside the window row
    const uint32_t* w = win + (row + oy + kWin) * kWinWords + (bc >> 2);
    const int sh = bc & 3;
    const uint32_t rw = sh ? __builtin_amdgcn_alignbyte(w[1], w[0], sh) : w[0];
    return wave_sum((int)__builtin_amdgcn_sad_u8(sw, rw, 0u));
}

// sum |Y - mean| of a 16x16 MB, one wave (lane: 4 samples of row l / 4)
__device__ __forceinline__ int mb_activity(uint32_t sw) {
    const int psum = (int)(sw & 255) + (int)((sw >> 8) & 255) + (int)((sw >> 16) & 255) + (int)(sw >> 24);
    const int mean = (wave_sum(psum) + 128) >> 8;
    int dev = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) dev += sk_abs((int)((sw >> (8 * i)) & 255) - mean);
    return wave_sum(dev);
}

__global__ __launch_bounds__(64) void k_motion_search(FrameArgs a) {
    __shared__ uint32_t win[32 * kWinWords];
    int nmb = a.mb_w * a.mb_h;
    int idx = xcd_remap(blockIdx.x, gridDim.x);
    if (idx >= nmb) return;
    int mbx = idx % a.mb_w, mby = idx / a.mb_w;
    int s = mby / a.rows_per_slice;
    const SliceTask t = a.tasks[s];
    if (t.action != ACT_P && t.action != ACT_I) return;
    int l = lane_id();
    int row = l >> 2, col4 = (l & 3) * 4;
    uint32_t sw = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)(mby * 16 + row) * a.stride_y +
                                                     mbx * 16 + col4);
    if (t.action == ACT_I) {   // planned key frame: only the activity (K10's intra complexity)
        const int dev = mb_activity(sw);
        if (l == 0) a.me[idx] = MeResult{0, 0, 0, dev, 0, 0, 0};
        return;
    }
    int ylo = t.pic_row0 * 16, yhi = (t.pic_row0 + t.pic_rows) * 16 - 1;
    const int lam = lambda_for_qp(rc_me_qp(*a.rc, t.qp));
    const int R = a.me_range;
    // candidates (same order as the CPU reference)
    int cx[7], cy[7], n = 0;
    cx[0] = 0; cy[0] = 0; n = 1;
    auto add = [&](int ox, int oy) {
        int j = oy * a.mb_w + ox;
        cx[n] = sk_clip(a.mvfield[2 * j], -R, R);
        cy[n] = sk_clip(a.mvfield[2 * j + 1], -R, R);
        n++;
    };
    add(mbx, mby);
    if (mbx > 0) add(mbx - 1, mby);
    if (mbx + 1 < a.mb_w) add(mbx + 1, mby);
    if (mby - 1 >= t.pic_row0) add(mbx, mby - 1);
    if (mby + 1 < t.pic_row0 + t.pic_rows) add(mbx, mby + 1);
    if (a.me_full && a.mb_dirty[idx]) {   // K4a winner (k_me_mfma)
        cx[n] = sk_clip(a.fs_mv[2 * idx], -R, R);
        cy[n] = sk_clip(a.fs_mv[2 * idx + 1], -R, R);
        n++;
    }
    int bx = 0, by = 0;
    int bsad = me_sad(a, a.ref.y, sw, mbx, mby, 0, 0, ylo, yhi);
    int bcost = bsad + lam * (sk_se_bits(0) + sk_se_bits(0));
    for (int i = 1; i < n; i++) {
        int sd = me_sad(a, a.ref.y, sw, mbx, mby, cx[i], cy[i], ylo, yhi);
        int c = sd + lam * (sk_se_bits(4 * cx[i]) + sk_se_bits(4 * cy[i]));
        if (c < bcost) { bcost = c; bx = cx[i]; by = cy[i]; bsad = sd; }
    }
    // fill the LDS window around the best predictor: lane -> (row l>>1, 5 words)
    const int cx0 = bx, cy0 = by;
    {
        const int r = l >> 1, h = l & 1;
        const int y = sk_clip(mby * 16 + cy0 - kWin + r, ylo, yhi);
        const uint8_t* rowp = a.ref.y + (size_t)y * a.stride_y;
        const int x0 = mbx * 16 + cx0 - kWin + 16 * h;
#pragma unroll
        for (int k = 0; k < 5; k++) win[r * kWinWords + 4 * h + k] = load_ref4(rowp, x0 + 4 * k, a.stride_y);
    }
    wave_sync();
    const int ddx[4] = {0, -1, 1, 0}, ddy[4] = {-1, 0, 0, 1};
    for (int it = 0; it < a.me_iters; it++) {
        int nb = -1, ncost = bcost, nsad = 0;
        // common case: the whole diamond lies in the LDS window -> 4 SADs in two
        // packed wave sums (independent chains) instead of four sequential ones
        bool all_in = true;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int ox = bx + ddx[k] - cx0, oy = by + ddy[k] - cy0;
            all_in = all_in && ox >= -kWin && ox <= kWin && oy >= -kWin && oy <= kWin;
        }
        if (all_in) {
            uint32_t p[4];
#pragma unroll
            for (int k = 0; k < 4; k++) p[k] = win_sad_lane(win, sw, bx + ddx[k] - cx0, by + ddy[k] - cy0);
            const uint32_t s01 = (uint32_t)wave_sum((int)(p[0] | (p[1] << 16)));
            const uint32_t s23 = (uint32_t)wave_sum((int)(p[2] | (p[3] << 16)));
            const int sds[4] = {(int)(s01 & 0xffff), (int)(s01 >> 16), (int)(s23 & 0xffff), (int)(s23 >> 16)};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                int x = bx + ddx[k], y = by + ddy[k];
                if (x < -R || x > R || y < -R || y > R) continue;
                int c = sds[k] + lam * (sk_se_bits(4 * x) + sk_se_bits(4 * y));
                if (c < ncost) { ncost = c; nb = k; nsad = sds[k]; }
            }
            if (nb < 0) break;
            bx += ddx[nb]; by += ddy[nb]; bcost = ncost; bsad = nsad;
            continue;
        }
#pragma unroll
        for (int k = 0; k < 4; k++) {
            int x = bx + ddx[k], y = by + ddy[k];
            if (x < -R || x > R || y < -R || y > R) continue;
            const int ox = x - cx0, oy = y - cy0;
            int sd = (ox >= -kWin && ox <= kWin && oy >= -kWin && oy <= kWin)
                         ? win_sad(win, sw, ox, oy)
                         : me_sad(a, a.ref.y, sw, mbx, mby, x, y, ylo, yhi);
            int c = sd + lam * (sk_se_bits(4 * x) + sk_se_bits(4 * y));
            if (c < ncost) { ncost = c; nb = k; nsad = sd; }
        }
        if (nb < 0) break;
        bx += ddx[nb]; by += ddy[nb]; bcost = ncost; bsad = nsad;
    }
    const int dev = mb_activity(sw);   // scene-cut intra estimate
    int refi = 0;
    if (t.num_refs > 1 && a.mb_dirty[idx]) {   // second reference at the zero vector (CPU: same rule)
        const int s1 = me_sad(a, a.ref1.y, sw, mbx, mby, 0, 0, ylo, yhi);
        if (s1 + 3 * lam < bcost) {
            bx = by = 0;
            bsad = s1;
            refi = 1;
        }
    }
    if (l == 0) {
        MeResult r;
        r.mvx = (int16_t)bx;
        r.mvy = (int16_t)by;
        r.sad = bsad;
        r.intra_est = dev;
        r.ref = (int16_t)refi;
        r.fx = r.fy = 0;
        a.me[idx] = r;  // per-slice sums are reduced in k_decide (no same-line atomics)
    }
}

// ---------------------------------------------------------------------------
// K4a: exhaustive +-16 integer search on the matrix cores, one wave per dirty MB
// of a P slice (csrc/codec/h264_core.h fs_key; CPU reference full_search).
// With 128-offset samples s' (block) and w' (48x48 reference window),
//   cost(dx,dy) = sum w'^2 - 2 sum s' w'   over the 16x16 block at (dx,dy),
// and the cross term for all 32x32 candidates is one int8 GEMM:
//   D[dxw][dyw] = sum_{r', c} W[r'][dxw + c] * S[(r', c)][dyw],  S[(r',c)][dyw] = s'[r' - dyw][c]
// (zero outside the block): 2 (dx) x 2 (dy) tiles of v_mfma_i32_16x16x64_i8, K = 4
// window rows x 16 columns per instruction, 8 of the 12 K steps per dy tile (the
// others are all-zero in S) = 32 MFMAs per MB. A fragments are unaligned 16-byte
// runs of a window row (5 LDS dwords + v_alignbyte), B fragments aligned block rows.
// sum w'^2 per candidate comes from separable 16-tap box sums in LDS. The wave
// min of fs_key gives the winner, which k_motion_search adds as a predictor.
typedef int v4i __attribute__((ext_vector_type(4)));

// LDS row strides are padded against bank conflicts (MI355X_MICROARCH.md §LDS lane
// groups; modelled per access in tools/lds_bank_model.py): window rows 13 dwords (odd:
// the box-sum row loads of 48 lanes and the A fragments' two rows per 32-lane group fall
// on distinct banks), block rows 5 dwords (B fragments read ~17 different rows per
// group), box-sum rows 36 ints (16-B aligned int4 stores of 8 consecutive lanes cover 32
// distinct banks; the fs_key reads are int4 too). 1512 -> 584 modelled LDS cycles per MB.
__global__ __launch_bounds__(256) void k_me_mfma(FrameArgs a) {
    constexpr int WW = kFsWin / 4;                       // window dwords per row (12)
    constexpr int WP = WW + 1;                           // padded window row stride
    constexpr int BP = 5;                                // padded block row stride
    constexpr int SP = 2 * kFsR + 4;                     // padded box-sum row stride (ints)
    __shared__ uint32_t win_s[4][kFsWin * WP];           // raw reference window per wave
    __shared__ uint32_t blk_s[4][16 * BP];               // raw 16x16 source block
    __shared__ __align__(16) int sq_s[4][kFsWin * SP];   // row box sums of w'^2, then |r_d|^2
    const int w = threadIdx.x >> 6, l = lane_id();
    const int nmb = a.mb_w * a.mb_h;
    const int idx = xcd_remap(blockIdx.x, gridDim.x) * 4 + w;
    if (idx >= nmb) return;
    const int mbx = idx % a.mb_w, mby = idx / a.mb_w;
    const SliceTask t = a.tasks[mby / a.rows_per_slice];
    if (t.action != ACT_P || !a.mb_dirty[idx]) return;
    const int ylo = t.pic_row0 * 16, yhi = (t.pic_row0 + t.pic_rows) * 16 - 1;
    {   // exact match at the MB's previous vector: skip the search (CPU: same rule)
        const int R = a.me_range;
        const int px = sk_clip(a.mvfield[2 * idx], -R, R), py = sk_clip(a.mvfield[2 * idx + 1], -R, R);
        const uint32_t sw = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)(mby * 16 + (l >> 2)) * a.stride_y +
                                                               mbx * 16 + (l & 3) * 4);
        if (me_sad(a, a.ref.y, sw, mbx, mby, px, py, ylo, yhi) == 0) {
            if (l == 0) {
                a.fs_mv[2 * idx] = (int16_t)px;
                a.fs_mv[2 * idx + 1] = (int16_t)py;
            }
            return;
        }
    }
    uint32_t* win = win_s[w];
    uint32_t* blk = blk_s[w];
    int* sq = sq_s[w];
    for (int i = l; i < kFsWin * WW; i += 64) {
        const int wy = i / WW, q = i - wy * WW;
        const int y = sk_clip(mby * 16 - kFsR + wy, ylo, yhi);
        win[wy * WP + q] = load_ref4(a.ref.y + (size_t)y * a.stride_y, mbx * 16 - kFsR + 4 * q, a.stride_y);
    }
    blk[(l >> 2) * BP + (l & 3)] = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)(mby * 16 + (l >> 2)) * a.stride_y +
                                                                     mbx * 16 + (l & 3) * 4);
    wave_sync();
    // |r_d|^2: 16-tap row box sums (lane = window row), then 16-tap column sums in
    // place. Each lane loads its whole row / column into registers before it stores
    // anything: no LDS read waits behind an earlier store (a read-modify-write
    // sliding loop over LDS serialised ~60 round trips per wave).
    if (l < kFsWin) {
        uint32_t rw[WW];
#pragma unroll
        for (int q = 0; q < WW; q++) rw[q] = win[l * WP + q];
        int sqv[kFsWin];
#pragma unroll
        for (int c = 0; c < kFsWin; c++) {
            const int v = (int)((rw[c >> 2] >> (8 * (c & 3))) & 255) - 128;
            sqv[c] = v * v;
        }
        int acc = 0;
#pragma unroll
        for (int c = 0; c < 16; c++) acc += sqv[c];
        int out[2 * kFsR];
        out[0] = acc;
#pragma unroll
        for (int x = 1; x < 2 * kFsR; x++) {
            acc += sqv[x + 15] - sqv[x - 1];
            out[x] = acc;
        }
#pragma unroll
        for (int x = 0; x < 2 * kFsR; x += 4)
            *reinterpret_cast<int4*>(&sq[l * SP + x]) = make_int4(out[x], out[x + 1], out[x + 2], out[x + 3]);
    }
    wave_sync();
    if (l < 2 * kFsR) {
        int col[kFsWin];
#pragma unroll
        for (int r = 0; r < kFsWin; r++) col[r] = sq[r * SP + l];
        int acc = 0;
#pragma unroll
        for (int r = 0; r < 16; r++) acc += col[r];
#pragma unroll
        for (int dy = 0; dy < 2 * kFsR; dy++) {
            sq[dy * SP + l] = acc;
            acc += col[dy + 16] - col[dy];
        }
    }
    // cross-correlation on MFMA: lane (i = l & 15, g = l >> 4)
    const int i16 = l & 15, g = l >> 4;
    v4i acc[2][2];
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) acc[mt][nt] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < kFsWin / 4; ks++) {
        const int rr = 4 * ks + g;                       // window row of this lane's K group
        v4i bf[2];
#pragma unroll
        for (int nt = 0; nt < 2; nt++) {
            const int src = rr - (16 * nt + i16);        // block row feeding candidate row dyw
            const bool in = src >= 0 && src < 16;
#pragma unroll
            for (int q = 0; q < 4; q++) bf[nt][q] = in ? (int)(blk[(in ? src : 0) * BP + q] ^ 0x80808080u) : 0;
        }
#pragma unroll
        for (int mt = 0; mt < 2; mt++) {
            const int b0 = 16 * mt + i16;                // first window column of candidate dxw
            const uint32_t* wr = win + rr * WP + (b0 >> 2);
            const int sh = b0 & 3;
            uint32_t w5[5];
#pragma unroll
            for (int q = 0; q < 5; q++) w5[q] = wr[q];
            v4i af;
#pragma unroll
            for (int q = 0; q < 4; q++) af[q] = (int)(__builtin_amdgcn_alignbyte(w5[q + 1], w5[q], sh) ^ 0x80808080u);
#pragma unroll
            for (int nt = 0; nt < 2; nt++)
                if (ks >= 4 * nt && ks <= 4 * nt + 7)
                    acc[mt][nt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(af, bf[nt], acc[mt][nt], 0, 0, 0);
        }
    }
    wave_sync();
    // D[dxw = 16 mt + 4 g + reg][dyw = 16 nt + i16]
    uint64_t best = ~0ull;
#pragma unroll
    for (int mt = 0; mt < 2; mt++)
#pragma unroll
        for (int nt = 0; nt < 2; nt++) {
            const int dyw = 16 * nt + i16;
            const int4 sv = *reinterpret_cast<const int4*>(&sq[dyw * SP + 16 * mt + 4 * g]);
            const int svr[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {
                const int dxw = 16 * mt + 4 * g + reg;
                const uint64_t k = fs_key(svr[reg] - 2 * acc[mt][nt][reg], dyw, dxw);
                best = k < best ? k : best;
            }
        }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t other = __shfl_xor(best, o);
        best = other < best ? other : best;
    }
    if (l == 0) {
        a.fs_mv[2 * idx] = (int16_t)fs_key_dx(best);
        a.fs_mv[2 * idx + 1] = (int16_t)fs_key_dy(best);
    }
}

// Frame controller on the GPU (one workgroup): commits the previous frame's
// final slice decisions, applies host keyframe requests (host-mapped counter)
// and plans this frame from the stripe dirty flags of k_convert_damage — the
// same plan_stripe/commit_* code the CPU backend runs (codec/h264_encoder.h),
// so no host round trip sits between damage detection and encoding.
__global__ __launch_bounds__(256) void k_plan(FrameArgs a) {
    const int ns = a.num_slices, tid = threadIdx.x;
    StripeState* st = a.plan_state;
    StripeState& pic = st[ns];
    if (a.plan_ctl[1] == 1) {  // deferred commit of the previous frame (2: imported state, committed)
        if (a.fullframe) {
            bool idr = true;
            for (int s = tid; s < ns; s += 256) idr &= a.tasks[s].final_action == ACT_I && a.tasks[s].idr_on_intra;
            idr = __syncthreads_and(idr);
            if (tid == 0) commit_picture(pic, idr, a.plan_cfg.num_refs);
        } else {
            for (int s = tid; s < ns; s += 256) commit_stripe(st[s], a.tasks[s].final_action, a.plan_cfg.num_refs);
        }
    }
    // host overrides (host-mapped snapshot): one round trip, six lanes in parallel; the
    // device copy is what k_rc_qp reads later in the frame
    __shared__ int hk[6];
    if (tid < 6) {
        hk[tid] = __hip_atomic_load(a.key_seq_host + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        a.key_dev[tid] = hk[tid];
    }
    __syncthreads();
    const int kq = hk[0];
    const bool key = kq != a.plan_ctl[0];
    __syncthreads();
    if (key) {
        for (int s = tid; s < ns; s += 256) st[s].need_idr = true;
        if (tid == 0) pic.need_idr = true;
    }
    __syncthreads();
    PlanConfig pc = a.plan_cfg;  // rate-control overrides from the host
    const int qo = hk[1];
    const int po = hk[2];
    if (qo > 0) pc.qp = qo;
    if (po > 0) pc.paint_qp = po;
    {   // K10 CBR: no paint-over refresh (the budget codes every slice at the frame QP anyway)
        const int mode = hk[5] != a.rc->seq ? hk[3] : a.rc->mode;
        if (mode == RC_CBR) pc.use_paint_over = 0;
    }
    for (int s = tid; s < ns; s += 256) {
        st[s].subpel_prev = st[s].subpel_hits;   // adaptive refinement gate (h264_frame.h subpel_gate)
        st[s].subpel_hits = 0;
        const int r0 = s * a.rows_per_slice, nr = min(a.rows_per_slice, a.mb_h - r0);
        plan_stripe(pc, st[s], pic, a.stripe_dirty[s] != 0, r0, nr, a.mb_h, a.tasks[s]);
        a.stripe_dirty[s] = 0;
    }
    __syncthreads();
    if (tid == 0) {
        a.plan_ctl[0] = kq;
        a.plan_ctl[1] = 1;
    }
    if (tid < 4) a.frame_params_dev[tid] = a.frame_params_host[tid];
}

// One workgroup per slice: scene-cut decision from the per-MB ME results.
__global__ __launch_bounds__(256) void k_decide(FrameArgs a) {
    __shared__ long long red[2][4];
    const int s = blockIdx.x;
    SliceTask& t = a.tasks[s];
    const bool planned_p = t.action == ACT_P;
    const bool p = planned_p && t.allow_scenecut;
    long long sad = 0, dev = 0;
    if (planned_p || t.action == ACT_I) {   // planned key frames: activity only (sad 0)
        const int first = t.first_row * a.mb_w, nmb = t.num_rows * a.mb_w;
        for (int i = threadIdx.x; i < nmb; i += 256) {
            const MeResult r = a.me[first + i];
            sad += r.sad;
            dev += r.intra_est;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        sad += __shfl_down(sad, o);
        dev += __shfl_down(dev, o);
    }
    if (lane_id() == 0) {
        red[0][threadIdx.x >> 6] = sad;
        red[1][threadIdx.x >> 6] = dev;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const long long ts = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        const long long td = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        t.final_action = (p && ts > td) ? ACT_I : t.action;
        a.rc_slice[2 * s] = ts;       // K10 complexity (k_rc_qp)
        a.rc_slice[2 * s + 1] = td;
        a.tasks_host[s] = t;  // final decision back to the host (host-mapped)
    }
}

// K10: frame QP from the complexity sums (same rc_apply as the CPU controller).
// Host overrides: key_seq_host[1] qp, [3] rc mode, [4] kbps, [5] change counter.
__device__ void rc_qp_serial(const FrameArgs& a) {
    RcState& rc = *a.rc;
    const int seq = a.key_dev[5];   // k_plan's copy of the host snapshot
    int plan_qp = a.plan_cfg.qp;
    const int qo = a.key_dev[1];
    if (qo > 0) plan_qp = qo;
    if (seq != rc.seq) {   // set_rate() from the host: re-initialise, keep the model if the mode stays
        const int mode = a.key_dev[3];
        const int kbps = a.key_dev[4];
        const RcState old = rc;
        rc_init(rc, mode, plan_qp, kbps, (float)a.rc_fps, a.W * a.H, old.vbv_ms, old.codec);
        if (old.mode == mode)
            for (int k = 0; k < 2; k++) {
                rc.last_qp[k] = old.last_qp[k];
                rc.last_qpf[k] = old.last_qpf[k];
                rc.last_bits[k] = old.last_bits[k];
                rc.last_cplx[k] = old.last_cplx[k];
            }
        if (old.mode == mode) rc.cplx_ema = old.cplx_ema;
        rc.seq = seq;
    }
    rc.base_qp = plan_qp;
    rc_apply(rc, a.tasks, a.rc_slice, a.rc_slice + 1, a.num_slices, a.mb_w, plan_qp, 2);
}
__global__ __launch_bounds__(64) void k_rc_qp(FrameArgs a) {
    if (threadIdx.x == 0) rc_qp_serial(a);
    __syncthreads();
    // the slice QPs to the host-mapped task copies, one lane per slice (uncached PCIe
    // writes: one wave-wide burst instead of a serial loop on lane 0)
    for (int s = threadIdx.x; s < a.num_slices; s += 64) a.tasks_host[s].qp = a.tasks[s].qp;
}

// per_slice > 0: sizes are per NAL, per_slice NALs per slice, counted for coded slices
__global__ __launch_bounds__(64) void k_rc_account(FrameArgs a, const int* sizes, int n, int stride, int per_slice) {
    long long b = 0;
    for (int i = threadIdx.x; i < n; i += 64)
        if (!per_slice || i % per_slice < slice_nals(a, a.tasks[i / per_slice])) b += sizes[(size_t)i * stride];
    for (int o = 32; o > 0; o >>= 1) b += __shfl_down(b, o);
    if (threadIdx.x == 0) rc_account(*a.rc, 8 * b);
}

// K10 CBR guard after k_slice_scan: every workgroup (one per slice) evaluates the same
// overflow test on the frame's payload; on a redo, workgroup 0 moves the slice QPs
// (rc_redo) and raises the flag for the gated second pass, and each workgroup clears
// the header / trailing bits the first k_slice_scan left in its RBSP slot.
__global__ __launch_bounds__(256) void k_rc_guard(FrameArgs a) {
    __shared__ long long part[4];
    const int s = blockIdx.x, tid = threadIdx.x;
    long long b = 0;
    for (int i = tid; i < a.num_slices; i += 256) {
        const int nn = slice_nals(a, a.tasks[i]);
        for (int j = 0; j < nn; j++) b += a.slice_info[4 * (i * a.nal_per_slice + j)];
    }
    for (int o = 32; o > 0; o >>= 1) b += __shfl_down(b, o);
    if ((tid & 63) == 0) part[tid >> 6] = b;
    __syncthreads();
    const long long bits = 8 * (part[0] + part[1] + part[2] + part[3]);
    // rc_redo changes only cur_qp / redos / tasks, none of which rc_redo_step reads:
    // every workgroup takes the same decision whatever the order
    const int step = rc_redo_step(*a.rc, bits);
    if (s == 0 && tid == 0) {
        const int applied = step ? rc_redo(*a.rc, a.tasks, a.num_slices, bits) : 0;
        *a.rc_redo = applied ? 1 : 0;
        if (applied)
            for (int i = 0; i < a.num_slices; i++) a.tasks_host[i].qp = a.tasks[i].qp;
    }
    if (!step || a.tasks[s].final_action == ACT_NONE) return;
    const int nn = slice_nals(a, a.tasks[s]);
    for (int j = 0; j < nn; j++) {
        uint32_t* rbsp = nal_rbsp(a, s, j);
        const int words = (a.slice_info[4 * (s * a.nal_per_slice + j)] + 3) / 4 + 1;
        for (int i = tid; i < words; i += 256) rbsp[i] = 0u;
    }
}

// K10 per-frame cap of the HEVC / AV1 back ends: the frame's payload is the sum of
// `sizes` (bytes: HEVC substreams, AV1 tiles, the units k_rc_account counts); over the
// cap, rc_redo moves the slice QPs / the frame QP coarser and raises *redo for the
// gated next coding pass. One workgroup; *redo is rewritten by the first guard of every
// frame; a later guard (chained: it checks the pass the flag ran) returns at once
// when the flag is down, leaving it down.
__global__ __launch_bounds__(256) void k_rc_guard_sizes(FrameArgs a, const int* sizes, int n, int* redo, int chained) {
    __shared__ long long part[4];
    if (chained && *redo == 0) return;
    const int tid = threadIdx.x;
    long long b = 0;
    for (int i = tid; i < n; i += 256) b += sizes[i];
    for (int o = 32; o > 0; o >>= 1) b += __shfl_down(b, o);
    if ((tid & 63) == 0) part[tid >> 6] = b;
    __syncthreads();
    if (tid != 0) return;
    const long long bits = 8 * (part[0] + part[1] + part[2] + part[3]);
    const int applied = rc_redo_step(*a.rc, bits) ? rc_redo(*a.rc, a.tasks, a.num_slices, bits) : 0;
    *redo = applied ? 1 : 0;
    if (applied)
        for (int i = 0; i < a.num_slices; i++) a.tasks_host[i].qp = a.tasks[i].qp;
}

// ---------------------------------------------------------------------------
// Macroblock residual coding shared by the inter and intra kernels.
struct MbScratch {                 // per-wave LDS
    int16_t coef[kCoefPerMb];      // levels, layout identical to global coefs
    int dcy[16];                   // I16: raw DC (raster) then dequantised DC
    int dcc[8];                    // chroma raw DC then dequantised DC
    int blk_stat[32];              // per-lane scratch
    int misc[8];
    uint8_t nnz[24];               // TotalCoeff per block (luma blkIdx, Cb, Cr)
    uint8_t pad[8];
    int cdcp[8];                   // chroma DC predictions [comp][block]
    uint8_t nb[64];                // intra neighbour samples (intra_pred_lanes layout)
    uint8_t nbtr[4];               // Intra4x4: p[16..19, -1] (above-right MB's bottom row)
    uint8_t ref13[32];             // Intra4x4: reference samples of the (<= 2) blocks being coded (I4RefView)
    uint8_t ry[256];               // Intra4x4: luma reconstruction of the MB so far (16x16)
};

// In-place 4x4 Hadamard H*X*H of a raster int[16] in LDS: rows by lanes 0..3,
// then columns by lanes 0..3 (3 LDS round trips instead of 16 serial reads).
__device__ __forceinline__ void lds_hadamard4x4(int* x) {
    const int l = lane_id();
    if (l < 4) {
        int a = x[l * 4 + 0], b = x[l * 4 + 1], c = x[l * 4 + 2], d = x[l * 4 + 3];
        int s01 = a + b, d01 = a - b, s23 = c + d, d23 = c - d;
        x[l * 4 + 0] = s01 + s23;
        x[l * 4 + 1] = s01 - s23;
        x[l * 4 + 2] = d01 - d23;
        x[l * 4 + 3] = d01 + d23;
    }
    wave_sync();
    if (l < 4) {
        int a = x[l], b = x[4 + l], c = x[8 + l], d = x[12 + l];
        int s01 = a + b, d01 = a - b, s23 = c + d, d23 = c - d;
        x[l] = s01 + s23;
        x[4 + l] = s01 - s23;
        x[8 + l] = d01 - d23;
        x[12 + l] = d01 + d23;
    }
    wave_sync();
}

// 4x4 Hadamard H*X*H of the values in lanes 0..15 (raster: lane = 4y + x) in registers:
// rows by DPP quad permutes, columns by lane shuffles (no LDS round trip, no wave_sync).
__device__ __forceinline__ int lane_hadamard16(int v) {
    const int l = lane_id(), x = l & 3, y = (l >> 2) & 3;
    int P = __builtin_amdgcn_mov_dpp(v, 0xA0, 0xF, 0xF, false);   // quad_perm [0,0,2,2]
    int Q = __builtin_amdgcn_mov_dpp(v, 0xF5, 0xF, 0xF, false);   // quad_perm [1,1,3,3]
    int a = (x & 1) ? P - Q : P + Q;                               // s01 d01 s23 d23
    P = __builtin_amdgcn_mov_dpp(a, 0x50, 0xF, 0xF, false);       // quad_perm [0,0,1,1]
    Q = __builtin_amdgcn_mov_dpp(a, 0xFA, 0xF, 0xF, false);       // quad_perm [2,2,3,3]
    a = (x == 0 || x == 3) ? P + Q : P - Q;
    const int pr = __shfl(a, l ^ 4);
    const int b = (y & 1) ? pr - a : a + pr;
    P = __shfl(b, (l & ~15) + x + 4 * (y >> 1));
    Q = __shfl(b, (l & ~15) + x + 4 * (2 + (y >> 1)));
    return (y == 0 || y == 3) ? P + Q : P - Q;
}

__device__ __forceinline__ int quad_max(int v) {
    v = sk_max(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));
    v = sk_max(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));
    return v;
}

// Sum across the 4 lanes of a quad (DPP), result in every lane of the quad.
__device__ __forceinline__ int quad_sum(int v) {
    v += __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
    v += __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
    return v;
}

// Per-lane quantisation of this lane's luma row and chroma row into LDS, then the
// same analysis as quant_luma / quant_chroma of the CPU path. Returns cbp and
// writes per-block TotalCoeff into S.nnz. The MB size check first uses a
// lane-parallel conservative bound and only runs the exact (nC-free) CAVLC bound
// of mb_bits_bound when that one exceeds the budget: same decisions as the CPU.
__device__ __forceinline__ int quant_mb_lanes(const int* wl, const int* wc, int qp, bool intra16, MbScratch& S,
                              int* bound_out, const CavlcTables& T, int* sl, int* sc,
                              unsigned long long* dbg = nullptr, int step = 0) {
    const int l = lane_id();
    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    const uint32_t izz_row = r == 0 ? 0x06050100u : (r == 1 ? 0x0C070402u : (r == 2 ? 0x0D0B0803u : 0x0F0E0A09u));
    int ln_l = 0, lc_l = 0;   // luma: non-zero count and bound bits of this lane's row
    int ln_c = 0, lc_c = 0;   // chroma AC row
    int lvl[4], lvc[4];       // this lane's quantised levels (|.|) for the bound
    int lastl = -1, lastc = -1;  // highest scan position holding a non-zero level
    // ---- luma ----
    {
        int qbits = 15 + qp / 6;
        int f = quant_f(qbits, intra16);
        const int* mf = H264_QUANT_MF[qp % 6];
        int m0 = mf[0], m1 = mf[1], m2 = mf[2];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int pos = r * 4 + j;
            int lv = quant_coef(wl[j], sel3(pos_class(pos), m0, m1, m2), f, qbits);
            if (intra16 && pos == 0) lv = 0;
            sl[j] = lv;   // kept in registers for the reconstruction
            S.coef[kCoefLuma + b * 16 + ((izz_row >> (8 * j)) & 255)] = (int16_t)lv;
            lvl[j] = sk_abs(lv);
            ln_l += lv != 0;
            if (lv) lastl = sk_max(lastl, (int)((izz_row >> (8 * j)) & 255));
        }

        if (!intra16 && l < 16) S.coef[kCoefLumaDC + l] = 0;
    }
    // ---- chroma ----
    int qpc = chroma_qp(qp);
    {
        int qbits = 15 + qpc / 6;
        int f = quant_f(qbits, intra16);
        const int* mf = H264_QUANT_MF[qpc % 6];
        int m0 = mf[0], m1 = mf[1], m2 = mf[2];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int pos = r * 4 + j;
            int lv = pos == 0 ? 0 : quant_coef(wc[j], sel3(pos_class(pos), m0, m1, m2), f, qbits);
            sc[j] = lv;
            if (l < 32) S.coef[kCoefChromaAC + (comp * 4 + cb) * 16 + ((izz_row >> (8 * j)) & 255)] = (int16_t)lv;
            lvc[j] = sk_abs(lv);
            ln_c += lv != 0;
            if (lv) lastc = sk_max(lastc, (int)((izz_row >> (8 * j)) & 255));
        }
        if (l < 32 && r == 0) S.dcc[comp * 4 + cb] = wc[0];
    }
    STAMP_S(dbg, step, 9);
    {
        int sl_l = suffix_len_cap(quad_max(sk_max(sk_max(lvl[0], lvl[1]), sk_max(lvl[2], lvl[3]))));
        int sl_c = suffix_len_cap(quad_max(sk_max(sk_max(lvc[0], lvc[1]), sk_max(lvc[2], lvc[3]))));
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (lvl[j]) lc_l += level_bits_bound(lvl[j], sl_l);
            if (lvc[j]) lc_c += level_bits_bound(lvc[j], sl_c);
        }
        lastl = quad_max(lastl);
        lastc = quad_max(lastc);
    }
    int bn_l = quad_sum(ln_l), bc_l = quad_sum(lc_l);   // per luma block
    int bn_c = quad_sum(ln_c), bc_c = quad_sum(lc_c);   // per chroma block (lanes < 32)
    wave_sync();
    // I16 luma DC: Hadamard + quant (lanes 0..15 = raster positions)
    int dc_crude = 0, dc_nz = 0;
    if (intra16) {
        // gather the 16 DC coefficients (block b's lane 4b, row 0) into raster lanes 0..15
        const int dc_raw = __shfl(wl[0], 4 * blk_from_xy(l & 3, (l >> 2) & 3));
        const int dc_h = lane_hadamard16(dc_raw);
        if (l < 16) {
            int qbits = 15 + qp / 6;
            int f = quant_f(qbits, true);
            int mf0 = H264_QUANT_MF[qp % 6][0];
            int lv = quant_coef(i16_dc_fwd_round(dc_h), mf0, 2 * f, qbits + 1);
            S.coef[kCoefLumaDC + inv_zigzag4x4(l)] = (int16_t)lv;
            if (lv) { dc_nz = 1; dc_crude = level_bits_bound(sk_abs(lv), 6) + 3; }
        }
    }
    // chroma DC 2x2 Hadamard + quant (lanes 0..7 = comp*4 + i)
    int cdc_crude = 0, cdc_nz = 0;
    if (l < 8) {
        int c = l >> 2, i = l & 3;
        int qbits = 15 + qpc / 6;
        int f = quant_f(qbits, intra16);
        int mf0 = H264_QUANT_MF[qpc % 6][0];
        int d0 = S.dcc[c * 4 + 0], d1 = S.dcc[c * 4 + 1], d2 = S.dcc[c * 4 + 2], d3 = S.dcc[c * 4 + 3];
        int v = i == 0 ? d0 + d1 + d2 + d3 : (i == 1 ? d0 - d1 + d2 - d3 : (i == 2 ? d0 + d1 - d2 - d3 : d0 - d1 - d2 + d3));
        int lv = quant_coef(v, mf0, 2 * f, qbits + 1);
        S.coef[kCoefChromaDC + c * 4 + i] = (int16_t)lv;
        if (lv) { cdc_nz = 1; cdc_crude = level_bits_bound(sk_abs(lv), 6) + 3; }
    }
    wave_sync();
    STAMP_S(dbg, step, 10);
    // ---- cbp analysis ----
    int cbp_l;
    if (intra16) {
        cbp_l = __ballot(bn_l > 0) ? 15 : 0;
    } else {
        // decimation scores (sequential per block, lanes 0..15)
        int score = l < 16 ? decimate_score(S.coef + kCoefLuma + l * 16, 16) : 0;
        int s4 = score + __shfl_down(score, 1) + __shfl_down(score, 2) + __shfl_down(score, 3);
        int sc8[4];
#pragma unroll
        for (int k = 0; k < 4; k++) sc8[k] = __shfl(s4, 4 * k);
        int mb_score = sc8[0] + sc8[1] + sc8[2] + sc8[3];
        cbp_l = 0;
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (sc8[k] >= 4) cbp_l |= 1 << k;
        if (mb_score < 6) cbp_l = 0;
    }
    // chroma: per component decimation (inter), cbp chroma; block b of lanes 4b..4b+3
    int comp_ac[2], chroma_score[2];
    {
        int cscore = 0;
        if (!intra16 && l < 8) cscore = decimate_score(S.coef + kCoefChromaAC + l * 16 + 1, 15);
#pragma unroll
        for (int c = 0; c < 2; c++) {
            comp_ac[c] = __ballot(l >= 16 * c && l < 16 * c + 16 && bn_c > 0) != 0ull;
            chroma_score[c] = wave_sum((l >= 4 * c && l < 4 * c + 4) ? cscore : 0);
        }
    }
    bool zero_comp[2];
#pragma unroll
    for (int c = 0; c < 2; c++) {
        zero_comp[c] = !intra16 && comp_ac[c] && chroma_score[c] < 7;
        if (zero_comp[c]) comp_ac[c] = 0;
    }
    bool any_dc = __ballot(cdc_nz != 0) != 0ull;
    int cbp_c = (comp_ac[0] || comp_ac[1]) ? 2 : (any_dc ? 1 : 0);
    // zero decimated blocks (LDS) and their counts
    bool luma_coded = intra16 ? (cbp_l != 0) : ((cbp_l >> (b >> 2)) & 1);
    if (!intra16 && !luma_coded) {
        if (r == 0) {
            for (int k = 0; k < 16; k++) S.coef[kCoefLuma + b * 16 + k] = 0;
        }
        bn_l = 0;
        bc_l = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) sl[j] = 0;
    }
    if (l < 32 && zero_comp[comp]) {
        if (r == 0)
            for (int k = 0; k < 16; k++) S.coef[kCoefChromaAC + (comp * 4 + cb) * 16 + k] = 0;
        bn_c = 0;
        bc_c = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) sc[j] = 0;
    }
    // TotalCoeff per block for nC (written by the quad leader)
    if (r == 0) S.nnz[b] = luma_coded ? (uint8_t)bn_l : 0;
    if (l < 32 && r == 0) S.nnz[16 + comp * 4 + cb] = cbp_c == 2 ? (uint8_t)bn_c : 0;
    STAMP_S(dbg, step, 11);
    // ---- size check: conservative bound first ----
    // block bound: longest coeff_token for n, exact total_zeros code, run_before
    // <= 2/3 bits per coefficient while zerosLeft <= 2/6 (+8 beyond), level bounds
    auto block_bound = [&](int n, int last, int maxn, int lvbits) {
        if (n == 0) return 6;
        int tz = (maxn == 16 ? last + 1 : last) - n;  // AC blocks (15) start at scan index 1
        int b = T.ct_max_tc[n] + lvbits;
        if (n < maxn) b += T.tz_len[n - 1][tz];
        if (n > 1 && tz > 0) b += tz <= 2 ? 2 * (n - 1) : (tz <= 6 ? 3 * (n - 1) : 3 * (n - 1) + 8);
        return b;
    };
    const int lmax = intra16 ? 15 : 16;
    int crude = 0;
    if (r == 0) {
        if (luma_coded) crude += block_bound(bn_l, lastl, lmax, bc_l);
        if (l < 32 && cbp_c == 2) crude += block_bound(bn_c, lastc, 15, bc_c);
    }
    int dc_sum_n = wave_sum(dc_nz), dc_sum_c = wave_sum(dc_crude);
    int cdc_sum_c = wave_sum(cdc_crude), cdc_sum_n0 = wave_sum(l < 4 ? cdc_nz : 0),
        cdc_sum_n1 = wave_sum(l >= 4 && l < 8 ? cdc_nz : 0);
    int total_crude = 96 + wave_sum(crude);
    if (intra16)
        total_crude += dc_sum_n > 0 ? T.ct_max_tc[dc_sum_n] + (dc_sum_n < 16 ? T.tz_max_tc[dc_sum_n] : 0) + 8 + dc_sum_c : 6;
    // chroma DC: coeff_token <= 8, total_zeros <= 3, run_before <= 2 per coefficient
    if (cbp_c) total_crude += (cdc_sum_n0 > 0 ? 11 : 2) + (cdc_sum_n1 > 0 ? 11 : 2) + cdc_sum_c;
    wave_sync();
    STAMP_S(dbg, step, 12);
    if (dbg && blockIdx.x == SK_STAMP_BLOCK && threadIdx.x == 0 && (unsigned)(step - SK_STAMP_STEP0) < 64u)
        dbg[(step - SK_STAMP_STEP0) * 16 + 14] = total_crude;
    if (total_crude <= kMbBitBudget || intra16) {   // Intra16x16: the conservative bound decides
        *bound_out = total_crude;
        return cbp_l | (cbp_c << 4);
    }
    // ---- exact bound (same terms as mb_bits_bound) ----
    int bnd = 0;
    if (l < 16) {
        if (intra16) { if (cbp_l) bnd = cavlc_block_bits_bound(S.coef + kCoefLuma + l * 16 + 1, 15, T); }
        else if (cbp_l & (1 << (l >> 2))) bnd = cavlc_block_bits_bound(S.coef + kCoefLuma + l * 16, 16, T);
    } else if (l < 24) {
        if (cbp_c == 2) bnd = cavlc_block_bits_bound(S.coef + kCoefChromaAC + (l - 16) * 16 + 1, 15, T);
    } else if (l == 24) {
        if (intra16) bnd = cavlc_block_bits_bound(S.coef + kCoefLumaDC, 16, T);
    } else if (l == 25 || l == 26) {
        if (cbp_c) {
            BitCounter bc;
            cavlc_block(bc, S.coef + kCoefChromaDC + (l - 25) * 4, 4, -1, T);
            bnd = bc.n;
        }
    }
    *bound_out = 96 + wave_sum(bnd);
    return cbp_l | (cbp_c << 4);
}

// Reconstruct this lane's luma row (4 px) and chroma row (lanes < 32).
__device__ __forceinline__ void recon_mb_lanes(int qp, bool intra16, int cbp, MbScratch& S, const int* pred_l,
                               const int* pred_c, int* rec_l, int* rec_c, const int* sl, const int* sc) {
    const int l = lane_id();
    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    int cbp_l = cbp & 15, cbp_c = (cbp >> 4) & 3;
    int qpc = chroma_qp(qp);
    // DC dequant: luma (I16) via the LDS Hadamard, lanes 16..17 chroma components
    int dcy = 0;   // dequantised luma DC of raster block l (lanes 0..15), I16 only
    if (intra16) {
        const int c = l < 16 ? S.coef[kCoefLumaDC + inv_zigzag4x4(l)] : 0;
        const int acc = lane_hadamard16(c);
        const int ls = 16 * H264_DEQUANT_V[qp % 6][0];
        const int q6 = qp / 6;
        dcy = qp >= 36 ? (acc * ls) << (q6 - 6) : (acc * ls + (1 << (5 - q6))) >> (6 - q6);
    }
    if (l >= 16 && l < 18) {
        int c = l - 16;
        int lv[4], dd[4];
        for (int i = 0; i < 4; i++) lv[i] = cbp_c ? S.coef[kCoefChromaDC + c * 4 + i] : 0;
        chroma_dc_dequant(lv, dd, qpc);
        for (int i = 0; i < 4; i++) S.blk_stat[16 + c * 4 + i] = dd[i];
    }
    wave_sync();
    // luma
    {
        int d[4];
        bool coded = intra16 ? (cbp_l != 0) : ((cbp_l >> (b >> 2)) & 1);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int pos = r * 4 + j;
            d[j] = coded ? dequant_coef(sl[j], qp, pos) : 0;   // this lane's levels (registers)
        }
        const int dc_b = __shfl(dcy, blk_y(b) * 4 + blk_x(b));   // block b's DC from its raster lane
        if (intra16 && r == 0) d[0] = dc_b;
        int res[4];
        inv4_quad(d, r, res);
#pragma unroll
        for (int j = 0; j < 4; j++) rec_l[j] = sk_clip255(pred_l[j] + res[j]);
    }
    // chroma (all lanes execute for the DPP quads; lanes >= 32 duplicate)
    {
        int d[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int pos = r * 4 + j;
            d[j] = (cbp_c == 2 && pos != 0) ? dequant_coef(sc[j], qpc, pos) : 0;
        }
        if (r == 0) d[0] = S.blk_stat[16 + comp * 4 + cb];
        int res[4];
        inv4_quad(d, r, res);
#pragma unroll
        for (int j = 0; j < 4; j++) rec_c[j] = sk_clip255(pred_c[j] + res[j]);
    }
}

// Transform + quant (with QP escalation) + recon for one MB. Inputs per lane:
// src/pred of its luma row (4 px) and chroma row. Writes coefs + MbInfo fields.
__device__ __forceinline__ int code_mb(const int* src_l, const int* pred_l, const int* src_c, const int* pred_c,
                       int slice_qp, bool intra16, MbScratch& S, MbInfo& mb, int* rec_l, int* rec_c,
                       int16_t* gcoef, const CavlcTables& T, unsigned long long* dbg = nullptr,
                       int step = 0, int start_qp = -1, bool quant_only = false) {
    const int l = lane_id();
    const int r = l & 3;
    int x[4], wl[4], wc[4];
#pragma unroll
    for (int j = 0; j < 4; j++) x[j] = src_l[j] - pred_l[j];
    fwd4_quad(x, r, wl);
#pragma unroll
    for (int j = 0; j < 4; j++) x[j] = src_c[j] - pred_c[j];
    fwd4_quad(x, r, wc);
    int qp = start_qp >= 0 ? start_qp : slice_qp;
    int cap = sk_min(51, slice_qp + 24);
    int cbp = 0;
    int sl[4], sc[4];   // final levels of this lane's luma / chroma row
    STAMP_S(dbg, step, 3);
    qp = __builtin_amdgcn_readfirstlane(qp);   // wave-uniform: table lookups become scalar loads
    for (;;) {
        int bound;
        cbp = quant_mb_lanes(wl, wc, qp, intra16, S, &bound, T, sl, sc, dbg, step);
        if (dbg && blockIdx.x == SK_STAMP_BLOCK && threadIdx.x == 0 && (unsigned)(step - SK_STAMP_STEP0) < 64u) {
            unsigned long long& d = dbg[(step - SK_STAMP_STEP0) * 16 + 15];
            d = (d & 0xffff) + 1 + ((unsigned long long)bound << 32);
        }
        if (qp + 6 > cap || bound <= mb_bit_budget(intra16)) break;
        qp += 6;
        wave_sync();
    }
    STAMP_S(dbg, step, 4);
    mb.cbp = (uint8_t)cbp;
    mb.qp = (uint8_t)qp;
    if (quant_only) return qp;
    recon_mb_lanes(qp, intra16, cbp, S, pred_l, pred_c, rec_l, rec_c, sl, sc);
    STAMP_S(dbg, step, 5);
    // copy levels to global (816 B = 204 words)
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(S.coef);
    uint32_t* g32 = reinterpret_cast<uint32_t*>(gcoef);
    for (int i = l; i < kCoefPerMb / 2; i += 64) g32[i] = s32[i];
    return qp;
}

// mb_bits_crude_i16 of an Intra4x4 MB, lane-parallel: quad q = luma block q (and chroma
// AC block q for q < 8), each lane 4 scan positions; block terms as block_bits_crude.
__device__ __forceinline__ int i4_bound_lanes(const MbScratch& S, int cbp, const CavlcTables& T) {
    const int l = lane_id(), q = l >> 2, r = l & 3;
    const int cbp_l = cbp & 15, cbp_c = (cbp >> 4) & 3;
    auto block_term = [&](const int16_t* c, int maxn, bool on) __attribute__((always_inline)) {
        int n = 0, last = -1, mx = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int v = sk_abs((int)c[r * 4 + j]);
            if (v) { n++; last = r * 4 + j; mx = sk_max(mx, v); }
        }
        n = quad_sum(n);
        last = quad_max(last);
        mx = quad_max(mx);
        const int sl = suffix_len_cap(mx);
        int lv = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int v = sk_abs((int)c[r * 4 + j]);
            if (v) lv += level_bits_bound(v, sl);
        }
        lv = quad_sum(lv);
        int b = 6;
        if (n) {
            const int tz = (maxn == 16 ? last + 1 : last) - n;
            b = T.ct_max_tc[n] + lv;
            if (n < maxn) b += T.tz_len[n - 1][tz];
            if (n > 1 && tz > 0) b += tz <= 2 ? 2 * (n - 1) : (tz <= 6 ? 3 * (n - 1) : 3 * (n - 1) + 8);
        }
        return (on && r == 0) ? b : 0;
    };
    int t = block_term(S.coef + kCoefLuma + q * 16, 16, (cbp_l >> (q >> 2)) & 1);
    t += block_term(S.coef + kCoefChromaAC + (q & 7) * 16, 15, cbp_c == 2 && q < 8);
    int dn = 0, dc = 0;
    if (l < 8) {
        const int a = sk_abs((int)S.coef[kCoefChromaDC + l]);
        if (a) { dn = 1; dc = level_bits_bound(a, 6) + 3; }
    }
    const int n0 = wave_sum(l < 4 ? dn : 0), n1 = wave_sum(l >= 4 && l < 8 ? dn : 0), cc = wave_sum(dc);
    int total = 96 + wave_sum(t);
    if (cbp_c) total += (n0 > 0 ? 11 : 2) + (n1 > 0 ? 11 : 2) + cc;
    return total;
}

// Intra4x4 macroblock (h264_cpu.cpp code_i4_at): luma block by block in decoding order,
// the 4 lanes of quad b own block b (lane = one row of 4 samples), prediction from
// `sample(x, y)` (MB-relative; the chain passes LDS edges + the reconstruction so far,
// the open-loop pre-pass the source), DPP quad transforms, intra rounding, no decimation;
// then chroma as quant_chroma(intra) and the QP escalation on the conservative bound
// (mb_bits_crude_i16). Writes S.coef / S.nnz / S.ry, mb.cbp / qp; returns the QP.
template <class Smp>
__device__ __forceinline__ int code_mb_i4(Smp sample, const int* src_l, const int* src_c, const int* pred_c, int start_qp,
                          int slice_qp, bool aT, bool aL, bool aTR, MbScratch& S, MbInfo& mb, int* rec_l,
                          int* rec_c, int16_t* gcoef, const CavlcTables& T) {
    const int l = lane_id();
    const int q = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    int xc[4], wc[4];
#pragma unroll
    for (int j = 0; j < 4; j++) xc[j] = src_c[j] - pred_c[j];
    fwd4_quad(xc, r, wc);
    int qp = __builtin_amdgcn_readfirstlane(start_qp);
    const int cap = sk_min(51, slice_qp + 24);
    int scl[4];   // this lane's chroma AC levels (final iteration)
    for (;;) {
        const int qbits = 15 + qp / 6, f = quant_f(qbits, true);
        const int* mf = H264_QUANT_MF[qp % 6];
        const int m0 = mf[0], m1 = mf[1], m2 = mf[2];
        // diagonal wavefront over the 4x4 blocks: stage st codes the blocks with bx + 2 by == st
        // (left, top, top-left and top-right neighbours all belong to earlier stages), so
        // 16 blocks take 10 dependent stages with up to two blocks in flight
        const int qx = blk_x(q), qy = blk_y(q);
        const int m = i4_mode(mb, q);
        for (int st = 0; st < 10; st++) {
            const int by_lo = sk_max(0, (st - 2) >> 1), by_hi = sk_min(3, st >> 1);
            {   // reference samples: lanes 0..12 for the block of row by_lo, 16..28 for by_lo + 1
                const int slot = l >> 4, k = l & 15, by = by_lo + slot;
                if (k < 13 && by <= by_hi)
                    S.ref13[slot * 16 + k] =
                        (uint8_t)i4_ref_sample(sample, blk_from_xy(st - 2 * by, by), aT, aL, aTR, k);
            }
            wave_sync();
            const bool mine = qx + 2 * qy == st;
            // lanes of idle quads follow the first active block (same mode, same samples), so
            // the mode switch diverges over at most the two active modes
            const int b0 = blk_from_xy(st - 2 * by_lo, by_lo);
            const int qq = mine ? q : b0;
            const int me = mine ? m : i4_mode(mb, b0);
            const I4RefView ref{S.ref13 + (mine ? (qy - by_lo) * 16 : 0), i4_has_top(qq, aT), i4_has_left(qq, aL)};
            int pred[4], res[4], w[4], lv[4], d[4], rr[4], n = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                pred[j] = i4_pred_px(me, ref, j, r);
                res[j] = src_l[j] - pred[j];
            }
            fwd4_quad(res, r, w);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int pos = r * 4 + j;
                lv[j] = quant_coef(w[j], sel3(pos_class(pos), m0, m1, m2), f, qbits);
                n += lv[j] != 0;
                d[j] = dequant_coef(lv[j], qp, pos);
                if (mine) S.coef[kCoefLuma + q * 16 + inv_zigzag4x4(pos)] = (int16_t)lv[j];
            }
            n = quad_sum(n);
            if (mine && r == 0) S.nnz[q] = (uint8_t)n;
            inv4_quad(d, r, rr);
            if (mine) {
#pragma unroll
                for (int j = 0; j < 4; j++) S.ry[(qy * 4 + r) * 16 + qx * 4 + j] = (uint8_t)sk_clip255(pred[j] + rr[j]);
            }
            wave_sync();   // the next stage predicts from these blocks
        }
        // chroma: quant_chroma(intra): DC 2x2 Hadamard, AC with intra rounding, no decimation
        const int qpc = chroma_qp(qp), qbc = 15 + qpc / 6, fc = quant_f(qbc, true);
        const int* mfc = H264_QUANT_MF[qpc % 6];
        int nc = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int pos = r * 4 + j;
            const int lvc = pos == 0 ? 0 : quant_coef(wc[j], sel3(pos_class(pos), mfc[0], mfc[1], mfc[2]), fc, qbc);
            scl[j] = lvc;
            nc += lvc != 0;
            if (l < 32) S.coef[kCoefChromaAC + (comp * 4 + cb) * 16 + inv_zigzag4x4(pos)] = (int16_t)lvc;
        }
        if (l < 32 && r == 0) S.dcc[comp * 4 + cb] = wc[0];
        if (l < 16) S.coef[kCoefLumaDC + l] = 0;
        nc = quad_sum(nc);
        wave_sync();
        int cdc_nz = 0;
        if (l < 8) {
            const int c = l >> 2, i = l & 3;
            const int d0 = S.dcc[c * 4 + 0], d1 = S.dcc[c * 4 + 1], d2 = S.dcc[c * 4 + 2], d3 = S.dcc[c * 4 + 3];
            const int v = i == 0 ? d0 + d1 + d2 + d3 : (i == 1 ? d0 - d1 + d2 - d3 : (i == 2 ? d0 + d1 - d2 - d3 : d0 - d1 - d2 + d3));
            const int lv = quant_coef(v, mfc[0], 2 * fc, qbc + 1);
            S.coef[kCoefChromaDC + c * 4 + i] = (int16_t)lv;
            cdc_nz = lv != 0;
        }
        const bool ac0 = __ballot(l < 16 && nc > 0) != 0ull, ac1 = __ballot(l >= 16 && l < 32 && nc > 0) != 0ull;
        const bool any_dc = __ballot(cdc_nz != 0) != 0ull;
        const int cbp_c = (ac0 || ac1) ? 2 : (any_dc ? 1 : 0);
        if (l < 32 && r == 0) S.nnz[16 + comp * 4 + cb] = cbp_c == 2 ? (uint8_t)nc : 0;
        wave_sync();
        int cbp_l = 0;
        for (int b8 = 0; b8 < 4; b8++)
            if (S.nnz[4 * b8] | S.nnz[4 * b8 + 1] | S.nnz[4 * b8 + 2] | S.nnz[4 * b8 + 3]) cbp_l |= 1 << b8;
        mb.cbp = (uint8_t)(cbp_l | (cbp_c << 4));
        mb.qp = (uint8_t)qp;
        // conservative size bound (every lane evaluates the same serial sum over LDS)
        const int bound = i4_bound_lanes(S, mb.cbp, T);
        if (qp + 6 > cap || bound <= mb_bit_budget(true)) break;
        qp += 6;
        wave_sync();
    }
    int zero[4] = {0, 0, 0, 0}, dummy[4];
    recon_mb_lanes(qp, false, mb.cbp & 0x30, S, zero, pred_c, dummy, rec_c, zero, scl);   // chroma only
    {
        const int y = blk_y(q) * 4 + r, x0 = blk_x(q) * 4;
#pragma unroll
        for (int j = 0; j < 4; j++) rec_l[j] = S.ry[y * 16 + x0 + j];
    }
    if (gcoef) {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(S.coef);
        uint32_t* g32 = reinterpret_cast<uint32_t*>(gcoef);
        for (int i = l; i < kCoefPerMb / 2; i += 64) g32[i] = s32[i];
    }
    return qp;
}

// ---------------------------------------------------------------------------
// MB-level AQ (h264_mb.h aq_offset): one wave per MB of a coded (P / I) slice, lane =
// one row quarter (4 pixels); sum and sum of squares by wave reduction.
__global__ __launch_bounds__(256) void k_aq(FrameArgs a) {
    const int nmb = a.mb_w * a.mb_h;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= nmb) return;   // wave-uniform
    const int mbx = idx % a.mb_w, mby = idx / a.mb_w;
    const int act = a.tasks[mby / a.rows_per_slice].final_action;
    if (act != ACT_P && act != ACT_I) return;
    const int l = lane_id();
    const uint32_t w = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)(mby * 16 + (l >> 2)) * a.stride_y +
                                                          mbx * 16 + 4 * (l & 3));
    uint32_t sum = 0, ssq = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint32_t v = (w >> (8 * j)) & 255u;
        sum += v;
        ssq += v * v;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        ssq += __shfl_xor(ssq, o);
    }
    if (l == 0) a.aq[idx] = (int8_t)aq_offset(aq_energy(sum, ssq), a.aq_strength);
}

// ---------------------------------------------------------------------------
// Quarter-pel interpolation through LDS (same values as h264_core.h luma_qpel_sample):
// a 24x24 window of clamped reference samples around the MB's integer vector, its
// half-sample planes b (horizontal), h (vertical) and j (centre, from the unclipped b1),
// then any quarter position (Table 8-12) is one to four LDS reads. Window origin: the
// integer vector minus 3 samples, so quarter offsets -3..+3 around it stay inside.
struct QpelLds {
    uint8_t win[24][24];
    int16_t b1[24][24];
    uint8_t bp[24][24], hp[24][24], jp[24][24];
};
__device__ __forceinline__ int qtap6(int a, int b, int c, int d, int e, int f) {
    return a - 5 * b + 20 * c + 20 * d - 5 * e + f;
}
// Compact variant (one output per lane step, few live registers) for k_code_inter,
// whose occupancy would suffer from qpel_fill_fast's register windows.
__device__ void qpel_fill(QpelLds& Q, const uint8_t* ref, int stride, int w, int ylo, int yhi, int ox, int oy) {
    const int l = lane_id();
    for (int i = l; i < 576; i += 64) {
        const int r = i / 24, c = i - 24 * r;
        Q.win[r][c] = ref[(size_t)sk_clip(oy + r, ylo, yhi) * stride + sk_clip(ox + c, 0, w - 1)];
    }
    wave_sync();
    for (int i = l; i < 576; i += 64) {
        const int r = i / 24, c = i - 24 * r;
        if (c >= 2 && c <= 20) {
            const int b1 = qtap6(Q.win[r][c - 2], Q.win[r][c - 1], Q.win[r][c], Q.win[r][c + 1], Q.win[r][c + 2],
                                 Q.win[r][c + 3]);
            Q.b1[r][c] = (int16_t)b1;
            Q.bp[r][c] = (uint8_t)sk_clip255((b1 + 16) >> 5);
        }
        if (r >= 2 && r <= 20) {
            const int h1 = qtap6(Q.win[r - 2][c], Q.win[r - 1][c], Q.win[r][c], Q.win[r + 1][c], Q.win[r + 2][c],
                                 Q.win[r + 3][c]);
            Q.hp[r][c] = (uint8_t)sk_clip255((h1 + 16) >> 5);
        }
    }
    wave_sync();
    for (int i = l; i < 576; i += 64) {
        const int r = i / 24, c = i - 24 * r;
        if (r >= 2 && r <= 20 && c >= 2 && c <= 20)
            Q.jp[r][c] = (uint8_t)sk_clip255((qtap6(Q.b1[r - 2][c], Q.b1[r - 1][c], Q.b1[r][c], Q.b1[r + 1][c],
                                                    Q.b1[r + 2][c], Q.b1[r + 3][c]) + 512) >> 10);
    }
    wave_sync();
}
// The 6-tap passes slide along a row (b1/bp), a column (hp) or a column of b1 (jp) in
// registers: each lane reads its <= 15 window samples once instead of 6 per output.
__device__ void qpel_fill_fast(QpelLds& Q, const uint8_t* ref, int stride, int w, int ylo, int yhi, int ox, int oy) {
    const int l = lane_id();
    for (int i = l; i < 576; i += 64) {
        const int r = i / 24, c = i - 24 * r;
        Q.win[r][c] = ref[(size_t)sk_clip(oy + r, ylo, yhi) * stride + sk_clip(ox + c, 0, w - 1)];
    }
    wave_sync();
    if (l < 48) {
        const int k = l >> 1, half = l & 1;
        // horizontal: b1 / bp of row k, columns [2, 11] or [12, 20]
        {
            const int c0 = half ? 12 : 2, n = half ? 9 : 10;
            int v[15];
#pragma unroll
            for (int i = 0; i < 15; i++) v[i] = (i < n + 5) ? Q.win[k][c0 - 2 + i] : 0;
#pragma unroll
            for (int i = 0; i < 10; i++) {
                if (i < n) {
                    const int b1 = qtap6(v[i], v[i + 1], v[i + 2], v[i + 3], v[i + 4], v[i + 5]);
                    Q.b1[k][c0 + i] = (int16_t)b1;
                    Q.bp[k][c0 + i] = (uint8_t)sk_clip255((b1 + 16) >> 5);
                }
            }
        }
        // vertical: hp of column k, rows [2, 11] or [12, 20]
        {
            const int r0 = half ? 12 : 2, n = half ? 9 : 10;
            int v[15];
#pragma unroll
            for (int i = 0; i < 15; i++) v[i] = (i < n + 5) ? Q.win[r0 - 2 + i][k] : 0;
#pragma unroll
            for (int i = 0; i < 10; i++)
                if (i < n)
                    Q.hp[r0 + i][k] = (uint8_t)sk_clip255((qtap6(v[i], v[i + 1], v[i + 2], v[i + 3], v[i + 4],
                                                                 v[i + 5]) + 16) >> 5);
        }
    }
    wave_sync();
    if (l < 57) {   // centre: jp of column 2 + l % 19, rows [2, 8], [9, 14] or [15, 20]
        const int c = 2 + l % 19, seg = l / 19;
        const int r0 = seg == 0 ? 2 : (seg == 1 ? 9 : 15), n = seg == 0 ? 7 : 6;
        int v[12];
#pragma unroll
        for (int i = 0; i < 12; i++) v[i] = (i < n + 5) ? Q.b1[r0 - 2 + i][c] : 0;
#pragma unroll
        for (int i = 0; i < 7; i++)
            if (i < n)
                Q.jp[r0 + i][c] = (uint8_t)sk_clip255((qtap6(v[i], v[i + 1], v[i + 2], v[i + 3], v[i + 4], v[i + 5]) +
                                                       512) >> 10);
    }
    wave_sync();
}
// Sample for MB-relative pixel (x, y) at quarter offset (dqx, dqy) in [-3, 3] from the
// window's integer vector.
__device__ __forceinline__ int qpel_lookup(const QpelLds& Q, int x, int y, int dqx, int dqy) {
    const int cx = x + 3 + (dqx >> 2), cy = y + 3 + (dqy >> 2), fx = dqx & 3, fy = dqy & 3;
    const int G = Q.win[cy][cx];
    if (!(fx | fy)) return G;
    if (fy == 0) {
        const int b = Q.bp[cy][cx];
        return fx == 2 ? b : ((fx == 1 ? G : Q.win[cy][cx + 1]) + b + 1) >> 1;
    }
    if (fx == 0) {
        const int h = Q.hp[cy][cx];
        return fy == 2 ? h : ((fy == 1 ? G : Q.win[cy + 1][cx]) + h + 1) >> 1;
    }
    if (fx == 2 && fy == 2) return Q.jp[cy][cx];
    if (fx == 2) return (Q.bp[cy + (fy >> 1)][cx] + Q.jp[cy][cx] + 1) >> 1;
    if (fy == 2) return (Q.hp[cy][cx + (fx >> 1)] + Q.jp[cy][cx] + 1) >> 1;
    return (Q.bp[cy + (fy >> 1)][cx] + Q.hp[cy][cx + (fx >> 1)] + 1) >> 1;
}

// ---------------------------------------------------------------------------
// K4c quarter-pel refinement (CpuH264Encoder::subpel_refine): one wave per MB of a P
// slice, lane = 4 pixels of one row; the integer vector, its 8 half-sample and then 8
// quarter-sample neighbours are scored by SAD against the 6-tap interpolation
// (luma_qpel_sample, computed on the fly from the reference plane).
__global__ __launch_bounds__(256) void k_subpel(FrameArgs a) {
    __shared__ QpelLds Qw[4];
    QpelLds& Q = Qw[threadIdx.x >> 6];
    const int nmb = a.mb_w * a.mb_h;
    const int idx = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    if (idx >= nmb) return;   // wave-uniform; no block barriers below
    const int mbx = idx % a.mb_w, mby = idx / a.mb_w;
    const SliceTask t = a.tasks[mby / a.rows_per_slice];
    if (t.final_action != ACT_P) return;
    const MeResult r = a.me[idx];
    const int l = lane_id();
    const int sl = mby / a.rows_per_slice;
    if (r.sad <= kSubpelMinSad || !subpel_gate(t.frame_num, a.plan_state[sl].subpel_prev, t.num_rows * a.mb_w)) {
        if (l == 0) { a.me[idx].fx = 0; a.me[idx].fy = 0; }
        return;
    }
    const int ylo = t.pic_row0 * 16, yhi = (t.pic_row0 + t.pic_rows) * 16 - 1;
    qpel_fill_fast(Q, r.ref ? a.ref1.y : a.ref.y, a.stride_y, a.stride_y, ylo, yhi, mbx * 16 + r.mvx - 3,
              mby * 16 + r.mvy - 3);
    const int yy = l >> 2, xx = 4 * (l & 3);
    const uint32_t sw = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)(mby * 16 + yy) * a.stride_y +
                                                          mbx * 16 + xx);
    auto sad_q = [&](int dqx, int dqy) __attribute__((always_inline)) {
        int s = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
            s += sk_abs((int)((sw >> (8 * j)) & 255u) - qpel_lookup(Q, xx + j, yy, dqx, dqy));
        return wave_sum(s);
    };
    int bx = 0, by = 0, best = sad_q(0, 0);
    const int int_sad = best;
    for (int step = 2; step >= 1; step--) {
        const int cx = bx, cy = by;
        for (int k = 0; k < 8; k++) {   // ring order of the host reference
            const int kk = k < 4 ? k : k + 1;
            const int qx = cx + step * (kk % 3 - 1), qy = cy + step * (kk / 3 - 1);
            const int c = sad_q(qx, qy);
            if (c < best) {
                best = c;
                bx = qx;
                by = qy;
            }
        }
    }
    if (l == 0) {
        a.me[idx].fx = (int8_t)bx;
        a.me[idx].fy = (int8_t)by;
        if ((bx | by) && subpel_hit(best, int_sad)) atomicAdd(&a.plan_state[mby / a.rows_per_slice].subpel_hits, 1);
    }
}

// ---------------------------------------------------------------------------
// K6 inter: one wave per MB of a P slice (SKIPALL slices just record skips).
// 4 waves per workgroup, one MB per wave: the CAVLC tables are loaded once per 4 MBs.
__global__ __launch_bounds__(256) void k_code_inter(FrameArgs a) {
    if (a.gate && *a.gate == 0) return;   // CBR second pass not needed
    __shared__ MbScratch Sw[4];
    __shared__ QpelLds Qw[4];   // fractional-MV luma MC
    __shared__ CavlcTables T;
    MbScratch& S = Sw[threadIdx.x >> 6];
    int nmb = a.mb_w * a.mb_h;
    int idx = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    const bool valid = idx < nmb;
    int mbx = valid ? idx % a.mb_w : 0, mby = valid ? idx / a.mb_w : 0;
    int s = mby / a.rows_per_slice;
    const SliceTask t = a.tasks[s];
    int l = lane_id();
    if (valid && t.final_action == ACT_SKIPALL && l == 0) {
        MbInfo z;
        memset(&z, 0, sizeof(z));
        a.mbs[idx] = z;
        a.me[idx].mvx = 0;
        a.me[idx].mvy = 0;
        a.me[idx].ref = 0;
        a.me[idx].fx = a.me[idx].fy = 0;
    }
    // Blocks with no P macroblock (skipped / intra / out-of-range) leave before the table load.
    const bool coded = valid && t.final_action == ACT_P;
    if (!__syncthreads_or(coded)) return;
    load_cavlc_tables(T, a.cavlc_tabs);
    __syncthreads();
    if (!coded) return;
    // MV prediction from the final motion field (all MBs of a P slice are inter)
    auto nbr = [&](int ox, int oy, bool ok) {
        MvNb n;
        n.avail = ok;
        n.ref = ok ? a.me[oy * a.mb_w + ox].ref : -1;
        n.mvx = ok ? me_qx(a.me[oy * a.mb_w + ox]) : 0;
        n.mvy = ok ? me_qy(a.me[oy * a.mb_w + ox]) : 0;
        return n;
    };
    bool top = mby > t.first_row;
    MvNb A = nbr(mbx - 1, mby, mbx > 0);
    MvNb B = nbr(mbx, mby - 1, top);
    MvNb C = nbr(mbx + 1, mby - 1, top && mbx + 1 < a.mb_w);
    if (!C.avail) C = nbr(mbx - 1, mby - 1, top && mbx > 0);
    const int refi = a.me[idx].ref;
    const Planes& rp = refi ? a.ref1 : a.ref;
    int pmx, pmy, smx, smy;
    mv_pred16x16(A, B, C, refi, &pmx, &pmy);
    mv_pskip(A, B, C, &smx, &smy);
    int mvx = me_qx(a.me[idx]), mvy = me_qy(a.me[idx]);

    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    int ylo = t.pic_row0 * 16, yhi = (t.pic_row0 + t.pic_rows) * 16 - 1;
    // luma source + MC prediction (integer: one 4-byte load; fractional: 6-tap, qpel)
    int px = mbx * 16 + blk_x(b) * 4, py = mby * 16 + blk_y(b) * 4 + r;
    uint32_t sw = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)py * a.stride_y + px);
    int src_l[4], pred_l[4];
    if (!((mvx | mvy) & 3)) {   // wave-uniform
        int sy = sk_clip(py + (mvy >> 2), ylo, yhi);
        uint32_t pw = load_ref4(rp.y + (size_t)sy * a.stride_y, px + (mvx >> 2), a.stride_y);
#pragma unroll
        for (int j = 0; j < 4; j++) pred_l[j] = (pw >> (8 * j)) & 255;
    } else {   // fractional: interpolation window through LDS (k_subpel's QpelLds)
        QpelLds& Q = *reinterpret_cast<QpelLds*>(&Qw[threadIdx.x >> 6]);
        qpel_fill(Q, rp.y, a.stride_y, a.stride_y, ylo, yhi, mbx * 16 + (mvx >> 2) - 3, mby * 16 + (mvy >> 2) - 3);
#pragma unroll
        for (int j = 0; j < 4; j++)
            pred_l[j] = qpel_lookup(Q, px - mbx * 16 + j, py - mby * 16, mvx & 3, mvy & 3);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) src_l[j] = (sw >> (8 * j)) & 255;
    // chroma source + bilinear MC prediction
    const uint8_t* cs = comp ? a.src.v : a.src.u;
    const uint8_t* crf = comp ? rp.v : rp.u;
    int cx0 = mbx * 8 + (cb & 1) * 4, cy0 = mby * 8 + (cb >> 1) * 4 + r;
    uint32_t csw = *reinterpret_cast<const uint32_t*>(cs + (size_t)cy0 * a.stride_c + cx0);
    int src_c[4], pred_c[4];
    const uint8_t* cbase = crf + (size_t)(t.pic_row0 * 8) * a.stride_c;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        src_c[j] = (csw >> (8 * j)) & 255;
        pred_c[j] = chroma_mc_sample(cbase, a.stride_c, a.stride_c, t.pic_rows * 8, cx0 + j,
                                     cy0 - t.pic_row0 * 8, mvx, mvy);
    }
    MbInfo mb;
    memset(&mb, 0, sizeof(mb));
    mb.type = MB_P_16x16;
    int rec_l[4], rec_c[4];
    code_mb(src_l, pred_l, src_c, pred_c, t.qp, false, S, mb, rec_l, rec_c,
            a.coefs + (size_t)idx * kCoefPerMb, T, nullptr, 0,
            a.aq_strength > 0 ? aq_start_qp(t.qp, a.aq[idx]) : -1);
    // recon
    uint32_t rw = (uint32_t)rec_l[0] | ((uint32_t)rec_l[1] << 8) | ((uint32_t)rec_l[2] << 16) |
                  ((uint32_t)rec_l[3] << 24);
    *reinterpret_cast<uint32_t*>(a.rec.y + (size_t)py * a.stride_y + px) = rw;
    if (l < 32) {
        uint8_t* cr = comp ? a.rec.v : a.rec.u;
        uint32_t cw = (uint32_t)rec_c[0] | ((uint32_t)rec_c[1] << 8) | ((uint32_t)rec_c[2] << 16) |
                      ((uint32_t)rec_c[3] << 24);
        *reinterpret_cast<uint32_t*>(cr + (size_t)cy0 * a.stride_c + cx0) = cw;
    }
    if (l == 0) {
        mb.mvx = (int16_t)mvx;
        mb.mvy = (int16_t)mvy;
        mb.ref = (uint8_t)refi;
        if (mb.cbp == 0 && refi == 0 && mvx == smx && mvy == smy) {
            mb.type = MB_P_SKIP;
        } else {
            mb.mvdx = (int16_t)(mvx - pmx);
            mb.mvdy = (int16_t)(mvy - pmy);
        }
        for (int i = 0; i < 24; i++) mb.nnz[i] = S.nnz[i];
        a.mbs[idx] = mb;
    }
}

// ---------------------------------------------------------------------------
// Luma (I16) and chroma intra modes of one MB by wave-wide SADs: luma in the
// evaluation order DC, V, H, Plane; chroma DC, H, V, Plane (first minimum wins).
// topp/leftp/ctop/cleft: neighbour samples (zeros when unavailable), lane layout
// as everywhere (b, r luma rows; comp/cb chroma rows).
__device__ __forceinline__ void intra_modes_wave(const int* src_l, const int* src_c, const uint8_t* topp, const uint8_t* leftp,
                                 int tl, const uint8_t* const* ctop, const uint8_t* const* cleft, const int* ctl,
                                 bool aT, bool aL, int* cdcp, int* luma_mode, int* chroma_mode,
                                 int* luma_sad = nullptr) {
    const int l = lane_id();
    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    const int lx = blk_x(b) * 4, ly = blk_y(b) * 4 + r;
    int dc = i16_dc(topp, leftp, aT, aL);
    int pa = 0, pb = 0, pc = 0;
    if (aT && aL) i16_plane_params(topp, leftp, tl, &pa, &pb, &pc);
    const int order[4] = {2, 0, 1, 3};
    int best_mode = 2, best_sad = 0x7fffffff;
    for (int oi = 0; oi < 4; oi++) {
        int m = order[oi];
        if ((m == 0 && !aT) || (m == 1 && !aL) || (m == 3 && !(aT && aL))) continue;
        int sad = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
            sad += sk_abs(src_l[j] - i16_pred_pixel(m, lx + j, ly, topp, leftp, tl, aT, aL, dc, pa, pb, pc));
        sad = wave_sum(sad);
        if (sad < best_sad) { best_sad = sad; best_mode = m; }
    }
    const uint8_t* ct = ctop[comp];
    const uint8_t* cf = cleft[comp];
    const int clx = (cb & 1) * 4, cly = (cb >> 1) * 4 + r;
    int qa = 0, qb = 0, qc = 0;
    if (aT && aL) chroma_plane_params(ct, cf, ctl[comp], &qa, &qb, &qc);
    if (l < 8) cdcp[l] = chroma_dc_block(l & 1, (l >> 1) & 1, ctop[l >> 2], cleft[l >> 2], aT, aL);
    wave_sync();
    const int cdc_mine = cdcp[comp * 4 + cb];
    int best_cm = 0, best_csad = 0x7fffffff;
    for (int m = 0; m < 4; m++) {
        if ((m == 1 && !aL) || (m == 2 && !aT) || (m == 3 && !(aT && aL))) continue;
        int sad = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            int x = clx + j, y = cly, v;
            if (m == 0) v = cdc_mine;
            else if (m == 1) v = cf[y];
            else if (m == 2) v = ct[x];
            else v = sk_clip255((qa + qb * (x - 3) + qc * (y - 3) + 16) >> 5);
            sad += sk_abs(src_c[j] - v);
        }
        sad = wave_sum(l < 32 ? sad : 0);
        if (sad < best_csad) { best_csad = sad; best_cm = m; }
    }
    *luma_mode = best_mode;
    *chroma_mode = best_cm;
    if (luma_sad) *luma_sad = best_sad;
}

// Sum of v over the lanes of a wave-uniform lane mask (DPP + readlanes).
__device__ __forceinline__ int wave_sum_masked(int v, bool on) { return wave_sum(on ? v : 0); }

// This lane's luma / chroma prediction row for the given (wave-uniform) modes.
// nb: the wave's neighbour samples in LDS, top 16 | left 16 | ctop[2][8] | cleft[2][8]
// (zeros when unavailable); tl / ctl: corner samples. Sums (DC, plane gradients) are
// wave reductions, so no lane walks the edges serially.
__device__ __forceinline__ void intra_pred_lanes(int mode, int cmode, const uint8_t* nb, int tl, const int* ctl, bool aT, bool aL,
                                 int* pred_l, int* pred_c) {
    const int l = lane_id();
    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    const int lx = blk_x(b) * 4, ly = blk_y(b) * 4 + r;
    const int clx = (cb & 1) * 4, cly = (cb >> 1) * 4 + r;
    const int e = nb[l];   // this lane's edge sample
    // ---- luma ----
    if (mode == 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) pred_l[j] = nb[lx + j];
    } else if (mode == 1) {
        const int v = nb[16 + ly];
#pragma unroll
        for (int j = 0; j < 4; j++) pred_l[j] = v;
    } else if (mode == 2) {
        const int st = wave_sum_masked(e, l < 16), sl = wave_sum_masked(e, l >= 16 && l < 32);
        const int dc = (aT && aL) ? (st + sl + 16) >> 5 : (aL ? (sl + 8) >> 4 : (aT ? (st + 8) >> 4 : 128));
#pragma unroll
        for (int j = 0; j < 4; j++) pred_l[j] = dc;
    } else {
        // lanes 0..7: H terms (top), 8..15: V terms (left); i = l & 7
        const int i = l & 7, base = l < 8 ? 0 : 16;
        const int p1 = nb[base + 8 + i];
        const int p0 = 6 - i >= 0 ? nb[base + sk_max(6 - i, 0)] : tl;
        const int term = (i + 1) * (p1 - p0);
        const int H = wave_sum_masked(term, l < 8), V = wave_sum_masked(term, l >= 8 && l < 16);
        const int pa = 16 * (nb[16 + 15] + nb[15]);
        const int pb = (5 * H + 32) >> 6, pc = (5 * V + 32) >> 6;
#pragma unroll
        for (int j = 0; j < 4; j++) pred_l[j] = sk_clip255((pa + pb * (lx + j - 7) + pc * (ly - 7) + 16) >> 5);
    }
    // ---- chroma ----
    const int ct = 32 + 8 * comp, cf = 48 + 8 * comp;   // this lane's component edges in nb
    if (cmode == 0) {
        // quad sums over the chroma edge lanes: lane 32 + 8c + 4bx -> top sum of block column bx,
        // lane 48 + 8c + 4by -> left sum of block row by
        const int q = quad_sum(e);
        const int st = __shfl(q, 32 + 8 * comp + 4 * (cb & 1));
        const int sl = __shfl(q, 48 + 8 * comp + 4 * (cb >> 1));
        const int bx = cb & 1, by = cb >> 1;
        int v;
        if (bx == by) v = (aT && aL) ? (st + sl + 4) >> 3 : (aL ? (sl + 2) >> 2 : (aT ? (st + 2) >> 2 : 128));
        else if (bx == 1) v = aT ? (st + 2) >> 2 : (aL ? (sl + 2) >> 2 : 128);
        else v = aL ? (sl + 2) >> 2 : (aT ? (st + 2) >> 2 : 128);
#pragma unroll
        for (int j = 0; j < 4; j++) pred_c[j] = v;
    } else if (cmode == 1) {
        const int v = nb[cf + cly];
#pragma unroll
        for (int j = 0; j < 4; j++) pred_c[j] = v;
    } else if (cmode == 2) {
#pragma unroll
        for (int j = 0; j < 4; j++) pred_c[j] = nb[ct + clx + j];
    } else {
        // lanes 0..31: component l >> 4, (l >> 3) & 1 selects the H (top) or V (left) terms, i = l & 3
        const int tc = (l >> 4) & 1, isv = (l >> 3) & 1, i = l & 3;
        const int base = isv ? 48 + 8 * tc : 32 + 8 * tc;
        const int p1 = nb[base + 4 + i];
        const int p0 = 2 - i >= 0 ? nb[base + sk_max(2 - i, 0)] : ctl[tc];
        const int term = (l & 4) ? 0 : (i + 1) * (p1 - p0);   // lanes with (l & 4) are padding
        const int H0 = wave_sum_masked(term, l < 8), V0 = wave_sum_masked(term, l >= 8 && l < 16);
        const int H1 = wave_sum_masked(term, l >= 16 && l < 24), V1 = wave_sum_masked(term, l >= 24 && l < 32);
        const int H = comp ? H1 : H0, V = comp ? V1 : V0;
        const int pa = 16 * (nb[cf + 7] + nb[ct + 7]);
        const int pb = (34 * H + 32) >> 6, pc = (34 * V + 32) >> 6;
#pragma unroll
        for (int j = 0; j < 4; j++) pred_c[j] = sk_clip255((pa + pb * (clx + j - 3) + pc * (cly - 3) + 16) >> 5);
    }
}

// Loads the neighbour layout nb (see intra_pred_lanes) of one MB from a plane set.
__device__ void load_nb_planes(const Planes& P, int sy, int sc, int mbx, int mby, bool aT, bool aL, uint8_t* nb,
                               int* tl, int* ctl) {
    const int l = lane_id();
    int v = 0;
    if (l < 16) v = aT ? P.y[(size_t)(mby * 16 - 1) * sy + mbx * 16 + l] : 0;
    else if (l < 32) v = aL ? P.y[(size_t)(mby * 16 + l - 16) * sy + mbx * 16 - 1] : 0;
    else if (l < 48) {
        const uint8_t* C = (l & 8) ? P.v : P.u;
        v = aT ? C[(size_t)(mby * 8 - 1) * sc + mbx * 8 + (l & 7)] : 0;
    } else {
        const uint8_t* C = (l & 8) ? P.v : P.u;
        v = aL ? C[(size_t)(mby * 8 + (l & 7)) * sc + mbx * 8 - 1] : 0;
    }
    nb[l] = (uint8_t)v;
    *tl = (aT && aL) ? P.y[(size_t)(mby * 16 - 1) * sy + mbx * 16 - 1] : 0;
    ctl[0] = (aT && aL) ? P.u[(size_t)(mby * 8 - 1) * sc + mbx * 8 - 1] : 0;
    ctl[1] = (aT && aL) ? P.v[(size_t)(mby * 8 - 1) * sc + mbx * 8 - 1] : 0;
    wave_sync();
}

// K5 open-loop pre-pass, one wave per MB of an I slice (all MBs in parallel): intra
// modes against the SOURCE neighbours and the QP the MB needs under the bit budget
// with that prediction. k_code_intra's wavefront then only predicts, quantises from
// that QP and reconstructs (no mode search, usually no escalation in the chain).
__global__ __launch_bounds__(256) void k_intra_prep(FrameArgs a) {
    if (a.gate && *a.gate == 0) return;   // CBR second pass not needed
    __shared__ MbScratch Sw[4];
    __shared__ CavlcTables T;
    __shared__ uint8_t nb_w[4][64];   // top 16 | left 16 | ctop 2x8 | cleft 2x8
    MbScratch& S = Sw[threadIdx.x >> 6];
    uint8_t* nb = nb_w[threadIdx.x >> 6];
    const int nmb = a.mb_w * a.mb_h;
    const int idx = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    const bool valid = idx < nmb;
    const int mbx = valid ? idx % a.mb_w : 0, mby = valid ? idx / a.mb_w : 0;
    const SliceTask t = a.tasks[mby / a.rows_per_slice];
    const bool coded = valid && t.final_action == ACT_I;
    if (!__syncthreads_or(coded)) return;
    load_cavlc_tables(T, a.cavlc_tabs);
    __syncthreads();
    if (!coded) return;
    const int l = lane_id();
    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    bool aT = mby > t.first_row, aL = mbx > 0;
    if (split_i(a, t)) {   // K5 sub-slice: left neighbour inside it only, never the top
        aT = false;
        aL = aL && (idx - t.first_row * a.mb_w) % kIntraSubMbs != 0;
    }
    // source neighbours into LDS (zeros when unavailable)
    int tl, ctl[2];
    load_nb_planes(a.src, a.stride_y, a.stride_c, mbx, mby, aT, aL, nb, &tl, ctl);
    const uint8_t* ctop[2] = {nb + 32, nb + 40};
    const uint8_t* cleft[2] = {nb + 48, nb + 56};
    int px = mbx * 16 + blk_x(b) * 4, py = mby * 16 + blk_y(b) * 4 + r;
    uint32_t sw = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)py * a.stride_y + px);
    const uint8_t* cs = comp ? a.src.v : a.src.u;
    int cx0 = mbx * 8 + (cb & 1) * 4, cy0 = mby * 8 + (cb >> 1) * 4 + r;
    uint32_t csw = *reinterpret_cast<const uint32_t*>(cs + (size_t)cy0 * a.stride_c + cx0);
    int src_l[4], src_c[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        src_l[j] = (sw >> (8 * j)) & 255;
        src_c[j] = (csw >> (8 * j)) & 255;
    }
    int mode, cmode, sad16;
    intra_modes_wave(src_l, src_c, nb, nb + 16, tl, ctop, cleft, ctl, aT, aL, S.cdcp, &mode, &cmode, &sad16);
    int pred_l[4], pred_c[4];
    intra_pred_lanes(mode, cmode, nb, tl, ctl, aT, aL, pred_l, pred_c);
    const int start = a.aq_strength > 0 ? aq_start_qp(t.qp, a.aq[idx]) : -1;
    MbInfo cand;
    memset(&cand, 0, sizeof(cand));
    bool i4 = false;
    const bool aTR = aT && mbx + 1 < a.mb_w;
    // open-loop source samples, MB-relative (the pre-pass predicts from the source)
    auto src_smp = [&](int x, int y) __attribute__((always_inline)) -> int {
        return a.src.y[(size_t)(mby * 16 + y) * a.stride_y + mbx * 16 + x];
    };
    if (a.intra4x4) {
        // Intra4x4 decision (h264_mb.h i4_decide): the SAD of every mode of every block in
        // parallel (quad = block), then the predicted-mode costs in decoding order
        const int q = l >> 2;
        int* sads = reinterpret_cast<int*>(S.coef);   // 16 x 9, before any levels are written
        uint8_t* refs = S.ry;                          // 16 x 13 reference samples (quad = block)
        for (int k = r; k < 13; k += 4) refs[q * 13 + k] = (uint8_t)i4_ref_sample(src_smp, q, aT, aL, aTR, k);
        wave_sync();
        const I4RefView ref{refs + q * 13, i4_has_top(q, aT), i4_has_left(q, aL)};
        for (int m = 0; m < 9; m++) {
            int sad = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) sad += sk_abs(src_l[j] - i4_pred_px(m, ref, j, r));
            sad = quad_sum(sad);
            if (r == 0) sads[q * 9 + m] = i4_mode_ok(m, ref.hasT, ref.hasL) ? sad : -1;
        }
        wave_sync();
        const int lam = i4_lambda(t.qp);
        int total = 0;
        for (int b = 0; b < 16; b++) {
            // i4_decide: neighbours in other MBs count as DC (2) when available
            const int bx = blk_x(b), by = blk_y(b);
            const int ma = bx > 0 ? i4_mode(cand, blk_from_xy(bx - 1, by)) : (aL ? 2 : -1);
            const int mt = by > 0 ? i4_mode(cand, blk_from_xy(bx, by - 1)) : (aT ? 2 : -1);
            const int pm = i4_predicted(ma, mt);
            int best = 0x7fffffff, bm = I4_DC;
            for (int m = 0; m < 9; m++) {
                const int sd = sads[b * 9 + m];
                if (sd < 0) continue;
                const int cost = sd + lam * (m == pm ? 1 : 4);
                if (cost < best) { best = cost; bm = m; }
            }
            set_i4_mode(cand, b, bm);
            total += best;
        }
        i4 = i4_wins(total, sad16, t.qp);
        wave_sync();
    }
    MbInfo mb;
    memset(&mb, 0, sizeof(mb));
    int qp;
    if (i4) {
        mb.type = MB_I4x4;
        mb.chroma_mode = (uint8_t)cmode;
        mb.i4lo = cand.i4lo;
        mb.i4hi = cand.i4hi;
        int rec_l[4], rec_c[4];
        qp = code_mb_i4(src_smp, src_l, src_c, pred_c, start >= 0 ? start : t.qp, t.qp, aT, aL, aTR, S, mb, rec_l,
                        rec_c, nullptr, T);
    } else {
        int rec_l[4], rec_c[4];
        qp = code_mb(src_l, pred_l, src_c, pred_c, t.qp, true, S, mb, rec_l, rec_c, nullptr, T, nullptr, 0, start,
                     true);
    }
    if (l == 0) {
        MbInfo o;
        memset(&o, 0, sizeof(o));
        o.type = i4 ? MB_I4x4 : MB_I16x16;
        o.i16_mode = (uint8_t)mode;
        o.chroma_mode = (uint8_t)cmode;
        o.qp = (uint8_t)qp;
        o.i4lo = cand.i4lo;
        o.i4hi = cand.i4hi;
        a.mbs[idx] = o;
    }
}

// ---------------------------------------------------------------------------
// K5+K6 intra: one workgroup per I slice, wave w codes MB row w, MB x at step
// t = x + 2w (wavefront); neighbour edges travel through LDS rings. Modes and the
// start QP come from k_intra_prep, so a step is prediction, quantisation and
// reconstruction only; the next step's source rows and decisions are loaded ahead.
constexpr int kMaxRows = 16;
struct IntraEdges {
    uint8_t bot_y[kMaxRows][4][16];      // bottom luma row of MB (row, x mod 4)
    uint8_t bot_c[kMaxRows][4][2][8];
    uint8_t right_y[kMaxRows][16];       // right luma column of the previous MB in the row
    uint8_t right_c[kMaxRows][2][8];
};

// Source samples and pre-pass decisions of one MB, staged in LDS by the producer wave.
struct IntraSrc {
    uint32_t y[64];      // 16 rows x 16 px (row-major, 4 words per row)
    uint32_t c[32];      // Cb 8x8 then Cr 8x8 (2 words per row)
    int mode, cmode, qp, i4;   // i4: coded as Intra4x4 (pre-pass decision)
    uint32_t i4m[2];     // its 16 modes (MbInfo i4lo / i4hi)
};
constexpr int kIntraRing = 4;   // MB slots per row in flight (producer runs 2 steps ahead)

// One workgroup of MAXROWS coding waves + 1 producer wave per I slice. Coding wave w
// owns MB row w and codes MB x at step x + 2w (wavefront, neighbour edges through
// LDS). The producer wave loads the source rows of the MBs due two steps later into
// an LDS ring, so a coding wave never issues a global load: its only memory waits
// are LDS, and its global stores (reconstruction, levels, MB info) are never waited on.
template <int MAXROWS>
__global__ __launch_bounds__(64 * (MAXROWS + 1)) void k_code_intra(FrameArgs a) {
    if (a.gate && *a.gate == 0) return;   // CBR second pass not needed
    __shared__ MbScratch Sw[MAXROWS];
    __shared__ IntraEdges E;
    __shared__ IntraSrc R[MAXROWS][kIntraRing];
    __shared__ uint8_t zero16[16];
    __shared__ CavlcTables T;
    int s = blockIdx.x;
    const SliceTask t = a.tasks[s];
    // block-uniform: P/skipped slices and K5 sub-sliced ones (k_code_intra_sub) leave before the table load
    if (t.final_action != ACT_I || split_i(a, t)) return;
#ifdef SK_STAMPS
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c_start = __builtin_amdgcn_s_memtime();
    if (a.dbg && blockIdx.x == 0 && (threadIdx.x & 63) == 0)   // HW_ID of each wave (SIMD placement)
        a.dbg[1024 + 128 + (threadIdx.x >> 6)] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
    if (threadIdx.x < 16) zero16[threadIdx.x] = 0;
    load_cavlc_tables(T, a.cavlc_tabs);
    int w = threadIdx.x >> 6;
    int l = lane_id();
    const int rows = t.num_rows;
    const int steps = a.mb_w + 2 * (rows - 1);
    const bool producer = w == MAXROWS;
    // producer: stage the MBs coded at step `st` (MB x = st - 2*row of every row)
    auto produce = [&](int st) {
        for (int row = 0; row < rows; row++) {
            const int x = st - 2 * row;
            if (x < 0 || x >= a.mb_w) continue;
            const int my = t.first_row + row;
            IntraSrc& d = R[row][x & (kIntraRing - 1)];
            // luma: lane l -> row l >> 2, word l & 3
            d.y[l] = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)(my * 16 + (l >> 2)) * a.stride_y + x * 16 +
                                                        4 * (l & 3));
            if (l < 32) {   // chroma: comp l >> 4, row (l >> 1) & 7, word l & 1
                const uint8_t* P = (l >> 4) ? a.src.v : a.src.u;
                d.c[l] = *reinterpret_cast<const uint32_t*>(P + (size_t)(my * 8 + ((l >> 1) & 7)) * a.stride_c +
                                                            x * 8 + 4 * (l & 1));
            }
            if (l == 0) {
                const MbInfo pre = a.mbs[my * a.mb_w + x];
                d.mode = pre.i16_mode;
                d.cmode = pre.chroma_mode;
                d.qp = pre.qp;
                d.i4 = pre.type == MB_I4x4;
                d.i4m[0] = pre.i4lo;
                d.i4m[1] = pre.i4hi;
            }
        }
    };
    if (producer) {
        __builtin_amdgcn_s_setprio(2);
        produce(0);
        produce(1);
    }
    __syncthreads();
#ifdef SK_STAMPS
    const unsigned long long c_loop = __builtin_amdgcn_s_memtime();
#endif
    if (!producer) __builtin_amdgcn_s_setprio(3);   // the chain's waves issue first on a shared SIMD
    MbScratch& S = Sw[producer ? 0 : w];
    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    const int lx = blk_x(b) * 4, ly = blk_y(b) * 4 + r;
    const int clx = (cb & 1) * 4, cly = (cb >> 1) * 4 + r;
    const int mby = t.first_row + w;
    for (int step = 0; step < steps; step++) {
        if (producer) {
            if (step + 2 < steps) produce(step + 2);
        } else {
            const int mbx = step - 2 * w;
            const bool active = w < rows && mbx >= 0 && mbx < a.mb_w;
            if (active) {
                STAMP(step, 0);
                const IntraSrc& in = R[w][mbx & (kIntraRing - 1)];
                const uint32_t sw = in.y[ly * 4 + (lx >> 2)];
                const uint32_t csw = in.c[comp * 16 + cly * 2 + (clx >> 2)];
                // wave-uniform decisions (scalar registers / branches)
                const int mode = __builtin_amdgcn_readfirstlane(in.mode);
                const int cmode = __builtin_amdgcn_readfirstlane(in.cmode);
                const int start_qp = __builtin_amdgcn_readfirstlane(in.qp);
                const int idx = mby * a.mb_w + mbx;
                const bool aT = w > 0, aL = mbx > 0;
                // neighbour samples of this MB into the wave's nb layout (LDS)
                uint8_t* nb = S.nb;
                {
                    int v = 0;
                    if (l < 16) v = aT ? E.bot_y[w - 1][mbx & 3][l] : 0;
                    else if (l < 32) v = aL ? E.right_y[w][l - 16] : 0;
                    else if (l < 48) v = aT ? E.bot_c[w - 1][mbx & 3][(l >> 3) & 1][l & 7] : 0;
                    else v = aL ? E.right_c[w][(l >> 3) & 1][l & 7] : 0;
                    nb[l] = (uint8_t)v;
                }
                const int tl = (aT && aL) ? E.bot_y[w - 1][(mbx - 1) & 3][15] : 0;
                const int ctl[2] = {(aT && aL) ? E.bot_c[w - 1][(mbx - 1) & 3][0][7] : 0,
                                    (aT && aL) ? E.bot_c[w - 1][(mbx - 1) & 3][1][7] : 0};
                wave_sync();
                int src_l[4], src_c[4];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    src_l[j] = (sw >> (8 * j)) & 255;
                    src_c[j] = (csw >> (8 * j)) & 255;
                }
                const bool is_i4 = __builtin_amdgcn_readfirstlane(in.i4) != 0;
                int pred_l[4], pred_c[4];
                intra_pred_lanes(is_i4 ? 2 : mode, cmode, nb, tl, ctl, aT, aL, pred_l, pred_c);
                STAMP(step, 2);
                MbInfo mb;
                memset(&mb, 0, sizeof(mb));
                mb.chroma_mode = (uint8_t)cmode;
                int rec_l[4], rec_c[4];
                if (is_i4) {
                    const bool aTR = aT && mbx + 1 < a.mb_w;
                    if (l < 4) S.nbtr[l] = aTR ? E.bot_y[w - 1][(mbx + 1) & 3][l] : 0;
                    const uint32_t m0 = __builtin_amdgcn_readfirstlane(in.i4m[0]);
                    const uint32_t m1 = __builtin_amdgcn_readfirstlane(in.i4m[1]);
                    mb.i4lo = m0;
                    mb.i4hi = m1;
                    mb.type = MB_I4x4;
                    wave_sync();
                    // reconstruction so far (S.ry) inside the MB, LDS edges outside
                    auto smp = [&](int x, int y) __attribute__((always_inline)) -> int {
                        if (y >= 0 && x >= 0) return S.ry[y * 16 + x];
                        if (y < 0) return x < 0 ? tl : (x < 16 ? (int)nb[x] : (int)S.nbtr[x - 16]);
                        return nb[16 + y];
                    };
                    code_mb_i4(smp, src_l, src_c, pred_c, start_qp, t.qp, aT, aL, aTR, S, mb, rec_l, rec_c,
                               a.coefs + (size_t)idx * kCoefPerMb, T);
                } else {
                    mb.type = MB_I16x16;
                    mb.i16_mode = (uint8_t)mode;
                    code_mb(src_l, pred_l, src_c, pred_c, t.qp, true, S, mb, rec_l, rec_c,
                            a.coefs + (size_t)idx * kCoefPerMb, T, a.dbg, step, start_qp);
                }
                STAMP(step, 6);
                // edges for the neighbours first (LDS), then the global stores
                wave_sync();
                if (ly == 15)
                    for (int j = 0; j < 4; j++) E.bot_y[w][mbx & 3][lx + j] = (uint8_t)rec_l[j];
                if (lx + 3 == 15) E.right_y[w][ly] = (uint8_t)rec_l[3];
                if (l < 32) {
                    if (cly == 7)
                        for (int j = 0; j < 4; j++) E.bot_c[w][mbx & 3][comp][clx + j] = (uint8_t)rec_c[j];
                    if (clx + 3 == 7) E.right_c[w][comp][cly] = (uint8_t)rec_c[3];
                }
                const int px = mbx * 16 + lx, py = mby * 16 + ly;
                uint32_t rw = (uint32_t)rec_l[0] | ((uint32_t)rec_l[1] << 8) | ((uint32_t)rec_l[2] << 16) |
                              ((uint32_t)rec_l[3] << 24);
                *reinterpret_cast<uint32_t*>(a.rec.y + (size_t)py * a.stride_y + px) = rw;
                if (l < 32) {
                    uint8_t* crp = comp ? a.rec.v : a.rec.u;
                    uint32_t cw = (uint32_t)rec_c[0] | ((uint32_t)rec_c[1] << 8) | ((uint32_t)rec_c[2] << 16) |
                                  ((uint32_t)rec_c[3] << 24);
                    *reinterpret_cast<uint32_t*>(crp + (size_t)(mby * 8 + cly) * a.stride_c + mbx * 8 + clx) = cw;
                }
                if (l == 0) {
                    for (int i = 0; i < 24; i++) mb.nnz[i] = S.nnz[i];
                    a.mbs[idx] = mb;
                    a.me[idx].mvx = 0;
                    a.me[idx].mvy = 0;
                    a.me[idx].ref = 0;
                    a.me[idx].fx = a.me[idx].fy = 0;
                }
                STAMP(step, 7);
            }
        }
        __syncthreads();
        if (w == 0) STAMP(step, 8);
    }
#ifdef SK_STAMPS
    if (a.dbg && threadIdx.x == 0 && blockIdx.x < 32) {   // per-slice span (100 MHz realtime)
        a.dbg[1024 + 2 * blockIdx.x] = t_start;
        a.dbg[1024 + 2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        if (blockIdx.x < 32) a.dbg[1024 + 64 + 2 * blockIdx.x] = __builtin_amdgcn_s_memtime() - c_start;
        if (blockIdx.x == SK_STAMP_BLOCK) {
            a.dbg[1024 + 200] = c_start;
            a.dbg[1024 + 201] = __builtin_amdgcn_s_memtime();
            a.dbg[1024 + 202] = c_loop;
            a.dbg[1024 + 203] = steps;
        }
        if (blockIdx.x < 32) a.dbg[1024 + 64 + 2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
#endif
}

// ---------------------------------------------------------------------------
// K5+K6 intra of sub-sliced I slices (h264_encoder.h intra_split): one wave per
// sub-slice of kIntraSubMbs MBs. No MB has its top neighbour in its sub-slice, so a
// wave's chain is its MBs in raster order, predicting from the left neighbour's right
// column only (kept in the wave's LDS), and the sub-slices of every slice run in
// parallel (1080p: 17 slices x 12 sub-slices = 204 waves of at most 40 steps, where
// k_code_intra's wavefront is 17 chains of 126 steps). Modes and start QPs come from
// k_intra_prep; the next MB's source samples and decisions are loaded before the
// current MB is coded.
__global__ __launch_bounds__(256) void k_code_intra_sub(FrameArgs a) {
    if (a.gate && *a.gate == 0) return;   // CBR second pass not needed
    __shared__ MbScratch Sw[4];
    __shared__ uint8_t right_y[4][16];
    __shared__ uint8_t right_c[4][2][8];
    __shared__ CavlcTables T;
    const int w = threadIdx.x >> 6, l = lane_id();
    const int gw = blockIdx.x * 4 + w;
    const int s = gw / a.nal_per_slice, j = gw % a.nal_per_slice;
    bool mine = false;
    SliceTask t;
    if (s < a.num_slices) {
        t = a.tasks[s];
        mine = split_i(a, t) && j < intra_sub_count(t.num_rows * a.mb_w);
    }
    if (!__syncthreads_or(mine)) return;
    load_cavlc_tables(T, a.cavlc_tabs);
    __syncthreads();
    if (!mine) return;
    MbScratch& S = Sw[w];
    const int b = l >> 2, r = l & 3;
    const int cl = l & 31, comp = cl >> 4, cb = (cl >> 2) & 3;
    const int lx = blk_x(b) * 4, ly = blk_y(b) * 4 + r;
    const int clx = (cb & 1) * 4, cly = (cb >> 1) * 4 + r;
    const int first = t.first_row * a.mb_w;
    const int k0 = j * kIntraSubMbs, k1 = sk_min(t.num_rows * a.mb_w, k0 + kIntraSubMbs);
    const uint8_t* cplane = comp ? a.src.v : a.src.u;
    // source samples + pre-pass decisions of MB k (lane layout of code_mb)
    auto fetch = [&](int k, uint32_t& sw, uint32_t& csw, MbInfo& pre) {
        const int idx = first + k, mbx = idx % a.mb_w, mby = idx / a.mb_w;
        sw = *reinterpret_cast<const uint32_t*>(a.src.y + (size_t)(mby * 16 + ly) * a.stride_y + mbx * 16 + lx);
        csw = *reinterpret_cast<const uint32_t*>(cplane + (size_t)(mby * 8 + cly) * a.stride_c + mbx * 8 + clx);
        pre = a.mbs[idx];
    };
    uint32_t sw, csw;
    MbInfo pre;
    fetch(k0, sw, csw, pre);
    const int zc[2] = {0, 0};
    for (int k = k0; k < k1; k++) {
        const int idx = first + k, mbx = idx % a.mb_w, mby = idx / a.mb_w;
        const bool aL = mbx > 0 && k > k0;
        const int mode = __builtin_amdgcn_readfirstlane(pre.i16_mode);
        const int cmode = __builtin_amdgcn_readfirstlane(pre.chroma_mode);
        const int start_qp = __builtin_amdgcn_readfirstlane(pre.qp);
        // k_intra_prep's choice for this MB: read before `pre` is overwritten by the prefetch
        const bool is_i4 = __builtin_amdgcn_readfirstlane((int)pre.type) == MB_I4x4;
        const uint32_t m0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)pre.i4lo);
        const uint32_t m1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)pre.i4hi);
        int src_l[4], src_c[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            src_l[q] = (sw >> (8 * q)) & 255;
            src_c[q] = (csw >> (8 * q)) & 255;
        }
        if (k + 1 < k1) fetch(k + 1, sw, csw, pre);   // in flight while this MB is coded
        // neighbours: top unavailable (zeros), left = the previous MB's right column
        uint8_t* nb = S.nb;
        {
            int v = 0;
            if (l >= 16 && l < 32) v = aL ? right_y[w][l - 16] : 0;
            else if (l >= 48) v = aL ? right_c[w][(l >> 3) & 1][l & 7] : 0;
            nb[l] = (uint8_t)v;
        }
        wave_sync();
        int pred_l[4], pred_c[4];
        intra_pred_lanes(is_i4 ? 2 : mode, cmode, nb, 0, zc, false, aL, pred_l, pred_c);
        MbInfo mb;
        memset(&mb, 0, sizeof(mb));
        mb.chroma_mode = (uint8_t)cmode;
        int rec_l[4], rec_c[4];
        if (is_i4) {   // I_NxN: blocks in decoding order from the reconstruction so far and the left column
            mb.type = MB_I4x4;
            mb.i4lo = m0;
            mb.i4hi = m1;
            auto smp = [&](int x, int y) __attribute__((always_inline)) -> int {
                if (y >= 0 && x >= 0) return S.ry[y * 16 + x];
                if (y < 0) return 0;   // no top / top-right neighbour inside a sub-slice
                return nb[16 + y];
            };
            code_mb_i4(smp, src_l, src_c, pred_c, start_qp, t.qp, false, aL, false, S, mb, rec_l, rec_c,
                       a.coefs + (size_t)idx * kCoefPerMb, T);
        } else {
            mb.type = MB_I16x16;
            mb.i16_mode = (uint8_t)mode;
            code_mb(src_l, pred_l, src_c, pred_c, t.qp, true, S, mb, rec_l, rec_c, a.coefs + (size_t)idx * kCoefPerMb,
                    T, nullptr, 0, start_qp);
        }
        wave_sync();
        if (lx + 3 == 15) right_y[w][ly] = (uint8_t)rec_l[3];
        if (l < 32 && clx + 3 == 7) right_c[w][comp][cly] = (uint8_t)rec_c[3];
        const int px = mbx * 16 + lx, py = mby * 16 + ly;
        *reinterpret_cast<uint32_t*>(a.rec.y + (size_t)py * a.stride_y + px) =
            (uint32_t)rec_l[0] | ((uint32_t)rec_l[1] << 8) | ((uint32_t)rec_l[2] << 16) | ((uint32_t)rec_l[3] << 24);
        if (l < 32) {
            uint8_t* crp = comp ? a.rec.v : a.rec.u;
            *reinterpret_cast<uint32_t*>(crp + (size_t)(mby * 8 + cly) * a.stride_c + mbx * 8 + clx) =
                (uint32_t)rec_c[0] | ((uint32_t)rec_c[1] << 8) | ((uint32_t)rec_c[2] << 16) | ((uint32_t)rec_c[3] << 24);
        }
        if (l == 0) {
            for (int i = 0; i < 24; i++) mb.nnz[i] = S.nnz[i];
            a.mbs[idx] = mb;
            a.me[idx].mvx = 0;
            a.me[idx].mvy = 0;
            a.me[idx].ref = 0;
            a.me[idx].fx = a.me[idx].fy = 0;
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// K8: CAVLC, one wave per coded MB.
// 4 waves per workgroup, one MB per wave (tables shared). Lanes 0..26 each code one
// residual block ONCE into a private LDS stage; a wave scan of the bit counts gives
// the offsets and the staged words are OR-ed into the MB's bit buffer.
constexpr int kCavlcStageWords = 24;   // 768 bits per block; longer blocks are re-coded in place
__global__ __launch_bounds__(256) void k_cavlc(FrameArgs a) {
    if (a.gate && *a.gate == 0) return;   // CBR second pass not needed
    __shared__ uint32_t bits_w[4][kMbSlotBytes / 4];
    __shared__ uint32_t stage_w[4][27 * kCavlcStageWords];
    __shared__ int16_t coef_w[4][kCoefPerMb];
    __shared__ MbInfo mb_w[4];   // the MB's info in LDS: nnz[] is indexed per lane (a private copy would spill)
    __shared__ CavlcTables T;
    load_cavlc_tables(T, a.cavlc_tabs);
    __syncthreads();
    uint32_t* bits = bits_w[threadIdx.x >> 6];
    int16_t* coef = coef_w[threadIdx.x >> 6];
    int nmb = a.mb_w * a.mb_h;
    int idx = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    if (idx >= nmb) return;
    int mbx = idx % a.mb_w, mby = idx / a.mb_w;
    int s = mby / a.rows_per_slice;
    const SliceTask t = a.tasks[s];
    if (t.final_action != ACT_P && t.final_action != ACT_I) return;
    int l = lane_id();
    MbInfo& mb = mb_w[threadIdx.x >> 6];
    if (l < (int)(sizeof(MbInfo) / 4))
        reinterpret_cast<uint32_t*>(&mb)[l] = reinterpret_cast<const uint32_t*>(a.mbs + idx)[l];
    wave_sync();
    if (mb.type == MB_P_SKIP) {
        if (l == 0) a.mb_nbits[idx] = 0;
        return;
    }
    bool p_slice = t.final_action == ACT_P;
    int first = t.first_row * a.mb_w;
    if (split_i(a, t)) first += ((idx - first) / kIntraSubMbs) * kIntraSubMbs;   // K5: the MB's sub-slice
    // mb_skip_run: skipped MBs since the previous coded MB of the slice
    int run = 0;
    if (p_slice) {
        int j = idx - 1;
        while (j >= first) {
            int base = j - 63;
            int m = base + l;
            bool coded = m >= first && a.mbs[m].type != MB_P_SKIP;
            unsigned long long msk = __ballot(coded);
            if (msk) {
                int hi = 63 - __clzll(msk);
                run += j - (base + hi);
                break;
            }
            run += j - sk_max(base, first) + 1;
            j = base - 1;
        }
    }
    // QP predictor: QP of the previous MB that carried mb_qp_delta
    int qp_prev = t.qp;
    {
        int j = idx - 1;
        while (j >= first) {
            int base = j - 63;
            int m = base + l;
            bool has = m >= first && mb_has_qp_delta(a.mbs[m]);
            unsigned long long msk = __ballot(has);
            if (msk) {
                int hi = 63 - __clzll(msk);
                qp_prev = a.mbs[base + hi].qp;
                break;
            }
            j = base - 1;
        }
    }
    for (int i = l; i < kMbSlotBytes / 4; i += 64) bits[i] = 0;
    uint32_t* stage_all = stage_w[threadIdx.x >> 6];
    for (int i = l; i < 27 * kCavlcStageWords; i += 64) stage_all[i] = 0;
    const int16_t* gc = a.coefs + (size_t)idx * kCoefPerMb;
    for (int i = l; i < kCoefPerMb / 2; i += 64)
        reinterpret_cast<uint32_t*>(coef)[i] = reinterpret_cast<const uint32_t*>(gc)[i];
    wave_sync();
    MbNeighbours nb;
    nb.left = mbx > 0 && idx - 1 >= first ? &a.mbs[idx - 1] : nullptr;
    nb.top = mby > t.first_row && idx - a.mb_w >= first ? &a.mbs[idx - a.mb_w] : nullptr;
    int hdr_bits = 0;
    if (l == 0) {
        AtomicBitWriter w{bits, 0};
        if (p_slice) put_ue(w, (uint32_t)run);
        int dq = mb_has_qp_delta(mb) ? (int)mb.qp - qp_prev : 0;
        write_mb_header(w, mb, p_slice, dq, p_slice ? t.num_refs : 1, nb);
        hdr_bits = (int)w.pos;
    }
    hdr_bits = __shfl(hdr_bits, 0);
    // residual block list (bitstream order)
    int cbp_l = mb.cbp & 15, cbp_c = (mb.cbp >> 4) & 3;
    bool i16 = mb.type == MB_I16x16;
    const int16_t* bc = nullptr;
    int maxn = 0, nc = 0;
    bool act = false;
    if (l == 0) {
        if (i16) { act = true; bc = coef + kCoefLumaDC; maxn = 16; nc = luma_nc(mb, nb, 0); }
    } else if (l <= 16) {
        int blk = l - 1;
        if (i16) {
            if (cbp_l) { act = true; bc = coef + kCoefLuma + blk * 16 + 1; maxn = 15; }
        } else if (cbp_l & (1 << (blk >> 2))) {
            act = true; bc = coef + kCoefLuma + blk * 16; maxn = 16;
        }
        if (act) nc = luma_nc(mb, nb, blk);
    } else if (l <= 18) {
        if (cbp_c) { act = true; bc = coef + kCoefChromaDC + (l - 17) * 4; maxn = 4; nc = -1; }
    } else if (l <= 26) {
        if (cbp_c == 2) {
            int k = l - 19, c = k >> 2, bb = k & 3;
            act = true; bc = coef + kCoefChromaAC + (c * 4 + bb) * 16 + 1; maxn = 15;
            nc = chroma_nc(mb, nb, c, bb);
        }
    }
    int nbits = 0;
    uint32_t* stage = stage_all + (l < 27 ? l : 0) * kCavlcStageWords;
    StageBitWriter sw{stage, 0, kCavlcStageWords * 32, false};
    if (act) {
        cavlc_block(sw, bc, maxn, nc, T);
        nbits = (int)sw.pos;
    }
    int incl = wave_incl_scan(nbits);
    int off = hdr_bits + incl - nbits;
    if (act) {
        if (!sw.ovf) {
            const uint32_t sh = (uint32_t)off & 31;
            uint32_t wi = (uint32_t)off >> 5;
            for (int k = 0; k < (nbits + 31) >> 5; k++, wi++) {
                const uint32_t v = stage[k];   // zero past nbits
                atomicOr(&bits[wi], v >> sh);
                const uint32_t lo = sh ? v << (32 - sh) : 0u;
                if (lo) atomicOr(&bits[wi + 1], lo);
            }
        } else {
            AtomicBitWriter w{bits, (uint32_t)off};
            cavlc_block(w, bc, maxn, nc, T);
        }
    }
    int total = hdr_bits + __shfl(incl, 63);
    wave_sync();
    int nwords = (total + 31) >> 5;
    uint32_t* dst = a.mb_bits + (size_t)idx * (kMbSlotBytes / 4);
    for (int i = l; i < nwords; i += 64) dst[i] = bits[i];
    if (l == 0) a.mb_nbits[idx] = total;
}

// ---------------------------------------------------------------------------
// K9: slice assembly (one 256-thread workgroup per coded slice).
// ---------------------------------------------------------------------------
// K9: slice assembly, tile-parallel.
//   k_slice_scan  one workgroup per slice: slice header, exclusive scan of the MB
//                 bit counts -> per-MB bit offsets, trailing mb_skip_run + stop
//                 bit, packet prefix (stripe header, SPS/PPS on IDR, start code,
//                 NAL header) written straight into the host-mapped slot
//   k_mb_concat   one wave per MB: shifts its CAVLC words into the slice RBSP
//                 (plain stores; atomicOr only on the two edge words it shares)
//   k_ep_nz / k_ep_count / k_ep_write   4 KiB tiles of every slice in parallel:
//                 emulation prevention (7.4.1) — a 0x03 goes before byte i iff
//                 b_i <= 3 and the zero run z(i) right before i is even and >= 2,
//                 which only depends on the input bytes; a tile needs the last
//                 non-zero byte before it (prefix max of k_ep_nz) and the number
//                 of insertions before it (prefix sum of k_ep_count). k_ep_write
//                 stages its output in LDS, streams it to host memory with 16-byte
//                 stores and self-cleans the RBSP words it consumed.
constexpr int kTile = 4096;

__global__ __launch_bounds__(256) void k_slice_scan(FrameArgs a) {
    if (a.gate && *a.gate == 0) return;   // CBR second pass not needed
    __shared__ uint32_t hdr[32];
    __shared__ int wave_tot[5];
    __shared__ int sh_misc[4];
    // one workgroup per NAL slot: slice s, sub-slice j (K5; j = 0 is the whole slice otherwise)
    const int nal = blockIdx.x, s = nal / a.nal_per_slice, j = nal % a.nal_per_slice, tid = threadIdx.x;
    const SliceTask task = a.tasks[s];
    const int fin = task.final_action;
    int* info = a.slice_info + 4 * nal;
    const int nn = slice_nals(a, task);
    if (j >= nn) {
        if (tid == 0) {
            info[0] = 0;
            info[1] = 0;
            if (j == 0) a.host_size[s] = 0;
        }
        return;
    }
    const int snmb = task.num_rows * a.mb_w;
    const int k0 = nn > 1 ? j * kIntraSubMbs : 0;
    const int nmb = nn > 1 ? sk_min(snmb, k0 + kIntraSubMbs) - k0 : snmb;
    const int first = task.first_row * a.mb_w + k0;
    uint32_t* rbsp = nal_rbsp(a, s, j);
    const bool intra = fin == ACT_I;
    const bool idr = intra && task.idr_on_intra;
    if (tid < 32) hdr[tid] = 0;
    if (tid == 0) sh_misc[1] = -1;
    __syncthreads();
    if (tid == 0) {
        AtomicBitWriter w{hdr, 0};
        SliceHeaderParams h;
        h.first_mb = (a.fullframe ? task.first_row * a.mb_w : 0) + k0;
        h.slice_type = intra ? 2 : 0;
        h.idr = idr;
        h.frame_num = idr ? 0 : task.frame_num;
        h.idr_pic_id = task.idr_pic_id;
        h.slice_qp = task.qp;
        h.deblock = slice_deblock(a.deblock, task);
        h.num_refs = intra ? 1 : task.num_refs;
        write_slice_header(w, h);
        if (fin == ACT_SKIPALL) put_ue(w, (uint32_t)nmb);
        sh_misc[0] = (int)w.pos;
    }
    const int per = (nmb + 255) / 256;
    const int m0 = sk_min(nmb, tid * per), m1 = sk_min(nmb, m0 + per);
    int local = 0, last_coded = -1;
    if (fin != ACT_SKIPALL)
        for (int m = m0; m < m1; m++) {
            const int nb = a.mb_nbits[first + m];
            local += nb;
            if (nb > 0) last_coded = m;
        }
    if (last_coded >= 0) atomicMax(&sh_misc[1], last_coded);
    int total;
    const int excl = block_excl_scan<4>(local, wave_tot, &total);
    const int hb = sh_misc[0];
    if (fin != ACT_SKIPALL) {
        int off = hb + excl;
        for (int m = m0; m < m1; m++) {
            a.mb_off[first + m] = off;
            off += a.mb_nbits[first + m];
        }
    }
    if (tid < 32 && tid * 32 < hb) atomicOr(&rbsp[tid], hdr[tid]);  // last header word is shared with MB 0
    if (tid == 0) {
        AtomicBitWriter w{rbsp, (uint32_t)(hb + total)};
        if (fin == ACT_P) {
            const int trailing = nmb - 1 - sh_misc[1];
            if (trailing > 0) put_ue(w, (uint32_t)trailing);
        }
        w.put(1, 1);  // rbsp_stop_one_bit
        info[0] = (int)((w.pos + 7) >> 3);
        if (j > 0) {   // start code + NAL header: written by k_ep_write once the NALs before it are sized
            info[1] = 5;
        } else {       // packet prefix, written directly into the host-mapped slot
            uint8_t* slot = a.host_out + (size_t)s * a.out_slot_bytes;
            int p = 0;
            if (!a.fullframe) {
                const int y = task.first_row * 16;
                const int h = sk_min(a.H, (task.first_row + task.num_rows) * 16) - y;
                const int fid = a.frame_params_dev[0];
                uint8_t pre[10] = {0x04, (uint8_t)(idr ? 1 : 0), (uint8_t)(fid >> 8), (uint8_t)fid, (uint8_t)(y >> 8),
                                   (uint8_t)y, (uint8_t)(a.W >> 8), (uint8_t)a.W, (uint8_t)(h >> 8), (uint8_t)h};
                for (int i = 0; i < 10; i++) slot[i] = pre[i];
                p = 10;
                if (idr) {
                    const int len = a.param_set_len[s];
                    const uint8_t* ps = a.param_sets + (size_t)s * a.param_set_stride;
                    for (int i = 0; i < len; i++) slot[p + i] = ps[i];
                    p += len;
                }
            }
            slot[p++] = 0; slot[p++] = 0; slot[p++] = 0; slot[p++] = 1;
            slot[p++] = idr ? 0x65 : 0x41;
            info[1] = p;
        }
    }
}

__global__ __launch_bounds__(256) void k_mb_concat(FrameArgs a) {
    const int w = threadIdx.x >> 6, l = lane_id();
    const int mb = blockIdx.x * 4 + w;
    if (mb >= a.mb_w * a.mb_h) return;
    const int s = (mb / a.mb_w) / a.rows_per_slice;
    const SliceTask& task = a.tasks[s];
    const int fin = task.final_action;
    if (fin == ACT_NONE || fin == ACT_SKIPALL) return;
    const int nb = a.mb_nbits[mb];
    if (nb <= 0) return;
    const int sub = split_i(a, task) ? (mb - task.first_row * a.mb_w) / kIntraSubMbs : 0;   // K5 NAL of the MB
    const int p = a.mb_off[mb];
    const int w0 = p >> 5, w1 = (p + nb - 1) >> 5, sh = p & 31;
    const int nw = (nb + 31) >> 5;
    const uint32_t lastmask = (nb & 31) ? ~0u << (32 - (nb & 31)) : ~0u;
    const uint32_t* src = a.mb_bits + (size_t)mb * (kMbSlotBytes / 4);
    uint32_t* dst = nal_rbsp(a, s, sub);
    for (int j = w0 + l; j <= w1; j += 64) {
        const int k = j - w0;
        uint32_t lo = k < nw ? src[k] : 0u;
        if (k == nw - 1) lo &= lastmask;
        uint32_t v;
        if (sh == 0) {
            v = lo;
        } else {
            uint32_t hi = 0u;
            if (k >= 1) {
                hi = src[k - 1];
                if (k - 1 == nw - 1) hi &= lastmask;
            }
            v = (lo >> sh) | (k >= 1 ? hi << (32 - sh) : 0u);
        }
        if (j == w0 || j == w1) {
            if (v) atomicOr(&dst[j], v);
        } else {
            dst[j] = v;
        }
    }
}

__device__ __forceinline__ uint8_t rbsp_byte(uint32_t word, int q) { return (uint8_t)(word >> (24 - 8 * q)); }

// EP kernels: grid (tile, slice); a block loops over the slice's NALs (one for every
// slice but the sub-sliced I ones, so P pictures launch no per-NAL blocks).
__global__ __launch_bounds__(256) void k_ep_nz(FrameArgs a) {
    __shared__ int red[4];
    const int s = blockIdx.y, t = blockIdx.x, tid = threadIdx.x;
    const int nn = slice_nals(a, a.tasks[s]);
    for (int j = 0; j < nn; j++) {
    const int nal = s * a.nal_per_slice + j;
    const int n = a.slice_info[4 * nal];
    const int t0 = t * kTile;
    if (t0 >= n) continue;
    const uint32_t* rbsp = nal_rbsp(a, s, j);
    const int i0 = t0 + tid * 16;
    int lastnz = -1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int iq = i0 + 4 * q;
        const uint32_t wd = iq < n ? rbsp[iq >> 2] : 0u;
#pragma unroll
        for (int b = 0; b < 4; b++)
            if (iq + b < n && rbsp_byte(wd, b)) lastnz = iq + b;
    }
    for (int o = 32; o > 0; o >>= 1) lastnz = max(lastnz, __shfl_down(lastnz, o));
    if (lane_id() == 0) red[tid >> 6] = lastnz;
    __syncthreads();
    if (tid == 0) a.tile_nz[nal * a.max_tiles + t] = max(max(red[0], red[1]), max(red[2], red[3]));
    __syncthreads();
    }
}

// Per-thread EP decisions for 16 bytes starting at i0; `carry` = last non-zero
// byte index before the tile. Returns the insertion count; bytes and insertion
// mask through the out parameters.
__device__ __forceinline__ int ep_thread(const uint32_t* rbsp, int n, int t0, int carry, int* scan_lds,
                                         uint8_t* by, uint32_t* insmask) {
    const int tid = threadIdx.x, wv = tid >> 6, ln = tid & 63;
    const int i0 = t0 + tid * 16;
    int lastnz = -1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int iq = i0 + 4 * q;
        const uint32_t wd = iq < n ? rbsp[iq >> 2] : 0u;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            by[4 * q + j] = rbsp_byte(wd, j);
            if (iq + j < n && by[4 * q + j]) lastnz = iq + j;
        }
    }
    const int incl = wave_incl_scan_max(lastnz);
    int ex = __shfl_up(incl, 1);
    if (ln == 0) ex = -1;
    if (ln == 63) scan_lds[wv] = incl;
    __syncthreads();
    int prev = carry;
    for (int k = 0; k < wv; k++) prev = max(prev, scan_lds[k]);
    prev = max(prev, ex);
    int ins = 0;
    uint32_t mask = 0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        const int i = i0 + q;
        if (i < n) {
            const int z = i - 1 - prev;
            if (by[q] <= 3 && z >= 2 && !(z & 1)) {
                ins++;
                mask |= 1u << q;
            }
            if (by[q]) prev = i;
        }
    }
    *insmask = mask;
    return ins;
}

__device__ __forceinline__ int tile_carry(const FrameArgs& a, int nal, int t) {
    int c = -1;  // the NAL header byte before the RBSP is non-zero
    for (int k = 0; k < t; k++) c = max(c, a.tile_nz[nal * a.max_tiles + k]);
    return c;
}

__global__ __launch_bounds__(256) void k_ep_count(FrameArgs a) {
    __shared__ int scan_lds[4];
    __shared__ int red[4];
    const int s = blockIdx.y, t = blockIdx.x;
    const int nn = slice_nals(a, a.tasks[s]);
    for (int j = 0; j < nn; j++) {
        const int nal = s * a.nal_per_slice + j;
        const int n = a.slice_info[4 * nal];
        const int t0 = t * kTile;
        if (t0 >= n) continue;
        const uint32_t* rbsp = nal_rbsp(a, s, j);
        uint8_t by[16];
        uint32_t mask;
        int ins = ep_thread(rbsp, n, t0, tile_carry(a, nal, t), scan_lds, by, &mask);
        for (int o = 32; o > 0; o >>= 1) ins += __shfl_down(ins, o);
        if (lane_id() == 0) red[threadIdx.x >> 6] = ins;
        __syncthreads();
        if (threadIdx.x == 0) a.tile_ins[nal * a.max_tiles + t] = red[0] + red[1] + red[2] + red[3];
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_ep_write(FrameArgs a) {
    __shared__ int scan_lds[4];
    __shared__ int wave_tot[5];
    __shared__ int sh_before, sh_base;
    __shared__ uint8_t sOut[kTile + kTile / 2 + 16];
    const int s = blockIdx.y, t = blockIdx.x, tid = threadIdx.x;
    const SliceTask& task = a.tasks[s];
    const int nn = slice_nals(a, task);
    for (int j = 0; j < nn; j++) {
    const int nal = s * a.nal_per_slice + j;
    const int n = a.slice_info[4 * nal];
    const int t0 = t * kTile;
    if (t0 >= n) continue;
    if (tid < 64) {
        int b = 0;
        for (int k = tid; k < t; k += 64) b += a.tile_ins[nal * a.max_tiles + k];
        b = wave_sum(b);
        // K5: the slot bytes of the NALs before this one (prefix + RBSP + insertions)
        int base = 0;
        for (int jj = 0; jj < j; jj++) {
            const int q = s * a.nal_per_slice + jj, nq = a.slice_info[4 * q];
            int ins_q = 0;
            for (int k = tid; k * kTile < nq; k += 64) ins_q += a.tile_ins[q * a.max_tiles + k];
            base += a.slice_info[4 * q + 1] + nq + wave_sum(ins_q);
        }
        if (tid == 0) {
            sh_before = b;
            sh_base = base;
        }
    }
    uint32_t* rbsp = nal_rbsp(a, s, j);
    uint8_t by[16];
    uint32_t mask;
    const int ins = ep_thread(rbsp, n, t0, tile_carry(a, nal, t), scan_lds, by, &mask);
    int tile_ins;
    const int ex = block_excl_scan<4>(ins, wave_tot, &tile_ins);
    const int i0 = t0 + tid * 16;
    int o = tid * 16 + ex;
#pragma unroll
    for (int q = 0; q < 16; q++) {
        if (i0 + q < n) {
            if (mask & (1u << q)) sOut[o++] = 3;
            sOut[o++] = by[q];
        }
    }
    // self-clean the RBSP words of this tile for the next frame
#pragma unroll
    for (int q = 0; q < 4; q++)
        if (i0 + 4 * q < n) rbsp[(i0 >> 2) + q] = 0u;
    __syncthreads();
    const int len = sk_min(n - t0, kTile) + tile_ins;
    const int g0 = sh_base + a.slice_info[4 * nal + 1] + t0 + sh_before;
    uint8_t* dst = a.host_out + (size_t)s * a.out_slot_bytes;
    if (j > 0 && t == 0 && tid == 0) {   // this NAL's start code and header
        const bool idr = task.final_action == ACT_I && task.idr_on_intra;
        dst[sh_base] = 0; dst[sh_base + 1] = 0; dst[sh_base + 2] = 0; dst[sh_base + 3] = 1;
        dst[sh_base + 4] = idr ? 0x65 : 0x41;
    }
    const int head = sk_min(len, (16 - (g0 & 15)) & 15);
    if (tid < head) dst[g0 + tid] = sOut[tid];
    const int nvec = (len - head) >> 4;
    for (int v = tid; v < nvec; v += 256) {
        const uint8_t* q = sOut + head + 16 * v;
        uint4 x;
        x.x = q[0] | (q[1] << 8) | (q[2] << 16) | ((uint32_t)q[3] << 24);
        x.y = q[4] | (q[5] << 8) | (q[6] << 16) | ((uint32_t)q[7] << 24);
        x.z = q[8] | (q[9] << 8) | (q[10] << 16) | ((uint32_t)q[11] << 24);
        x.w = q[12] | (q[13] << 8) | (q[14] << 16) | ((uint32_t)q[15] << 24);
        *reinterpret_cast<uint4*>(dst + g0 + head + 16 * v) = x;
    }
    const int tail0 = head + 16 * nvec;
    if (tid < len - tail0) dst[g0 + tail0 + tid] = sOut[tail0 + tid];
    if (j == nn - 1 && t0 + kTile >= n && tid == 0) a.host_size[s] = g0 + len;
    __syncthreads();   // sOut / sh_* are rewritten by the next NAL
    }
}

// ---------------------------------------------------------------------------
// Reference update: rec -> ref for coded slices, MV field for the next frame's
// candidates. One workgroup per MB row segment of 16 MBs, 16-byte accesses.
__global__ __launch_bounds__(256) void k_commit(FrameArgs a) {
    const int mby = blockIdx.y, mbx0 = blockIdx.x * 16;
    const int s = mby / a.rows_per_slice;
    const int fin = a.tasks[s].final_action;
    if (fin == ACT_NONE) return;
    const int tid = threadIdx.x;
    const int nmbs = sk_min(16, a.mb_w - mbx0);
    if (tid < nmbs) {
        const int idx = mby * a.mb_w + mbx0 + tid;
        const bool zero = fin == ACT_SKIPALL;
        a.mvfield[2 * idx] = zero ? 0 : a.me[idx].mvx;
        a.mvfield[2 * idx + 1] = zero ? 0 : a.me[idx].mvy;
    }
    // This segment's samples, one uint4 (luma) / uint2..uint4 (chroma) per thread.
    auto copy = [&](const Planes& src, const Planes& dst) {
        {   // luma: 16 rows x (nmbs * 16) bytes
            const int row = tid >> 4, v = tid & 15;
            if (v < nmbs) {
                const size_t o = (size_t)(mby * 16 + row) * a.stride_y + (mbx0 + v) * 16;
                *reinterpret_cast<uint4*>(dst.y + o) = *reinterpret_cast<const uint4*>(src.y + o);
            }
        }
        if (tid < 128) {  // chroma: 2 planes x 8 rows x (nmbs * 8) bytes, uint4 = 2 MBs
            const int comp = tid >> 6, row = (tid >> 3) & 7, v = tid & 7;
            if (2 * v < nmbs) {
                const size_t o = (size_t)(mby * 8 + row) * a.stride_c + (mbx0 + 2 * v) * 8;
                uint8_t* d = comp ? dst.v : dst.u;
                const uint8_t* sp = comp ? src.v : src.u;
                if (2 * v + 1 < nmbs && (a.stride_c & 15) == 0) {
                    *reinterpret_cast<uint4*>(d + o) = *reinterpret_cast<const uint4*>(sp + o);
                } else {  // odd MB count per row: chroma rows are only 8-byte aligned
                    *reinterpret_cast<uint2*>(d + o) = *reinterpret_cast<const uint2*>(sp + o);
                    if (2 * v + 1 < nmbs)
                        *reinterpret_cast<uint2*>(d + o + 8) = *reinterpret_cast<const uint2*>(sp + o + 8);
                }
            }
        }
    };
    // sliding-window DPB: the current reference becomes reference 1 (a skip-all picture
    // is a reference too); the same thread then overwrites ref with rec below
    if (a.num_refs > 1) copy(a.ref, a.ref1);
    if (fin == ACT_SKIPALL || slice_deblock(a.deblock, a.tasks[s])) return;  // reference unchanged / written by k_deblock
    copy(a.rec, a.ref);
}

// ---------------------------------------------------------------------------
// K7: in-loop deblocking (8.7; shared filter code in codec/h264_deblock.h).
//   k_deblock_prep  one wave per MB: QP_Y chain (ballot scan back to the last MB
//                   of the slice that carried mb_qp_delta) -> DbInfo
//   k_deblock       one workgroup per coded slice, wave r filters MB row r, MB x at
//                   step x + 2r + 1. The 2-MB lag covers every raster-order
//                   dependency of 8.7 (left MB, top MB, and the top-right MB whose
//                   left edge rewrites the top MB's right columns). Each band keeps
//                   a 4-slot ring of its MBs in LDS: the next MB is prefetched from
//                   rec while the current one is filtered, and an MB is written to
//                   ref three steps after its own step, once the band below has
//                   filtered its top edge. Lanes 0-15 own a luma row (vertical
//                   edges) then a luma column (horizontal edges), lanes 16-31 the
//                   same for Cb/Cr; the 4 (2) edges of a line run in registers.
__global__ __launch_bounds__(256) void k_deblock_prep(FrameArgs a) {
    const int nmb = a.mb_w * a.mb_h;
    const int idx = xcd_remap(blockIdx.x, gridDim.x) * 4 + (threadIdx.x >> 6);
    if (idx >= nmb) return;
    const SliceTask t = a.tasks[(idx / a.mb_w) / a.rows_per_slice];
    if (t.final_action != ACT_P && t.final_action != ACT_I) return;
    if (!slice_deblock(a.deblock, t)) return;   // automatic deblocking: an unfiltered slice
    const int l = lane_id();
    int first = t.first_row * a.mb_w;
    if (split_i(a, t)) first += ((idx - first) / kIntraSubMbs) * kIntraSubMbs;   // K5: the chain restarts per sub-slice
    const MbInfo mb = a.mbs[idx];
    int qpy = mb.qp;
    if (!mb_has_qp_delta(mb)) {
        qpy = t.qp;
        int j = idx - 1;
        while (j >= first) {
            const int base = j - 63, m = base + l;
            const unsigned long long msk = __ballot(m >= first && mb_has_qp_delta(a.mbs[m]));
            if (msk) {
                qpy = a.mbs[base + 63 - __clzll(msk)].qp;
                break;
            }
            j = base - 1;
        }
    }
    if (l == 0) a.db[idx] = db_info(mb, qpy);
}

__device__ __forceinline__ void unpack4(uint32_t w, int* d) {
    d[0] = w & 255;
    d[1] = (w >> 8) & 255;
    d[2] = (w >> 16) & 255;
    d[3] = w >> 24;
}
__device__ __forceinline__ uint32_t pack4(const int* d) {
    return (uint32_t)d[0] | ((uint32_t)d[1] << 8) | ((uint32_t)d[2] << 16) | ((uint32_t)d[3] << 24);
}

__device__ __forceinline__ DbInfo as_db(uint2 v) {
    DbInfo d;
    __builtin_memcpy(&d, &v, sizeof(d));
    return d;
}

// Workgroup barrier ordering LDS only: __syncthreads() would also drain vmcnt and
// stall on the prefetch loads issued this step.
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Per-QP filter parameters packed in one dword: alpha | beta << 8 | tC0(bS 1, 2, 3) << 16/21/26.
__device__ __forceinline__ uint32_t db_pack_par(int i) {
    return (uint32_t)H264_DB_ALPHA[i] | ((uint32_t)H264_DB_BETA[i] << 8) | ((uint32_t)H264_DB_TC0[i][0] << 16) |
           ((uint32_t)H264_DB_TC0[i][1] << 21) | ((uint32_t)H264_DB_TC0[i][2] << 26);
}

// One edge of one line in the unified luma/chroma form: v = {p3 p2 p1 p0 q0 q1 q2 q3}.
// A chroma line is a luma line whose ap/aq are forced false and whose tC is tC0 + 1
// (8.7.2.3): then p1/q1/p2/q2 stay, bS < 4 moves p0/q0 by the clipped delta and
// bS = 4 gives (2p1 + p0 + q1 + 2) >> 2 — exactly db_filter_chroma. One straight-line
// sequence for all 32 active lanes (no luma/chroma divergence).
// |a - b| of two samples (0..255) in one v_sad_u16; clip3 as v_max + v_min.
__device__ __forceinline__ int adiff(int a, int b) { return (int)__builtin_amdgcn_sad_u16((uint32_t)a, (uint32_t)b, 0u); }
__device__ __forceinline__ int clip3(int x, int lo, int hi) { return min(max(x, lo), hi); }

template <bool kMbEdge>   // bS = 4 only occurs on MB edges: internal edges skip the strong filter
__device__ __forceinline__ void db_filter_line(int* v, int bs, uint32_t par, bool chroma) {
    const int alpha = par & 255, beta = (par >> 8) & 31;
    const int tc0 = __builtin_amdgcn_ubfe(par, 16 + 5 * sk_clip(bs - 1, 0, 2), 5);
    const int p3 = v[0], p2 = v[1], p1 = v[2], p0 = v[3], q0 = v[4], q1 = v[5], q2 = v[6], q3 = v[7];
    const bool on = (bs != 0) & (adiff(p0, q0) < alpha) & (adiff(p1, p0) < beta) & (adiff(q1, q0) < beta);
    const bool ap = !chroma & (adiff(p2, p0) < beta), aq = !chroma & (adiff(q2, q0) < beta);
    const int tc = tc0 + (chroma ? 1 : (int)ap + (int)aq);
    const int d = clip3((((q0 - p0) * 4) + (p1 - q1) + 4) >> 3, -tc, tc);
    const int avg = (p0 + q0 + 1) >> 1;
    int np0 = sk_clip255(p0 + d), nq0 = sk_clip255(q0 - d);
    int np1 = ap ? p1 + clip3((p2 + avg - (p1 * 2)) >> 1, -tc0, tc0) : p1;
    int nq1 = aq ? q1 + clip3((q2 + avg - (q1 * 2)) >> 1, -tc0, tc0) : q1;
    int np2 = p2, nq2 = q2;
    if (kMbEdge) {
        const bool strong = bs == 4;
        const bool sm = adiff(p0, q0) < ((alpha >> 2) + 2);
        const bool ps = ap & sm, qs = aq & sm;
        const int sp0 = ps ? (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3 : (2 * p1 + p0 + q1 + 2) >> 2;
        const int sq0 = qs ? (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3 : (2 * q1 + q0 + p1 + 2) >> 2;
        np0 = strong ? sp0 : np0;
        nq0 = strong ? sq0 : nq0;
        np1 = strong ? (ps ? (p2 + p1 + p0 + q0 + 2) >> 2 : p1) : np1;
        nq1 = strong ? (qs ? (p0 + q0 + q1 + q2 + 2) >> 2 : q1) : nq1;
        np2 = (strong & ps) ? (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3 : p2;
        nq2 = (strong & qs) ? (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3 : q2;
    }
    v[1] = on ? np2 : p2;
    v[2] = on ? np1 : p1;
    v[3] = on ? np0 : p0;
    v[4] = on ? nq0 : q0;
    v[5] = on ? nq1 : q1;
    v[6] = on ? nq2 : q2;
}

// Per-MB edge record (3 x 16 bytes), built in parallel by k_deblock_edges so the
// sequential wavefront only extracts bits:
//   w[0..1]  bS of the vertical edges, 4 bits per (edge le, 4x4 row b) at bit 16*(le&1) + 4*b of w[le>>1]
//   w[2..3]  the same for the horizontal edges (b = 4x4 column)
//   w[4..6]  luma params (db_pack_par) of the left, top and internal edges
//   w[7..9]  chroma params of the left, top and internal edges
//   w[10]    edge mask: bit le (vertical) / 4 + le (horizontal) set if any bS of that edge is non-zero
// The left edge of MB column 0 and the top edge of a slice's first row are off (idc 2),
// as are the edges between the sub-slices of a split I slice.
__global__ __launch_bounds__(256) void k_deblock_edges(FrameArgs a) {
    const int nmb = a.mb_w * a.mb_h;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= nmb) return;
    const int mbx = idx % a.mb_w, mby = idx / a.mb_w;
    const SliceTask t = a.tasks[mby / a.rows_per_slice];
    if (t.final_action != ACT_P && t.final_action != ACT_I) return;
    if (!slice_deblock(a.deblock, t)) return;
    const DbInfo cur = a.db[idx];
    int sub0 = t.first_row * a.mb_w;   // K5 sub-slices: no edge leaves the MB's sub-slice (idc 2)
    if (split_i(a, t)) sub0 += ((idx - sub0) / kIntraSubMbs) * kIntraSubMbs;
    const bool hl = mbx > 0 && idx - 1 >= sub0, ht = mby > t.first_row && idx - a.mb_w >= sub0;
    const DbInfo left = hl ? a.db[idx - 1] : cur, top = ht ? a.db[idx - a.mb_w] : cur;
    uint32_t w[12] = {};
#pragma unroll
    for (int le = 0; le < 4; le++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int sh = 16 * (le & 1) + 4 * b;
            const int pe = le == 0 ? 3 : le - 1;
            const int bv = (le == 0 && !hl) ? 0 : db_bs(le == 0 ? left : cur, cur, le == 0, b * 4 + pe, b * 4 + le);
            const int bh = (le == 0 && !ht) ? 0 : db_bs(le == 0 ? top : cur, cur, le == 0, pe * 4 + b, le * 4 + b);
            w[le >> 1] |= (uint32_t)bv << sh;
            w[2 + (le >> 1)] |= (uint32_t)bh << sh;
            w[10] |= (bv ? 1u << le : 0u) | (bh ? 16u << le : 0u);
        }
    const int qc = cur.qpy, cc = H264_CHROMA_QP[qc];
    w[4] = db_pack_par((left.qpy + qc + 1) >> 1);
    w[5] = db_pack_par((top.qpy + qc + 1) >> 1);
    w[6] = db_pack_par(qc);
    w[7] = db_pack_par((H264_CHROMA_QP[left.qpy] + cc + 1) >> 1);
    w[8] = db_pack_par((H264_CHROMA_QP[top.qpy] + cc + 1) >> 1);
    w[9] = db_pack_par(cc);
    uint4* o = a.dbe + 3 * (size_t)idx;
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
    o[2] = make_uint4(w[8], w[9], w[10], 0);
}

// K7 deblocking of one slice. Wave r owns MB row r ("band") and filters MB x at step
// k = x + 2r + 1; the 2-MB lag covers every raster-order dependency of 8.7 (left MB,
// top MB, and the top-right MB whose left edge rewrites the top MB's right columns).
// Per band an 8-slot LDS ring holds MBs as 32 lines x 16 bytes (luma rows 0-15, Cb
// rows 16-23, Cr rows 24-31; chroma lines use 8 of the 16 bytes). Lanes 0-31 own one
// line each: its row for the vertical edges, its column for the horizontal ones,
// through the unified filter (db_filter_line). Pixels and side info of MB x + 2 are
// loaded into registers at step k and land in LDS at step k + 1, so a whole step
// hides the global latency; MB x - 3 (final once the band below filtered its top
// edge) is stored to ref. Edges whose bS is 0 on every line are skipped wave-uniformly
// (static desktop regions: P_Skip runs filter nothing).
template <int MAXR>
__global__ __launch_bounds__(64 * MAXR) void k_deblock(FrameArgs a) {
    constexpr int kSlots = 8;
    __shared__ uint32_t ring[MAXR][kSlots][32][4];
    __shared__ uint4 erec[MAXR][kSlots][3];   // edge record (k_deblock_edges) of the slot's MB
    const SliceTask t = a.tasks[blockIdx.x];
    if (t.final_action != ACT_P && t.final_action != ACT_I) return;
    if (!slice_deblock(a.deblock, t)) return;   // k_commit copied rec -> ref
    const int r = threadIdx.x >> 6, l = lane_id();
    const int R = t.num_rows, W = a.mb_w;
    const int mby = t.first_row + r;
    const bool band = r < R;
    const bool act = l < 32, chroma = l >= 16;
    const int li = chroma ? (l & 7) : (l & 15);      // row / column inside the component
    const int nrows = chroma ? 8 : 16;
    const int lbase = chroma ? 16 + (l & 8) : 0;     // first line of the component
    const int ldw = chroma ? 1 : 3;                  // dword holding a line's last 4 samples
    const int bsh = 4 * (chroma ? li >> 1 : li >> 2);   // nibble of this line's 4x4 row / column
    const uint8_t* src = chroma ? ((l & 8) ? a.rec.v : a.rec.u) : a.rec.y;
    uint8_t* dst = chroma ? ((l & 8) ? a.ref.v : a.ref.u) : a.ref.y;
    const int mbyc = sk_min(mby, t.first_row + R - 1);   // idle waves of a short slice load valid rows
    const size_t rowoff = chroma ? (size_t)(mbyc * 8 + li) * a.stride_c : (size_t)(mbyc * 16 + li) * a.stride_y;
    const int mbbytes = chroma ? 8 : 16;

    // Loads run unconditionally on clamped addresses (results for MBs outside the
    // slice are never stored): no zero-fill of in-flight registers, no extra waits.
    // A line is two 8-byte halves; chroma lines (8 bytes) load/store their half twice.
    const int half2 = chroma ? 0 : 8;
    auto load_px = [&](int x) {
        const uint8_t* p0 = src + rowoff + sk_clip(x, 0, W - 1) * mbbytes;
        const uint2 lo = *reinterpret_cast<const uint2*>(p0), hi = *reinterpret_cast<const uint2*>(p0 + half2);
        return make_uint4(lo.x, lo.y, hi.x, hi.y);
    };
    auto load_rec = [&](int x) {   // lanes 32..34 fetch the 3 x 16-byte edge record
        return a.dbe[3 * ((size_t)mbyc * W + sk_clip(x, 0, W - 1)) + sk_min(sk_max(l - 32, 0), 2)];
    };

    int x = -1 - 2 * r;   // MB of step 0
    // In flight across one step, stored to LDS at the top of the next: no register
    // rotation of loaded values, so the only wait is for last step's loads.
    uint4 pre = make_uint4(0, 0, 0, 0);
    if (band) pre = act ? load_px(x + 1) : load_rec(x + 1);
    const int steps = W + 2 * R + 2;
    for (int k = 0; k < steps; k++, x++) {
        if (band) {
            if (x + 1 >= 0 && x + 1 < W) {
                const int sn = (x + 1) & (kSlots - 1);
                if (act) *reinterpret_cast<uint4*>(ring[r][sn][l]) = pre;
                else if (l < 35) erec[r][sn][l - 32] = pre;
            }
            pre = act ? load_px(x + 2) : load_rec(x + 2);
            wave_sync();

            if (x >= 0 && x < W) {
                const int sl = x & (kSlots - 1);
                const uint4 e0 = erec[r][sl][0], e1 = erec[r][sl][1], e2 = erec[r][sl][2];
                // slot e runs if luma edge e or, for chroma slot 1, luma edge 2 has a non-zero bS
                const uint32_t emask = e2.z | ((e2.z & 0x44u) >> 1);
                // per line: bS of edge slot e (chroma slots 0/1 = luma edges 0/2, slots 2/3 off)
                auto bs_of = [&](uint32_t w01, uint32_t w23, int e) -> int {
                    if (chroma) {
                        if (e >= 2) return 0;
                        return __builtin_amdgcn_ubfe(e == 0 ? w01 : w23, bsh, 4);
                    }
                    return __builtin_amdgcn_ubfe(e < 2 ? w01 : w23, 16 * (e & 1) + bsh, 4);
                };
                const uint32_t p_left = chroma ? e1.w : e1.x, p_top = chroma ? e2.x : e1.y;
                const uint32_t p_in = chroma ? e2.y : e1.z;
                uint32_t* own = ring[r][sl][0];
                if (emask & 15u) {   // vertical edges: lane = line (row)
                    uint32_t* lp = ring[r][(x - 1) & (kSlots - 1)][act ? l : 0];
                    uint32_t* op = own + 4 * (act ? l : 0);
                    int v[20];
                    unpack4((emask & 1u) ? lp[ldw] : 0u, v);
#pragma unroll
                    for (int q = 0; q < 4; q++) unpack4(op[q], v + 4 + 4 * q);
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if (emask & (1u << e)) {
                            const int bs = act ? bs_of(e0.x, e0.y, e) : 0;
                            if (e == 0) db_filter_line<true>(v, bs, p_left, chroma);
                            else db_filter_line<false>(v + 4 * e, bs, p_in, chroma);
                        }
                    if (act) {
                        if (emask & 1u) lp[ldw] = pack4(v);
#pragma unroll
                        for (int q = 0; q < 4; q++) op[q] = pack4(v + 4 + 4 * q);
                    }
                    wave_sync();
                }
                if (emask & 0xF0u) {   // horizontal edges: lane = line (column)
                    uint8_t* ob = reinterpret_cast<uint8_t*>(own) + lbase * 16 + li;
                    uint8_t* tb = reinterpret_cast<uint8_t*>(ring[sk_max(r - 1, 0)][sl][0]) +
                                  (lbase + nrows - 4) * 16 + li;
                    const bool top_on = (emask & 16u) && act;
                    int v[20];
#pragma unroll
                    for (int q = 0; q < 4; q++) v[q] = top_on ? tb[q * 16] : 0;
#pragma unroll
                    for (int q = 0; q < 16; q++) v[4 + q] = act ? ob[sk_min(q, nrows - 1) * 16] : 0;
#pragma unroll
                    for (int e = 0; e < 4; e++)
                        if (emask & (16u << e)) {
                            const int bs = act ? bs_of(e0.z, e0.w, e) : 0;
                            if (e == 0) db_filter_line<true>(v, bs, p_top, chroma);
                            else db_filter_line<false>(v + 4 * e, bs, p_in, chroma);
                        }
                    if (act) {
                        if (top_on) {
#pragma unroll
                            for (int q = 1; q < 4; q++) tb[q * 16] = (uint8_t)v[q];
                        }
#pragma unroll
                        for (int q = 0; q < 16; q++)
                            if (q < nrows) ob[q * 16] = (uint8_t)v[4 + q];
                    }
                    wave_sync();
                }
            }
            // MB x - 3 is final (the band below filtered its top edge last step)
            const int xb = x - 3;
            if (act && xb >= 0 && xb < W) {
                const uint4 q = *reinterpret_cast<const uint4*>(ring[r][xb & (kSlots - 1)][l]);
                uint8_t* p0 = dst + rowoff + xb * mbbytes;
                *reinterpret_cast<uint2*>(p0) = make_uint2(q.x, q.y);
                *reinterpret_cast<uint2*>(p0 + half2) = chroma ? make_uint2(q.x, q.y) : make_uint2(q.z, q.w);
            }
        }
        lds_barrier();
    }
}

// ---------------------------------------------------------------------------
void launch_convert_damage(const FrameArgs& a, hipStream_t s) {
    dim3 grid((a.mb_w + 15) / 16, a.mb_h);
    if (a.yuv_fmt) hipLaunchKernelGGL(k_yuv_damage, grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_convert_damage, grid, dim3(256), 0, s, a);
}

void launch_frontend(const FrameArgs& a, hipStream_t s) {
    int nmb = a.mb_w * a.mb_h;
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(256), 0, s, a);
    if (a.me_full) hipLaunchKernelGGL(k_me_mfma, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_motion_search, dim3(nmb), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_decide, dim3(a.num_slices), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_rc_qp, dim3(1), dim3(64), 0, s, a);
    // K4c quarter-pel refinement (H.264 and HEVC; the HEVC back end codes the vectors
    // with its own 8-tap filters)
    if (a.subpel) hipLaunchKernelGGL(k_subpel, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
}

void launch_rc_guard_sizes(const FrameArgs& a, const int* sizes, int n, int* redo, bool chained, hipStream_t s) {
    hipLaunchKernelGGL(k_rc_guard_sizes, dim3(1), dim3(256), 0, s, a, sizes, n, redo, chained ? 1 : 0);
}

void launch_rc_account(const FrameArgs& a, const int* sizes, int n, int stride, int per_slice, hipStream_t s) {
    hipLaunchKernelGGL(k_rc_account, dim3(1), dim3(64), 0, s, a, sizes, n, stride, per_slice);
}

// Transform / quantisation / reconstruction / CAVLC / slice scan of every coded slice.
static void launch_code(const FrameArgs& a, hipStream_t s) {
    int nmb = a.mb_w * a.mb_h;
    hipLaunchKernelGGL(k_code_inter, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_intra_prep, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
    if (a.rows_per_slice <= 4)
        hipLaunchKernelGGL(k_code_intra<4>, dim3(a.num_slices), dim3(64 * 5), 0, s, a);
    else
        hipLaunchKernelGGL(k_code_intra<kMaxRows - 1>, dim3(a.num_slices), dim3(64 * kMaxRows), 0, s, a);
    if (a.nal_per_slice > 1)   // K5 sub-sliced I slices: one wave per sub-slice
        hipLaunchKernelGGL(k_code_intra_sub, dim3((a.num_slices * a.nal_per_slice + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_cavlc, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_slice_scan, dim3(a.num_slices * a.nal_per_slice), dim3(256), 0, s, a);
}

void launch_encode(const FrameArgs& a, hipStream_t s, bool guard) {
    int nmb = a.mb_w * a.mb_h;
    launch_frontend(a, s);
    if (a.aq_strength > 0) hipLaunchKernelGGL(k_aq, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
    launch_code(a, s);
    if (guard && a.rc_redo) {   // K10 CBR: VBV overflow -> one coarser pass (kernels exit early otherwise)
        hipLaunchKernelGGL(k_rc_guard, dim3(a.num_slices), dim3(256), 0, s, a);
        FrameArgs b = a;
        b.gate = a.rc_redo;
        launch_code(b, s);
    }
    hipLaunchKernelGGL(k_mb_concat, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
    const dim3 tiles(a.max_tiles, a.num_slices);
    hipLaunchKernelGGL(k_ep_nz, tiles, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_ep_count, tiles, dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_ep_write, tiles, dim3(256), 0, s, a);
    launch_rc_account(a, a.slice_info, a.num_slices * a.nal_per_slice, 4, a.nal_per_slice, s);
}

void launch_commit(const FrameArgs& a, hipStream_t s) {
    hipLaunchKernelGGL(k_commit, dim3((a.mb_w + 15) / 16, a.mb_h), dim3(256), 0, s, a);
    if (a.deblock) {
        const int nmb = a.mb_w * a.mb_h;
        hipLaunchKernelGGL(k_deblock_prep, dim3((nmb + 3) / 4), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_deblock_edges, dim3((nmb + 255) / 256), dim3(256), 0, s, a);
        if (a.rows_per_slice <= 4)
            hipLaunchKernelGGL(k_deblock<4>, dim3(a.num_slices), dim3(64 * a.rows_per_slice), 0, s, a);
        else
            hipLaunchKernelGGL(k_deblock<kMaxRows>, dim3(a.num_slices), dim3(64 * a.rows_per_slice), 0, s, a);
    }
}

}  // namespace gpu
}  // namespace h264
}  // namespace sk
