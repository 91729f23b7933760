// gfx950 (CDNA4) kernels of the HEVC back end. One 64-lane wavefront per 16x16 CU:
//   k_hevc_inter       P slices: merge/AMVP decision on the front end's motion field,
//                      quarter-pel 8-tap luma MC + 4-tap chroma MC, 16x16 / 8x8 DCT (LDS, lane =
//                      row x 4 columns), quantisation, reconstruction (SKIPALL: all skip)
//   k_hevc_intra_prep  I slices, every CU in parallel: intra mode (all 35) against the source
//   k_hevc_intra       I slices: CTB wavefront (wave = CTB row, lag 2 = WPP order)
//   k_hevc_bins        CU syntax -> CABAC bin entries (hevc_core.h code_cu)
//   k_hevc_sync        WPP: context states at every CTB row start (state-only replay of
//                      the first two CTBs of the row above, lane = context)
//   k_pc_*             chunk-parallel CABAC of the row substreams (codec/hevc_pcabac.h):
//                      context chains, range maps, composition, per-CTB coding, merge
//   k_hevc_hdr         slice header with entry points, NAL prefix, substream offsets
//   k_hevc_ep_copy     wave-parallel emulation prevention + copy into host-mapped slots
//   k_hevc_dbk_v/h     in-loop deblocking (before the syntax: SAO decides on its output)
//   k_hevc_sao_*       SAO: stats + own decision per CTB (lane-parallel tables), merge
//                      candidate distortions, row merge pass (LDS), filter + copy back
// Bit-exact with the CPU reference (codec/hevc_cpu.cpp): integer math only.
#include "hevc_gpu.h"

namespace sk {
namespace hevc {
namespace gpu {

using h264::ACT_I;
using h264::ACT_P;
using h264::ACT_SKIPALL;
using h264::SliceTask;
using h264::gpu::FrameArgs;
using h264::gpu::Planes;

__device__ __forceinline__ int lane() { return threadIdx.x & 63; }
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int wsum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// Per-wave LDS working set of one CU.
struct CuLds {
    uint8_t src[kCoefPerCu];     // Y 16x16 | Cb 8x8 | Cr 8x8 (raster)
    uint8_t pred[kCoefPerCu];
    int32_t a[kCoefPerCu];       // residual / dequantised coefficients
    int32_t b[kCoefPerCu];       // transform intermediate
    uint8_t ref[65 + 65 + 33 + 33];   // intra: luma raw | luma filtered | Cb | Cr
    uint8_t refm[3][64];              // intra, directional modes: main reference arrays (Y, Cb, Cr)
    int misc[4];
    int mlx[kMaxMergeCand], mly[kMaxMergeCand], px[2], py[2];   // inter: merge / AMVP candidates
};

// LDS copy of the 16-point DCT matrix (the 8-point one is its even rows).
__device__ __forceinline__ void load_t16(int8_t* t) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) t[i] = HEVC_T16[i >> 4][i & 15];
}

// Transform, quantisation and reconstruction of the CU in L (src, pred filled).
// Lane mapping: luma outputs (row l >> 2, columns 4*(l & 3) .. +3), chroma outputs
// (component l >> 5, row (l >> 2) & 7, columns 2*(l & 3) .. +1). Writes the levels to
// `gcoef` (global) and the reconstruction into L.pred; returns the cbf bits.
__device__ __forceinline__ int code_cu_wave(CuLds& L, const int8_t* T, int qp, bool intra, int16_t* gcoef) {
    const int l = lane();
    const int qpc = chroma_qp(qp);
    const int ly = l >> 2, lx0 = 4 * (l & 3);
    const int cc = l >> 5, cy = (l >> 2) & 7, cx0 = 2 * (l & 3);
    const int cbase = kCoefCb + cc * 64;
    for (int i = l; i < kCoefPerCu; i += 64) L.a[i] = (int)L.src[i] - (int)L.pred[i];
    wsync();
    // forward stage 1 (rows): b[y][u] = (sum_x T[u][x] a[y][x] + rnd) >> sh1
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int u = lx0 + k;
        int s = 0;
#pragma unroll
        for (int x = 0; x < 16; x++) s += (int)T[u * 16 + x] * L.a[ly * 16 + x];
        L.b[ly * 16 + u] = (s + 4) >> 3;
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int u = cx0 + k;
        int s = 0;
#pragma unroll
        for (int x = 0; x < 8; x++) s += (int)T[(2 * u) * 16 + x] * L.a[cbase + cy * 8 + x];
        L.b[cbase + cy * 8 + u] = (s + 2) >> 2;
    }
    wsync();
    // forward stage 2 (columns) + quantisation + dequantisation; levels to global
    int nzl = 0, nzc = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int u = lx0 + k, v = ly;
        int s = 0;
#pragma unroll
        for (int y = 0; y < 16; y++) s += (int)T[v * 16 + y] * L.b[y * 16 + u];
        const int c = (s + 512) >> 10;
        const int lv = quant_level(c, qp, 4, intra);
        nzl |= lv;
        gcoef[v * 16 + u] = (int16_t)lv;
        L.a[v * 16 + u] = dequant_level(lv, qp, 4);
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int u = cx0 + k, v = cy;
        int s = 0;
#pragma unroll
        for (int y = 0; y < 8; y++) s += (int)T[(2 * v) * 16 + y] * L.b[cbase + y * 8 + u];
        const int c = (s + 256) >> 9;
        const int lv = quant_level(c, qpc, 3, intra);
        nzc |= lv;
        gcoef[cbase + v * 8 + u] = (int16_t)lv;
        L.a[cbase + v * 8 + u] = dequant_level(lv, qpc, 3);
    }
    const int cbf = (__ballot(nzl != 0) ? 1 : 0) | ((__ballot(nzc != 0 && cc == 0) ? 1 : 0) << 1) |
                    ((__ballot(nzc != 0 && cc == 1) ? 1 : 0) << 2);
    wsync();
    // inverse stage 1 (columns): b[y][x] = clip16((sum_j T[j][y] a[j][x] + 64) >> 7)
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = lx0 + k, y = ly;
        int s = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) s += (int)T[j * 16 + y] * L.a[j * 16 + x];
        L.b[y * 16 + x] = sk_clip((s + 64) >> 7, -32768, 32767);
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int x = cx0 + k, y = cy;
        int s = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) s += (int)T[(2 * j) * 16 + y] * L.a[cbase + j * 8 + x];
        L.b[cbase + y * 8 + x] = sk_clip((s + 64) >> 7, -32768, 32767);
    }
    wsync();
    // inverse stage 2 (rows) + reconstruction into pred
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = lx0 + k, y = ly;
        int s = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) s += (int)T[j * 16 + x] * L.b[y * 16 + j];
        const int i = y * 16 + x;
        L.pred[i] = (uint8_t)sk_clip255((int)L.pred[i] + ((s + 2048) >> 12));
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
        const int x = cx0 + k, y = cy;
        int s = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) s += (int)T[(2 * j) * 16 + x] * L.b[cbase + y * 8 + j];
        const int i = cbase + y * 8 + x;
        L.pred[i] = (uint8_t)sk_clip255((int)L.pred[i] + ((s + 2048) >> 12));
    }
    wsync();
    return cbf;
}

// Source samples of CU (cx, cy) into L.src; reconstruction L.pred to the rec planes.
__device__ __forceinline__ void load_src(CuLds& L, const FrameArgs& f, int cx, int cy) {
    const int l = lane();
    for (int i = l; i < kCoefPerCu; i += 64) {
        uint8_t v;
        if (i < 256) v = f.src.y[(size_t)(cy * 16 + (i >> 4)) * f.stride_y + cx * 16 + (i & 15)];
        else {
            const int j = i - 256, c = j >> 6, r = (j >> 3) & 7, x = j & 7;
            v = (c ? f.src.v : f.src.u)[(size_t)(cy * 8 + r) * f.stride_c + cx * 8 + x];
        }
        L.src[i] = v;
    }
}
__device__ __forceinline__ void store_rec(const CuLds& L, const FrameArgs& f, int cx, int cy) {
    const int l = lane();
    for (int i = l; i < kCoefPerCu; i += 64) {
        if (i < 256) f.rec.y[(size_t)(cy * 16 + (i >> 4)) * f.stride_y + cx * 16 + (i & 15)] = L.pred[i];
        else {
            const int j = i - 256, c = j >> 6, r = (j >> 3) & 7, x = j & 7;
            (c ? f.rec.v : f.rec.u)[(size_t)(cy * 8 + r) * f.stride_c + cx * 8 + x] = L.pred[i];
        }
    }
}

// ---------------------------------------------------------------------------
// K6 inter (P slices) and skip-all slices: one wave per CU, 4 CUs per workgroup.
__global__ __launch_bounds__(256) void k_hevc_inter(HevcArgs A) {
    __shared__ CuLds Lw[4];
    __shared__ int8_t T[256];
    const FrameArgs& f = A.f;
    CuLds& L = Lw[threadIdx.x >> 6];
    const int n = f.mb_w * f.mb_h;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    const bool valid = idx < n;
    const int cx = valid ? idx % f.mb_w : 0, cy = valid ? idx / f.mb_w : 0;
    const SliceTask t = f.tasks[cy / f.rows_per_slice];
    const int l = lane();
    if (valid && t.final_action == ACT_SKIPALL && l == 0) {
        CuInfo z;
        memset(&z, 0, sizeof(z));
        z.mode = CU_SKIP;
        z.qp = (uint8_t)t.qp;
        A.cus[idx] = z;
    }
    const bool coded = valid && t.final_action == ACT_P;
    if (!__syncthreads_or(coded)) return;
    load_t16(T);
    __syncthreads();
    if (!coded) return;
    const int W = f.mb_w;
    auto nb = [&](int ox, int oy, bool ok) {
        NbMv m;
        m.av = ok;
        m.mvx = ok ? h264::me_qx(f.me[oy * W + ox]) : 0;
        m.mvy = ok ? h264::me_qy(f.me[oy * W + ox]) : 0;
        return m;
    };
    const bool top = cy > t.first_row;
    const NbMv A1 = nb(cx - 1, cy, cx > 0), B1 = nb(cx, cy - 1, top);
    const NbMv B0 = nb(cx + 1, cy - 1, top && cx + 1 < W), B2 = nb(cx - 1, cy - 1, top && cx > 0);
    // candidate lists in LDS (dynamically indexed: private arrays would live in scratch);
    // every lane writes the same values
    int *mlx = L.mlx, *mly = L.mly, *px = L.px, *py = L.py;
    merge_list(A1, B1, B0, B2, mlx, mly);
    amvp_list(A1, B1, B0, B2, px, py);
    wsync();
    const int mvx = h264::me_qx(f.me[idx]), mvy = h264::me_qy(f.me[idx]);   // quarter-pel (k_subpel)
    const int pic_w = f.stride_y, pic_h = f.mb_h * 16;
    load_src(L, f, cx, cy);
    {   // luma MC (hevc_core.h luma_mc_sample, separable form): the 23x23 integer window
        // into LDS (L.a as bytes, row pitch 24), horizontal 8-tap pass into L.b (23 rows x
        // 16), vertical pass into pred (lane = row l >> 2, 4 columns). L.a / L.b are free
        // until code_cu_wave.
        const int fx = mvx & 3, fy = mvy & 3;
        const int x0 = cx * 16 + (mvx >> 2) - 3, y0 = cy * 16 + (mvy >> 2) - 3;
        uint8_t* win = reinterpret_cast<uint8_t*>(L.a);
        for (int i = l; i < 23 * 23; i += 64) {
            const int r = i / 23, c = i - r * 23;
            win[r * 24 + c] = f.ref.y[(size_t)sk_clip(y0 + r, 0, pic_h - 1) * f.stride_y + sk_clip(x0 + c, 0, pic_w - 1)];
        }
        wsync();
        for (int i = l; i < 23 * 16; i += 64) {
            const uint8_t* w = win + (i >> 4) * 24 + (i & 15);
            int s = (int)w[3] << 6;
            if (fx) {
                s = 0;
#pragma unroll
                for (int k = 0; k < 8; k++) s += HEVC_LUMA_FILTER[fx][k] * (int)w[k];
            }
            L.b[i] = s;
        }
        wsync();
        const int y = l >> 2;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int x = 4 * (l & 3) + k;
            int v = L.b[(y + 3) * 16 + x];
            if (fy) {
                v = 0;
#pragma unroll
                for (int j = 0; j < 8; j++) v += HEVC_LUMA_FILTER[fy][j] * L.b[(y + j) * 16 + x];
                v >>= 6;
            }
            L.pred[y * 16 + x] = (uint8_t)sk_clip255((v + 32) >> 6);
        }
        // chroma: lane -> component l >> 5, row (l >> 2) & 7, 2 columns
        const int c = l >> 5, r = (l >> 2) & 7;
        const uint8_t* plane = c ? f.ref.v : f.ref.u;
#pragma unroll
        for (int k = 0; k < 2; k++) {
            const int x = 2 * (l & 3) + k;
            L.pred[kCoefCb + c * 64 + r * 8 + x] = (uint8_t)chroma_mc_sample(
                plane, f.stride_c, f.stride_c, f.mb_h * 8, cx * 8 + x, cy * 8 + r, mvx, mvy);
        }
    }
    wsync();
    const int cbf = code_cu_wave(L, T, t.qp, false, A.coefs + (size_t)idx * kCoefPerCu);
    store_rec(L, f, cx, cy);
    if (l == 0) {
        CuInfo cu;
        memset(&cu, 0, sizeof(cu));
        int midx = -1;
        for (int i = 0; i < kMaxMergeCand && midx < 0; i++)
            if (mlx[i] == mvx && mly[i] == mvy) midx = i;
        cu.cbf = (uint8_t)cbf;
        cu.qp = (uint8_t)t.qp;
        cu.mvx = (int16_t)mvx;
        cu.mvy = (int16_t)mvy;
        if (midx >= 0) {
            cu.mode = cbf ? CU_MERGE : CU_SKIP;
            cu.merge_idx = (uint8_t)midx;
        } else {
            cu.mode = CU_AMVP;
            const int c0 = mvd_bits_est(mvx - px[0]) + mvd_bits_est(mvy - py[0]);
            const int c1 = mvd_bits_est(mvx - px[1]) + mvd_bits_est(mvy - py[1]);
            const int k = c1 < c0 ? 1 : 0;
            cu.mvp_idx = (uint8_t)k;
            cu.mvdx = (int16_t)(mvx - px[k]);
            cu.mvdy = (int16_t)(mvy - py[k]);
        }
        A.cus[idx] = cu;
    }
}

// ---------------------------------------------------------------------------
// Intra reference samples (8.4.4.2.2, substitution in closed form for CTB = CU: the
// bottom-left half is never available) of an n x n block at (x0, y0): linear layout
// of build_intra_ref. Every lane writes the entries i = lane, lane + 64.
__device__ __forceinline__ void fill_ref(const uint8_t* P, int stride, int x0, int y0, int n, bool left, bool top, bool tr,
                         uint8_t* ref) {
    const int len = 4 * n + 1;
    for (int i = lane(); i < len; i += 64) {
        int v;
        if (!left && !top) {
            v = 128;
        } else if (i < 2 * n) {
            const int y = 2 * n - 1 - i;
            v = left ? P[(size_t)(y0 + sk_min(y, n - 1)) * stride + x0 - 1] : P[(size_t)(y0 - 1) * stride + x0];
        } else if (i == 2 * n) {
            v = (left && top) ? P[(size_t)(y0 - 1) * stride + x0 - 1]
                              : (left ? P[(size_t)y0 * stride + x0 - 1] : P[(size_t)(y0 - 1) * stride + x0]);
        } else {
            const int x = i - 2 * n - 1;
            if (x < n) v = top ? P[(size_t)(y0 - 1) * stride + x0 + x] : P[(size_t)y0 * stride + x0 - 1];
            else v = tr ? P[(size_t)(y0 - 1) * stride + x0 + x]
                        : (top ? P[(size_t)(y0 - 1) * stride + x0 + n - 1] : P[(size_t)y0 * stride + x0 - 1]);
        }
        ref[i] = (uint8_t)v;
    }
}
__device__ __forceinline__ void filter_ref(const uint8_t* r, int n, uint8_t* out) {
    const int len = 4 * n + 1;
    for (int i = lane(); i < len; i += 64)
        out[i] = (i == 0 || i == len - 1) ? r[i] : (uint8_t)((r[i - 1] + 2 * r[i] + r[i + 1] + 2) >> 2);
}
// Prediction sample for the encoder's modes (planar 0, DC 1, horizontal 10, vertical 26),
// identical to intra_pred_sample for them. dc: the block's DC value.
__device__ __forceinline__ int pred_fast(const uint8_t* r, int n, int log2n, int mode, bool luma, int dc, int x,
                                         int y) {
    auto Lf = [&](int yy) { return (int)r[2 * n - 1 - yy]; };
    auto Tf = [&](int xx) { return (int)r[2 * n + 1 + xx]; };
    if (mode == 0)
        return ((n - 1 - x) * Lf(y) + (x + 1) * Tf(n) + (n - 1 - y) * Tf(x) + (y + 1) * Lf(n) + n) >> (log2n + 1);
    if (mode == 1) {
        if (luma) {
            if (x == 0 && y == 0) return (Lf(0) + 2 * dc + Tf(0) + 2) >> 2;
            if (y == 0) return (Tf(x) + 3 * dc + 2) >> 2;
            if (x == 0) return (Lf(y) + 3 * dc + 2) >> 2;
        }
        return dc;
    }
    if (mode == 26) return (luma && x == 0) ? sk_clip255(Tf(0) + ((Lf(y) - Lf(-1)) >> 1)) : Tf(x);
    return (luma && y == 0) ? sk_clip255(Lf(0) + ((Tf(x) - Tf(-1)) >> 1)) : Lf(y);
}
// DC value of an n x n block: (sum of n top + n left references + n) >> (log2n + 1).
__device__ __forceinline__ int dc_value(const uint8_t* r, int n, int log2n) {
    const int l = lane();
    int v = 0;
    if (l < n) v = r[2 * n + 1 + l];               // top
    else if (l < 2 * n) v = r[2 * n - 1 - (l - n)];   // left
    return (wsum(v) + n) >> (log2n + 1);
}
// Main reference array of a directional mode (8.4.4.2.6) for an n x n block from the
// linear reference r: out[k + n] = ref[k], k = -n .. 2n (lane = k + n), with the other side
// projected through invAngle for negative angles (entries no sample reads stay 0).
__device__ __forceinline__ void build_refm(const uint8_t* r, int n, int mode, uint8_t* out) {
    const int k = lane() - n;
    if (k > 2 * n) return;
    const int angle = HEVC_INTRA_ANGLE[mode];
    const bool vert = mode >= 18;
    int v = 0;
    if (k >= 0) {
        v = vert ? r[2 * n + k] : r[2 * n - k];   // p[k-1][-1] / p[-1][k-1]
    } else if (angle < 0) {
        const int last = (n * angle) >> 5;
        if (last < -1 && k >= last) {
            const int j = (k * intra_inv_angle(mode) + 128) >> 8;
            v = vert ? r[2 * n - j] : r[2 * n + j];
        }
    }
    out[k + n] = (uint8_t)v;
}
// Directional prediction sample (x, y) from build_refm's array (intra_pred_sample's
// angular branch; the axis modes 10 / 26 go through pred_fast).
__device__ __forceinline__ int pred_angular(const uint8_t* refm, int n, int mode, int x, int y) {
    const int angle = HEVC_INTRA_ANGLE[mode];
    const bool vert = mode >= 18;
    const int a = vert ? y : x, b = vert ? x : y;
    const int idx = ((a + 1) * angle) >> 5, fact = ((a + 1) * angle) & 31;
    const uint8_t* p = refm + n + b + idx + 1;
    return fact ? ((32 - fact) * (int)p[0] + fact * (int)p[1] + 16) >> 5 : (int)p[0];
}
// Luma references of `mode` for a 16x16 CU: the [1 2 1]-filtered copy when filterFlag.
__device__ __forceinline__ const uint8_t* luma_ref(const CuLds& L, int mode) {
    return intra_filter_flag(mode, 4, 0) ? L.ref + 65 : L.ref;
}
// Intra prediction of the whole CU into L.pred for `mode` (refs in L.ref).
__device__ __forceinline__ void intra_pred_cu(CuLds& L, int mode) {
    const int l = lane();
    const uint8_t* ry = luma_ref(L, mode);
    const bool basic = intra_mode_basic(mode);
    const int dcy = dc_value(L.ref, 16, 4);
    const int dcu = dc_value(L.ref + 130, 8, 3), dcv = dc_value(L.ref + 163, 8, 3);
    if (!basic) {
        build_refm(ry, 16, mode, L.refm[0]);
        build_refm(L.ref + 130, 8, mode, L.refm[1]);
        build_refm(L.ref + 163, 8, mode, L.refm[2]);
        wsync();
    }
    for (int i = l; i < kCoefPerCu; i += 64) {
        int v;
        if (i < 256) {
            v = basic ? pred_fast(ry, 16, 4, mode, true, dcy, i & 15, i >> 4)
                      : pred_angular(L.refm[0], 16, mode, i & 15, i >> 4);
        } else {
            const int j = i - 256, c = j >> 6;
            v = basic ? pred_fast(L.ref + 130 + 33 * c, 8, 3, mode, false, c ? dcv : dcu, j & 7, (j >> 3) & 7)
                      : pred_angular(L.refm[1 + c], 8, mode, j & 7, (j >> 3) & 7);
        }
        L.pred[i] = (uint8_t)v;
    }
    wsync();
}
__device__ __forceinline__ void intra_refs(CuLds& L, const Planes& P, const FrameArgs& f, int cx, int cy, bool left, bool top,
                           bool tr) {
    fill_ref(P.y, f.stride_y, cx * 16, cy * 16, 16, left, top, tr, L.ref);
    fill_ref(P.u, f.stride_c, cx * 8, cy * 8, 8, left, top, tr, L.ref + 130);
    fill_ref(P.v, f.stride_c, cx * 8, cy * 8, 8, left, top, tr, L.ref + 163);
    wsync();
    filter_ref(L.ref, 16, L.ref + 65);
    wsync();
}

// Open-loop intra mode per CU of I slices (all CUs in parallel).
__global__ __launch_bounds__(256) void k_hevc_intra_prep(HevcArgs A) {
    __shared__ CuLds Lw[4];
    const FrameArgs& f = A.f;
    CuLds& L = Lw[threadIdx.x >> 6];
    const int n = f.mb_w * f.mb_h;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= n) return;   // wave-uniform; no block barriers below
    const int cx = idx % f.mb_w, cy = idx / f.mb_w;
    const SliceTask t = f.tasks[cy / f.rows_per_slice];
    if (t.final_action != ACT_I) return;
    const bool left = cx > 0, top = cy > t.first_row, tr = top && cx + 1 < f.mb_w;
    intra_refs(L, f.src, f, cx, cy, left, top, tr);
    load_src(L, f, cx, cy);
    wsync();
    const int l = lane();
    const int dc = dc_value(L.ref, 16, 4);
    int best = 1, best_sad = 0x7fffffff;
    for (int k = 0; k < 35; k++) {   // HEVC_INTRA_ORDER, SAD + intra_mode_bias (hevc_cpu.cpp)
        const int m = HEVC_INTRA_ORDER[k];
        const uint8_t* r = luma_ref(L, m);
        const bool basic = intra_mode_basic(m);
        if (!basic) {
            build_refm(r, 16, m, L.refm[0]);
            wsync();
        }
        int sad = 0;
        for (int i = l; i < 256; i += 64)
            sad += sk_abs((int)L.src[i] - (basic ? pred_fast(r, 16, 4, m, true, dc, i & 15, i >> 4)
                                                 : pred_angular(L.refm[0], 16, m, i & 15, i >> 4)));
        sad = wsum(sad) + intra_mode_bias(m, t.qp);
        if (sad < best_sad) { best_sad = sad; best = m; }
        wsync();   // refm is rebuilt by the next mode
    }
    if (l == 0) {
        CuInfo cu;
        memset(&cu, 0, sizeof(cu));
        cu.mode = CU_INTRA;
        cu.intra_mode = (uint8_t)best;
        A.cus[idx] = cu;
    }
}

// I slices: one workgroup per slice, wave w = CTB row w of the slice, CTB x coded at
// step x + 2w (the top-right CTB is one step older: WPP / intra availability order).
template <int MAXR>
__global__ __launch_bounds__(64 * MAXR) void k_hevc_intra(HevcArgs A) {
    __shared__ CuLds Lw[MAXR];
    __shared__ int8_t T[256];
    const FrameArgs& f = A.f;
    const SliceTask t = f.tasks[blockIdx.x];
    if (t.final_action != ACT_I) return;   // block-uniform
    load_t16(T);
    __syncthreads();
    const int w = threadIdx.x >> 6, l = lane();
    CuLds& L = Lw[w];
    const int rows = t.num_rows, steps = f.mb_w + 2 * (rows - 1);
    const int cy = t.first_row + w;
    __builtin_amdgcn_s_setprio(3);
    for (int step = 0; step < steps; step++) {
        const int cx = step - 2 * w;
        if (w < rows && cx >= 0 && cx < f.mb_w) {
            const int idx = cy * f.mb_w + cx;
            const bool left = cx > 0, top = cy > t.first_row, tr = top && cx + 1 < f.mb_w;
            const int mode = __builtin_amdgcn_readfirstlane(A.cus[idx].intra_mode);
            intra_refs(L, f.rec, f, cx, cy, left, top, tr);
            load_src(L, f, cx, cy);
            intra_pred_cu(L, mode);
            const int cbf = code_cu_wave(L, T, t.qp, true, A.coefs + (size_t)idx * kCoefPerCu);
            store_rec(L, f, cx, cy);
            if (l == 0) {
                CuInfo cu;
                memset(&cu, 0, sizeof(cu));
                cu.mode = CU_INTRA;
                cu.intra_mode = (uint8_t)mode;
                cu.cbf = (uint8_t)cbf;
                cu.qp = (uint8_t)t.qp;
                A.cus[idx] = cu;
                f.me[idx].mvx = 0;
                f.me[idx].mvy = 0;
                f.me[idx].ref = 0;
                f.me[idx].fx = f.me[idx].fy = 0;
            }
        }
        __syncthreads();   // this step's reconstruction is visible to the next step's neighbours
    }
}

// ---------------------------------------------------------------------------
// CU syntax -> bin entries: one thread per CU (a wave binarises 64 CUs at once).
__global__ __launch_bounds__(256) void k_hevc_bins(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int n = f.mb_w * f.mb_h;
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= n) return;
    const int cx = idx % f.mb_w, cy = idx / f.mb_w;
    const SliceTask t = f.tasks[cy / f.rows_per_slice];
    const bool p_slice = t.final_action != ACT_I;
    const bool left = cx > 0, top = cy > t.first_row;
    const CuInfo cu = A.cus[idx];
    const int skip_ctx = (left && A.cus[idx - 1].mode == CU_SKIP) + (top && A.cus[idx - f.mb_w].mode == CU_SKIP);
    const int cand_a = (left && A.cus[idx - 1].mode == CU_INTRA) ? A.cus[idx - 1].intra_mode : 1;
    BinBuf w{A.bins + (size_t)idx * kCuBinCap, 0};
    sao_bins(w, A.sao[idx], left, top);   // CTB-level SAO syntax (k_hevc_sao_row's decision)
    code_cu(w, cu, A.coefs + (size_t)idx * kCoefPerCu, p_slice, skip_ctx, cand_a);
    const bool last_row = cy == t.first_row + t.num_rows - 1;
    w.term(last_row && cx == f.mb_w - 1);
    if (!last_row && cx == f.mb_w - 1) w.term(1);   // end_of_subset_one_bit closes the row's substream
    A.bin_n[idx] = w.n;
}

// Lane `ln` (wave-uniform) of `v` takes the uniform value `x`: v_writelane_b32 with the
// lane index in M0 (one SGPR read per VALU op on gfx9; no compiler builtin for it).
__device__ __forceinline__ int writelane(int x, int ln, int v) {
    asm("s_nop 0\n\tv_writelane_b32 %0, %1, m0"
        : "+v"(v)
        : "s"(__builtin_amdgcn_readfirstlane(x)), "{m0}"(__builtin_amdgcn_readfirstlane(ln)));
    return v;
}

// WPP context states at each row start of a slice (9.3.2.4: the states after the second
// CTB of the row above). Thread c owns context c and replays only that context's bins
// of the two CTBs, from k_pc_sort's per-context lists: the chains run in parallel and
// each is a few entries long.
__global__ __launch_bounds__(192) void k_hevc_sync(HevcArgs A) {
    __shared__ uint8_t nlps[64];
    const FrameArgs& f = A.f;
    const SliceTask t = f.tasks[blockIdx.x];
    const int c = threadIdx.x;
    if (c < 64) nlps[c] = CABAC_NEXT_LPS[c];
    __syncthreads();
    if (c >= CTX_COUNT) return;
    const int it = t.final_action == ACT_I ? 0 : 1;
    const uint8_t init = ctx_init_state(HEVC_CTX_INIT[it][c], t.qp);
    uint32_t st = init;
    A.sync[(size_t)t.first_row * CTX_COUNT + c] = init;
    for (int r = 1; r < t.num_rows; r++) {
        const int prev = t.first_row + r - 1;
        if (f.mb_w >= 2) {
            const uint16_t* co = A.coff + ((size_t)prev * kPcCtxOff + c) * f.mb_w;
            for (int cx = 0; cx < 2; cx++) {
                const uint16_t* sp = A.srt + (size_t)(prev * f.mb_w + cx) * kCuBinCap;
                const int hi = co[f.mb_w + cx];
                for (int k = co[cx]; k < hi; k++) {
                    const uint32_t bin = sp[k] & 1u, mps = st & 1u, s6 = st >> 1;
                    st = bin == mps ? (((s6 < 62 ? s6 + 1 : 62) << 1) | mps)
                                    : (((uint32_t)nlps[s6] << 1) | (s6 == 0 ? mps ^ 1u : mps));
                }
            }
        } else {
            st = init;
        }
        A.sync[(size_t)(t.first_row + r) * CTX_COUNT + c] = (uint8_t)st;
    }
}

// ---------------------------------------------------------------------------
// Chunk-parallel substream coding (codec/hevc_pcabac.h has the derivation and the host
// model): k_pc_sort -> k_pc_model -> k_pc_rmap -> k_pc_compose -> k_pc_code ->
// k_pc_merge. Chunk = CTB, so every phase but the per-row composition and merge runs
// one wave per CTB or per (CTB row, context). Same bytes as CabacEncoder (hevc_core.h).
constexpr int kPcMaxRowCtb = 512;   // CTBs per row (8K width); alloc_hevc checks it

// One wave per CTB: stable counting sort of its context bins by context index.
__global__ __launch_bounds__(256) void k_pc_sort(HevcArgs A) {
    __shared__ int cnt_s[4][kPcCtxOff];
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int idx = blockIdx.x * 4 + w;
    if (idx >= f.mb_w * f.mb_h) return;
    int* cnt = cnt_s[w];
    for (int i = l; i < kPcCtxOff; i += 64) cnt[i] = 0;
    wsync();
    const uint16_t* b = A.bins + (size_t)idx * kCuBinCap;
    const int nb = __builtin_amdgcn_readfirstlane(A.bin_n[idx]);
    for (int base = 0; base < nb; base += 64) {
        const int i = base + l;
        const uint32_t e = i < nb ? b[i] : 0x8000u;
        if ((e & 0x80ffu) < (uint32_t)CTX_TERM) atomicAdd(&cnt[e & 0xffu], 1);
    }
    wsync();
    int v[3], sum = 0;   // exclusive prefix; lane l owns counters 3l .. 3l + 2
#pragma unroll
    for (int k = 0; k < 3; k++) {
        v[k] = 3 * l + k < kPcCtxOff ? cnt[3 * l + k] : 0;
        sum += v[k];
    }
    int inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o);
        if (l >= o) inc += t;
    }
    int run = inc - sum;
    wsync();
    // coff is [CTB row][context][CTB column]: k_pc_model and k_hevc_sync read one
    // context's offsets along a row as one contiguous run
    const int cy = idx / f.mb_w, cx = idx - cy * f.mb_w;
    uint16_t* co = A.coff + (size_t)cy * kPcCtxOff * f.mb_w + cx;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        if (3 * l + k < kPcCtxOff) {
            cnt[3 * l + k] = run;
            co[(size_t)(3 * l + k) * f.mb_w] = (uint16_t)run;
        }
        run += v[k];
    }
    wsync();
    uint16_t* sp = A.srt + (size_t)idx * kCuBinCap;
    const uint64_t lt = (1ull << l) - 1;
    for (int base = 0; base < nb; base += 64) {
        const int i = base + l;
        const uint32_t e = i < nb ? b[i] : 0x8000u;
        const bool valid = (e & 0x80ffu) < (uint32_t)CTX_TERM;
        const uint32_t key = e & 0xffu;
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; bit++) {
            const bool kb = (key >> bit) & 1u;
            const uint64_t bb = __ballot(kb);
            m &= kb ? bb : ~bb;
        }
        const int rank = __popcll(m & lt), tot = __popcll(m);
        const int at = valid ? cnt[key] : 0;
        wsync();
        if (valid && rank == tot - 1) cnt[key] = at + tot;
        wsync();
        if (valid) sp[at + rank] = (uint16_t)((i << 1) | ((e >> 8) & 1u));
    }
}

// One wave per (CTB row, context): the context's state chain along the row, from its
// WPP start state; each context bin is rewritten in place as a modelled entry (LPS state,
// is-LPS). The CTBs holding the context are listed with the prefix of their counts; the
// chain itself runs as up to 64 speculative segments, one per lane (below).
__global__ __launch_bounds__(256) void k_pc_model(HevcArgs A) {
    __shared__ uint2 lst_s[4][kPcMaxRowCtb + 1];   // (cx | lo << 16, chain position of its first entry)
    __shared__ uint8_t nl_s[4][64];                // CABAC_NEXT_LPS
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int cy = blockIdx.x, c = blockIdx.y * 4 + w;
    if (c >= CTX_COUNT) return;
    uint2* L = lst_s[w];
    const int row0 = cy * f.mb_w;
    const uint64_t lt = (1ull << l) - 1;
    int n = 0, tot = 0;
    for (int g = 0; g < f.mb_w; g += 64) {
        const int cx = g + l;
        int lo = 0, cnt = 0;
        if (cx < f.mb_w) {
            const uint16_t* co = A.coff + ((size_t)cy * kPcCtxOff + c) * f.mb_w + cx;
            lo = co[0];
            cnt = co[f.mb_w] - lo;
        }
        int inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(inc, o);
            if (l >= o) inc += t;
        }
        const uint64_t m = __ballot(cnt > 0);
        if (cnt > 0) L[n + __popcll(m & lt)] = make_uint2((uint32_t)cx | ((uint32_t)lo << 16), (uint32_t)(tot + inc - cnt));
        n += __popcll(m);
        tot += __builtin_amdgcn_readlane(inc, 63);
    }
    n = __builtin_amdgcn_readfirstlane(n);
    tot = __builtin_amdgcn_readfirstlane(tot);
    if (l == 0) L[n] = make_uint2(0u, (uint32_t)tot);
    wsync();
    if (tot == 0) return;
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane(A.sync[(size_t)cy * CTX_COUNT + c]);
    uint8_t* nl = nl_s[w];
    nl[l] = CABAC_NEXT_LPS[l];
    wsync();
    // The chain is cut into up to 64 segments, lane = segment (>= 32 entries each).
    // Pass 1 runs every segment from a guessed start state; CABAC states forget their
    // start quickly (MPS runs saturate, LPS steps contract), so segment j-1's end state
    // from the guess is almost always segment j's true start. Pass 2 runs from those
    // starts and writes the modelled entries; a start that does not match the true end
    // of the segment before it is corrected and its segment re-run (loop until none).
    const int seglen = tot > 64 * 32 ? (tot + 63) / 64 : 32;
    const int nseg = (tot + seglen - 1) / seglen;
    const int p0 = l * seglen, p1 = p0 + seglen < tot ? p0 + seglen : tot;
    const bool act = l < nseg;
    auto run_seg = [&](uint32_t s, bool write) __attribute__((always_inline)) -> uint32_t {
        int klo = 0, khi = n;   // the list item holding position p0: L[k].y <= p0 < L[k+1].y
        while (khi - klo > 1) {
            const int mid = (klo + khi) >> 1;
            if ((int)L[mid].y <= p0) klo = mid;
            else khi = mid;
        }
        int k = klo;
        uint2 it = L[k];
        int nxt = (int)L[k + 1].y;
        for (int p = p0; p < p1; p += 16) {
            uint32_t v[16], cu[16];
#pragma unroll
            for (int j = 0; j < 16; j++) {   // 16 independent loads in flight
                const int q = p + j < p1 ? p + j : p1 - 1;
                while (q >= nxt) {
                    k++;
                    it = L[k];
                    nxt = (int)L[k + 1].y;
                }
                cu[j] = (uint32_t)row0 + (it.x & 0xffffu);
                v[j] = A.srt[(size_t)cu[j] * kCuBinCap + (it.x >> 16) + (uint32_t)(q - (int)it.y)];
            }
#pragma unroll
            for (int j = 0; j < 16; j++) {
                if (p + j < p1) {
                    const uint32_t st6 = s >> 1, mps = s & 1u, lp = (v[j] & 1u) ^ mps;
                    if (write) A.bins[(size_t)cu[j] * kCuBinCap + (v[j] >> 1)] = (uint16_t)(kPcModeled | (lp << 6) | st6);
                    s = lp ? (((uint32_t)nl[st6] << 1) | (st6 == 0 ? mps ^ 1u : mps))
                           : (((st6 < 62u ? st6 + 1u : 62u) << 1) | mps);
                }
            }
        }
        return s;
    };
    uint32_t e1 = act ? run_seg(s0, false) : 0u;
    uint32_t T = (uint32_t)__shfl_up((int)e1, 1);
    if (l == 0) T = s0;
    bool need = act;
    for (;;) {
        const uint32_t e2 = need ? run_seg(T, true) : e1;
        e1 = e2;   // true end of every segment whose start was right
        uint32_t tn = (uint32_t)__shfl_up((int)e2, 1);
        if (l == 0) tn = s0;
        const uint64_t bad = __ballot(act && tn != T);
        if (!bad) break;
        const int first = (int)__builtin_ctzll(bad);
        need = act && l >= first;
        if (need) T = tn;
    }
}

// One wave per CTB: the chunk's range map. Lane l follows the start ranges 256 + 4l .. +3
// through the chunk's entries (bypass runs and terminating bins shift all of them alike).
__global__ __launch_bounds__(256) void k_pc_rmap(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int idx = blockIdx.x * 4 + w;
    if (idx >= f.mb_w * f.mb_h) return;
    const int lps_v = (int)((uint32_t)CABAC_LPS[l][0] | ((uint32_t)CABAC_LPS[l][1] << 8) |
                            ((uint32_t)CABAC_LPS[l][2] << 16) | ((uint32_t)CABAC_LPS[l][3] << 24));
    uint32_t r[4], K[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        r[k] = 256u + 4u * (uint32_t)l + (uint32_t)k;
        K[k] = 0;
    }
    uint32_t kb = 0;
    const uint16_t* b = A.bins + (size_t)idx * kCuBinCap;
    const int nb = __builtin_amdgcn_readfirstlane(A.bin_n[idx]);
    uint32_t cur = b[l < nb ? l : nb - 1];
    for (int base = 0; base < nb; base += 64) {
        const int pi = base + 64 + l;
        const uint32_t nxt = b[pi < nb ? pi : nb - 1];
        const int m = nb - base < 64 ? nb - base : 64;
        for (int i = 0; i < m; i++) {
            const uint32_t e = (uint32_t)__builtin_amdgcn_readlane((int)cur, i);
            if ((e & 0xC000u) == kPcModeled) {
                const uint32_t lps4 = (uint32_t)__builtin_amdgcn_readlane(lps_v, (int)(e & 63u));
                if (e & 64u) {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t nr = (lps4 >> ((r[k] >> 3) & 24u)) & 0xffu;
                        const uint32_t z = (uint32_t)__builtin_clz(nr) - 23u;
                        r[k] = nr << z;
                        K[k] += z;
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t nr = r[k] - ((lps4 >> ((r[k] >> 3) & 24u)) & 0xffu);
                        const uint32_t z = nr < 256u ? 1u : 0u;
                        r[k] = nr << z;
                        K[k] += z;
                    }
                }
            } else if (e & 0x8000u) {
                kb += ((e >> 12) & 7u) + 1u;
            } else if ((e >> 8) & 1u) {
#pragma unroll
                for (int k = 0; k < 4; k++) r[k] = 256u;
                kb += 7u;
            } else {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t nr = r[k] - 2u;
                    const uint32_t z = nr < 256u ? 1u : 0u;
                    r[k] = nr << z;
                    K[k] += z;
                }
            }
        }
        cur = nxt;
    }
    uint4 o;
    o.x = r[0] | ((K[0] + kb) << 9);
    o.y = r[1] | ((K[1] + kb) << 9);
    o.z = r[2] | ((K[2] + kb) << 9);
    o.w = r[3] | ((K[3] + kb) << 9);
    reinterpret_cast<uint4*>(A.rmap + (size_t)idx * 256)[l] = o;
}

// One wave per CTB row: start range and stream bit offset of every chunk, one map
// lookup each (a readlane); the maps of the next 8 CTBs are in flight.
__global__ __launch_bounds__(64) void k_pc_compose(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int cy = blockIdx.x, l = lane();
    const int row0 = cy * f.mb_w, nw = f.mb_w;
    constexpr int D = 8;
    uint4 buf[D];
#pragma unroll
    for (int d = 0; d < D; d++)
        buf[d] = reinterpret_cast<const uint4*>(A.rmap + (size_t)(row0 + (d < nw ? d : nw - 1)) * 256)[l];
    uint32_t r = 510, T = 0;
    int vr = 0, vt = 0;   // lane j: chunk j of the current 64
    for (int cx0 = 0; cx0 < nw; cx0 += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int cx = cx0 + d;
            if (cx < nw) {
                const int j = (int)r - 256, ln = j >> 2, comp = j & 3;
                const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)buf[d].x, ln);
                const uint32_t y = (uint32_t)__builtin_amdgcn_readlane((int)buf[d].y, ln);
                const uint32_t z = (uint32_t)__builtin_amdgcn_readlane((int)buf[d].z, ln);
                const uint32_t ww = (uint32_t)__builtin_amdgcn_readlane((int)buf[d].w, ln);
                const uint32_t val = comp == 0 ? x : (comp == 1 ? y : (comp == 2 ? z : ww));
                vr = writelane((int)r, cx & 63, vr);
                vt = writelane((int)T, cx & 63, vt);
                if ((cx & 63) == 63 || cx == nw - 1) {
                    if (l <= (cx & 63)) {
                        A.cu_r[row0 + (cx & ~63) + l] = (uint16_t)vr;
                        A.cu_t[row0 + (cx & ~63) + l] = (uint32_t)vt;
                    }
                }
                r = val & 511u;
                T += val >> 9;
            }
            const int nx = cx + D < nw ? cx + D : nw - 1;
            buf[d] = reinterpret_cast<const uint4*>(A.rmap + (size_t)(row0 + nx) * 256)[l];
        }
    }
    if (l == 0) A.row_bits[cy] = T;
}

// One wave per CTB: the chunk coded from V = 0 (PcCoder, scalar state) and fully
// flushed; bytes gathered in a VGPR (lane = 4 bytes) and stored every 256: the exclusive
// ones into the row substream, the last two into the chunk's tail.
__global__ __launch_bounds__(256) void k_pc_code(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int idx = blockIdx.x * 4 + w;
    if (idx >= f.mb_w * f.mb_h) return;
    const int cy = idx / f.mb_w, cx = idx - cy * f.mb_w;
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)A.cu_t[idx]);
    const uint32_t tn = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(cx + 1 < f.mb_w ? A.cu_t[idx + 1] : A.row_bits[cy]));
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)A.cu_r[idx]);
    const int g0 = (int)(t0 >> 3), nex = (int)(tn >> 3) - g0;
    uint8_t* out = A.sub + (size_t)cy * A.sub_stride + g0;
    uint8_t* tl = A.tail + (size_t)idx * 2;
    int ob = 0, opos = 0, flushed = 0;
    uint32_t acc = 0;
    auto store = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int p = 4 * l + k;
            if (p < opos) {
                const uint8_t byte = (uint8_t)((uint32_t)ob >> (8 * k));
                const int q = flushed + p;
                if (q < nex) out[q] = byte;
                else tl[q - nex] = byte;
            }
        }
        flushed += opos;
        opos = 0;
    };
    auto emit = [&](uint32_t byte) __attribute__((always_inline)) {
        acc |= (byte & 0xffu) << (8 * (opos & 3));
        opos++;
        if ((opos & 3) == 0) {
            ob = writelane((int)acc, (opos >> 2) - 1, ob);
            acc = 0;
            if (opos == 256) store();
        }
    };
    const int lps_v = (int)((uint32_t)CABAC_LPS[l][0] | ((uint32_t)CABAC_LPS[l][1] << 8) |
                            ((uint32_t)CABAC_LPS[l][2] << 16) | ((uint32_t)CABAC_LPS[l][3] << 24));
    auto lps4 = [&](uint32_t st) __attribute__((always_inline)) {
        return (uint32_t)__builtin_amdgcn_readlane(lps_v, (int)st);
    };
    PcCoder c;
    c.start(r0, (int)(t0 & 7));
    const uint16_t* b = A.bins + (size_t)idx * kCuBinCap;
    const int nb = __builtin_amdgcn_readfirstlane(A.bin_n[idx]);
    uint32_t cur = b[l < nb ? l : nb - 1];
    for (int base = 0; base < nb; base += 64) {
        const int pi = base + 64 + l;
        const uint32_t nxt = b[pi < nb ? pi : nb - 1];
        const int m = nb - base < 64 ? nb - base : 64;
        for (int i = 0; i < m; i++) c.code((uint32_t)__builtin_amdgcn_readlane((int)cur, i), emit, lps4);
        cur = nxt;
    }
    c.flush(emit);
    if (opos & 3) ob = writelane((int)acc, opos >> 2, ob);
    store();
}

// One wave per CTB row: adds every chunk's tail into the substream (a 256-byte window
// of it in a VGPR; carries run toward the start), writes the rbsp stop bit, then counts
// the emulation-prevention bytes (same rule as k_hevc_ep_copy).
__global__ __launch_bounds__(64) void k_pc_merge(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int cy = blockIdx.x, l = lane();
    const int row0 = cy * f.mb_w;
    const uint32_t T = (uint32_t)__builtin_amdgcn_readfirstlane((int)A.row_bits[cy]);
    const int excl = (int)(T >> 3), nbytes = excl + 2;
    uint8_t* out = A.sub + (size_t)cy * A.sub_stride;
    int wb = 0;
    uint32_t win = 0;
    auto load_win = [&]() __attribute__((always_inline)) {
        const int q = wb + 4 * l;
        uint32_t v = 0;
        if (q + 4 <= excl) {
            v = *reinterpret_cast<const uint32_t*>(out + q);
        } else {
            for (int k = 0; k < 4; k++)
                if (q + k < excl) v |= (uint32_t)out[q + k] << (8 * k);
        }
        win = v;
    };
    auto store_win = [&]() __attribute__((always_inline)) {
        const int q = wb + 4 * l;
        if (q + 4 <= nbytes) {
            *reinterpret_cast<uint32_t*>(out + q) = win;
        } else {
            for (int k = 0; k < 4; k++)
                if (q + k < nbytes) out[q + k] = (uint8_t)(win >> (8 * k));
        }
    };
    auto get = [&](int q) __attribute__((always_inline)) -> uint32_t {
        const int o = q - wb;
        return ((uint32_t)__builtin_amdgcn_readlane((int)win, o >> 2) >> ((o & 3) * 8)) & 0xffu;
    };
    auto set = [&](int q, uint32_t byte) __attribute__((always_inline)) {
        const int o = q - wb, sh = (o & 3) * 8;
        const uint32_t wv = (uint32_t)__builtin_amdgcn_readlane((int)win, o >> 2);
        win = (uint32_t)writelane((int)((wv & ~(0xffu << sh)) | (byte << sh)), o >> 2, (int)win);
    };
    load_win();
    for (int g = 0; g < f.mb_w; g += 64) {
        const int cx = g + l;
        int p_l = 0, t_l = 0;
        if (cx < f.mb_w) {
            p_l = (int)((cx + 1 < f.mb_w ? A.cu_t[row0 + cx + 1] : T) >> 3);
            t_l = (int)((uint32_t)A.tail[2 * (row0 + cx)] | ((uint32_t)A.tail[2 * (row0 + cx) + 1] << 8));
        }
        const int m = f.mb_w - g < 64 ? f.mb_w - g : 64;
        for (int j = 0; j < m; j++) {
            const int p = __builtin_amdgcn_readlane(p_l, j);
            const uint32_t tv = (uint32_t)__builtin_amdgcn_readlane(t_l, j);
            if (p + 2 > wb + 256) {
                store_win();
                __threadfence();
                wb = p & ~3;
                load_win();
            }
            uint32_t v = ((get(p) << 8) | get(p + 1)) + (((tv & 0xffu) << 8) | (tv >> 8));
            set(p + 1, v & 0xffu);
            set(p, (v >> 8) & 0xffu);
            for (int q = p - 1; (v >> 16) && q >= 0; q--) {   // carry (rare)
                if (q >= wb) {
                    v = get(q) + 1;
                    set(q, v & 0xffu);
                } else {
                    __threadfence();
                    v = (uint32_t)__builtin_amdgcn_readfirstlane((int)out[q]) + 1;
                    if (l == 0) out[q] = (uint8_t)v;
                }
                v <<= 8;
            }
        }
    }
    const uint32_t sb = T + 1;   // rbsp stop bit, then zeros
    const int qs = (int)(sb >> 3);
    set(qs, (get(qs) & (0xff00u >> (sb & 7))) | (0x80u >> (sb & 7)));
    store_win();
    __threadfence();
    const int size = qs + 1;
    int last_nz = -1, ins_total = 0;
    for (int base = 0; base < size; base += 64) {
        const int i = base + l;
        const int bv = i < size ? out[i] : 1;
        int p = bv != 0 ? i : -1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int q = __shfl_up(p, d);
            if (l >= d) p = max(p, q);
        }
        int prev_nz = __shfl_up(p, 1);
        if (l == 0) prev_nz = -1;
        prev_nz = max(prev_nz, last_nz);
        const int z = i - 1 - prev_nz;
        const int ins = (i < size && bv <= 3 && z >= 2 && (z & 1) == 0) ? 1 : 0;
        ins_total += wsum(ins);
        last_nz = max(last_nz, __shfl(p, 63));
    }
    if (l == 0) {
        A.sub_size[cy] = size;
        A.sub_esc[cy] = size + ins_total;
        if (A.dbg) {
            A.dbg[4 * cy + 0] = 0;
            A.dbg[4 * cy + 1] = T;
            A.dbg[4 * cy + 2] = (unsigned long long)size;
            A.dbg[4 * cy + 3] = 0;
        }
    }
}

// Slice header + NAL prefix per slice; substream offsets for k_hevc_ep_copy.
__global__ __launch_bounds__(64) void k_hevc_hdr(HevcArgs A) {
    __shared__ uint8_t hdr[1024];
    __shared__ int esc[256];
    const FrameArgs& f = A.f;
    const int s = blockIdx.x;
    const SliceTask t = f.tasks[s];
    const int l = lane();
    for (int i = l; i < 1024; i += 64) hdr[i] = 0;
    for (int i = l; i < t.num_rows; i += 64) esc[i] = A.sub_esc[t.first_row + i];
    bool idr = true;
    for (int i = l; i < f.num_slices; i += 64) idr &= f.tasks[i].final_action == ACT_I && f.tasks[i].idr_on_intra;
    idr = __syncthreads_and(idr);
    if (l == 0) {
        SliceHeader h;
        h.first_slice = s == 0;
        h.idr = idr;
        h.address = t.first_row * f.mb_w;
        h.address_bits = A.addr_bits;
        h.slice_type = t.final_action == ACT_I ? 2 : 1;
        h.poc_lsb = t.frame_num & ((1 << kLog2MaxPocLsb) - 1);
        h.qp_delta = t.qp - 26;
        h.num_entry = t.num_rows - 1;
        h.entry = esc;
        const int hn = write_slice_header(hdr, h);
        const int hesc = ep_escape(hdr, hn, nullptr);
        int total = 6 + hesc;
        int off = total;
        for (int r = 0; r < t.num_rows; r++) {
            A.row_off[t.first_row + r] = off;
            off += esc[r];
        }
        total = off;
        const bool fits = total <= A.out_slot;
        uint8_t* o = fits ? A.out_host + (size_t)s * A.out_slot : A.out_dev + (size_t)s * A.out_dev_slot;
        o[0] = 0; o[1] = 0; o[2] = 0; o[3] = 1;
        o[4] = (uint8_t)((idr ? kNalIdrWRadl : kNalTrailR) << 1);
        o[5] = 1;
        ep_escape(hdr, hn, o + 6);
        __hip_atomic_store(A.out_size + s, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Emulation prevention + copy of one row's substream, wave-parallel: byte i of the
// substream is preceded by an inserted 0x03 iff it is <= 3 and the zero run before it
// has even length >= 2 (equivalent to the sequential rule; the previous piece ends in a
// non-zero byte).
__global__ __launch_bounds__(64) void k_hevc_ep_copy(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int cy = blockIdx.x;
    const int s = cy / f.rows_per_slice;
    const int total = __hip_atomic_load(A.out_size + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const bool fits = total <= A.out_slot;
    uint8_t* o = (fits ? A.out_host + (size_t)s * A.out_slot : A.out_dev + (size_t)s * A.out_dev_slot) + A.row_off[cy];
    const uint8_t* in = A.sub + (size_t)cy * A.sub_stride;
    const int n = A.sub_size[cy];
    const int l = lane();
    int last_nz = -1;   // index of the last non-zero byte before the current chunk (-1: none yet,
                        // the byte before the substream is non-zero)
    int opos = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + l;
        const int b = i < n ? in[i] : 1;
        // inclusive max-scan of the positions of non-zero bytes
        int p = b != 0 ? i : -1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int q = __shfl_up(p, d);
            if (l >= d) p = max(p, q);
        }
        int prev_nz = __shfl_up(p, 1);
        if (l == 0) prev_nz = -1;
        prev_nz = max(prev_nz, last_nz);
        const int z = i - 1 - prev_nz;   // zeros immediately before byte i
        const int ins = (i < n && b <= 3 && z >= 2 && (z & 1) == 0) ? 1 : 0;
        int cnt = ins;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int q = __shfl_up(cnt, d);
            if (l >= d) cnt += q;
        }
        if (i < n) {
            const int at = i + opos + cnt;   // insertions before this chunk + up to this byte
            if (ins) o[at - 1] = 3;
            o[at] = (uint8_t)b;
        }
        opos += __shfl(cnt, 63);
        last_nz = max(last_nz, __shfl(p, 63));
    }
}

// Deblocking (hevc_core.h deblock_picture, in parallel): every edge segment is an
// independent work item (edges are 8 samples apart and a filter reads 4 / changes at
// most 3 samples per side). k_hevc_dbk_v: all vertical edges (luma 4-line segments on
// the 8x8 grid, chroma lines of CU edges); k_hevc_dbk_h: the horizontal edges on its
// output, none between slices.
__device__ __forceinline__ bool cu_intra_edge(const CuInfo& p, const CuInfo& q) {
    return p.mode == CU_INTRA || q.mode == CU_INTRA;
}
__global__ __launch_bounds__(256) void k_hevc_dbk_v(HevcArgs A) {
    const h264::gpu::FrameArgs& f = A.f;
    const int cw = f.mb_w, ch = f.mb_h, ne = cw - 1, nel = 2 * cw - 1;
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int nl = ch * 4 * nel, nc = ch * 8 * ne;
    if (e < nl) {
        const int x = 8 * (1 + e % nel), seg = e / nel;
        dbk_luma_edge(f.rec.y, f.stride_y, A.cus, cw, true, x, 4 * seg);
    } else if (e < nl + 2 * nc) {
        const int k0 = e - nl, plane = k0 / nc, k = k0 % nc;
        const int cx = 1 + k % ne, line = k / ne, cy = line >> 3;
        const CuInfo p = A.cus[cy * cw + cx - 1], q = A.cus[cy * cw + cx];
        if (cu_intra_edge(p, q))
            dbk_chroma_line((plane ? f.rec.v : f.rec.u) + (size_t)line * f.stride_c + cx * 8, 1, (p.qp + q.qp + 1) >> 1);
    }
}

__global__ __launch_bounds__(256) void k_hevc_dbk_h(HevcArgs A) {
    const h264::gpu::FrameArgs& f = A.f;
    const int cw = f.mb_w, ch = f.mb_h, ne = ch - 1, nel = 2 * ch - 1;
    if (nel <= 0) return;
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int nl = nel * cw * 4, nc = ne * cw * 8;
    if (e < nl) {
        const int y = 8 * (1 + e / (cw * 4)), x4 = e % (cw * 4);
        if (!(y & 8) && (y >> 4) % f.rows_per_slice == 0) return;   // slice boundary
        dbk_luma_edge(f.rec.y, f.stride_y, A.cus, cw, false, y, 4 * x4);
    } else if (e < nl + 2 * nc) {
        const int k0 = e - nl, plane = k0 / nc, k = k0 % nc;
        const int cy = 1 + k / (cw * 8), col = k % (cw * 8), cx = col >> 3;
        if (cy % f.rows_per_slice == 0) return;
        const CuInfo p = A.cus[(cy - 1) * cw + cx], q = A.cus[cy * cw + cx];
        if (cu_intra_edge(p, q))
            dbk_chroma_line((plane ? f.rec.v : f.rec.u) + (size_t)(cy * 8) * f.stride_c + col, f.stride_c, (p.qp + q.qp + 1) >> 1);
    }
}

// ---------------------------------------------------------------------------
// SAO (codec/hevc_sao.h). Stats + each CTB's own decision: one wave per CTB, lanes
// accumulate the sample statistics of the deblocked picture with LDS atomics (integer
// sums, so the result is the host loop's), lane 0 runs the shared decision. Slices
// that are not coded (skip-all) keep empty stats and decide "off", like the host.
__device__ __forceinline__ const uint8_t* plane_of(const Planes& P, int c) { return c == 0 ? P.y : (c == 1 ? P.u : P.v); }
__device__ __forceinline__ uint8_t* plane_of(Planes& P, int c) { return c == 0 ? P.y : (c == 1 ? P.u : P.v); }
// Sample i (0..383) of CTB (cx, cy): component and plane coordinates.
__device__ __forceinline__ void ctb_sample(int i, int cx, int cy, int* c, int* x, int* y) {
    if (i < 256) {
        *c = 0; *x = cx * 16 + (i & 15); *y = cy * 16 + (i >> 4);
    } else {
        const int j = i - 256;
        *c = 1 + (j >> 6); *x = cx * 8 + (j & 7); *y = cy * 8 + ((j >> 3) & 7);
    }
}
__device__ __forceinline__ SaoPlane sao_plane_of(const FrameArgs& f, int c) {
    const int n = c ? 8 : 16;
    return SaoPlane{f.mb_w * n, f.mb_h * n, n, f.rows_per_slice};
}

__global__ __launch_bounds__(256) void k_hevc_sao_stats(HevcArgs A) {
    __shared__ SaoStats Sw[4][3];
    __shared__ SaoTables Tw[4];
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int idx = blockIdx.x * 4 + w;
    if (idx >= f.mb_w * f.mb_h) return;   // wave-uniform; no block barriers below
    const int cx = idx % f.mb_w, cy = idx / f.mb_w;
    const SliceTask t = f.tasks[cy / f.rows_per_slice];
    SaoStats* st = Sw[w];
    int32_t* z = reinterpret_cast<int32_t*>(st);
    for (int i = l; i < 3 * kSaoStatsInts; i += 64) z[i] = 0;
    wsync();
    if (t.final_action == ACT_P || t.final_action == ACT_I) {
        for (int i = l; i < kCoefPerCu; i += 64) {
            int c, x, y;
            ctb_sample(i, cx, cy, &c, &x, &y);
            const SaoPlane pl = sao_plane_of(f, c);
            const int stride = c ? f.stride_c : f.stride_y;
            const uint8_t* rec = plane_of(f.rec, c);
            const int v = rec[(size_t)y * stride + x];
            const int d = (int)plane_of(f.src, c)[(size_t)y * stride + x] - v;
            atomicAdd(&st[c].bo_s[v >> 3], d);
            atomicAdd(&st[c].bo_n[v >> 3], 1);
#pragma unroll
            for (int cls = 0; cls < 4; cls++) {
                if (!pl.eo_ok(cls, x, y)) continue;
                const int a = rec[(size_t)(y + sao_dy(cls, 0)) * stride + x + sao_dx(cls, 0)];
                const int b = rec[(size_t)(y + sao_dy(cls, 1)) * stride + x + sao_dx(cls, 1)];
                const int e = sao_edge_idx(v, a, b);
                if (e) {
                    atomicAdd(&st[c].eo_s[cls][e - 1], d);
                    atomicAdd(&st[c].eo_n[cls][e - 1], 1);
                }
            }
        }
    }
    wsync();
    int32_t* g = reinterpret_cast<int32_t*>(A.sao_stats + (size_t)3 * idx);
    for (int i = l; i < 3 * kSaoStatsInts; i += 64) g[i] = z[i];
    // the decision's tables lane-parallel (144 best offsets, then 96 band windows), the
    // pick on lane 0: the same functions, in the same order, as the host
    SaoTables& T = Tw[w];
    const int lam = sao_lambda(t.qp);
    for (int i = l; i < kSaoTableEntries; i += 64) sao_table_entry(st, lam, i, T);
    wsync();
    for (int i = l; i < 96; i += 64) sao_window(lam, i, T);
    wsync();
    if (l == 0) {
        SaoParams p;
        A.sao_cost[idx] = sao_pick(T, lam, p);
        A.sao_own[idx] = p;
    }
}

// Merge-candidate distortions: one thread per (CTB, candidate) (sao_merge_dists).
__global__ __launch_bounds__(256) void k_hevc_sao_md(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= f.mb_w * f.mb_h * kSaoMd) return;
    const int idx = t / kSaoMd, j = t - idx * kSaoMd, cx = idx % f.mb_w;
    const SaoParams* own_row = A.sao_own + (idx - cx);
    const SaoStats* st = A.sao_stats + (size_t)3 * idx;
    long long d = 0;
    if (j == kSaoMergeWin) d = sao_params_dist(st, own_row[cx]);
    else if (cx - 1 - j >= 0) d = sao_params_dist(st, own_row[cx - 1 - j]);
    A.sao_md[t] = d;
}

// Merge pass: one workgroup per CTB row. The row's candidate distortions, own
// parameters and costs are staged in LDS by all lanes; lane 0 then walks the row left to
// right (a merged CTB copies its left neighbour's final parameters) touching only LDS.
__global__ __launch_bounds__(64) void k_hevc_sao_row(HevcArgs A) {
    __shared__ long long md[kPcMaxRowCtb * kSaoMd];
    __shared__ SaoParams own[kPcMaxRowCtb];
    __shared__ long long cost[kPcMaxRowCtb];
    const FrameArgs& f = A.f;
    const int cy = blockIdx.x, l = threadIdx.x, W = f.mb_w;
    const size_t o = (size_t)cy * W;
    for (int i = l; i < W * kSaoMd; i += 64) md[i] = A.sao_md[o * kSaoMd + i];
    for (int i = l; i < W; i += 64) {
        own[i] = A.sao_own[o + i];
        cost[i] = A.sao_cost[o + i];
    }
    __syncthreads();
    if (l == 0) {
        const SliceTask t = f.tasks[cy / f.rows_per_slice];
        sao_row_merge(md, own, cost, W, t.qp, cy > t.first_row, A.sao + o);
    }
}

__device__ __forceinline__ bool sao_any(const SaoParams& p) { return (p.type[0] | p.type[1] | p.type[2]) != 0; }

// The filter (8.7.3) of the CTBs SAO changes, from the deblocked picture into sao_tmp:
// one wave per CTB; k_hevc_sao_copy then writes those CTBs back (after every CTB has
// read its deblocked neighbours).
__global__ __launch_bounds__(256) void k_hevc_sao_apply(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= f.mb_w * f.mb_h) return;
    const SaoParams p = A.sao[idx];
    if (!sao_any(p)) return;
    const int cx = idx % f.mb_w, cy = idx / f.mb_w;
    for (int i = lane(); i < kCoefPerCu; i += 64) {
        int c, x, y;
        ctb_sample(i, cx, cy, &c, &x, &y);
        const int stride = c ? f.stride_c : f.stride_y;
        plane_of(A.sao_tmp, c)[(size_t)y * stride + x] =
            (uint8_t)sao_apply_sample(p, c, sao_plane_of(f, c), plane_of(f.rec, c), stride, x, y);
    }
}
__global__ __launch_bounds__(256) void k_hevc_sao_copy(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= f.mb_w * f.mb_h) return;
    if (!sao_any(A.sao[idx])) return;
    const int cx = idx % f.mb_w, cy = idx / f.mb_w;
    Planes rec = f.rec;
    for (int i = lane(); i < kCoefPerCu; i += 64) {
        int c, x, y;
        ctb_sample(i, cx, cy, &c, &x, &y);
        const size_t o = (size_t)y * (c ? f.stride_c : f.stride_y) + x;
        plane_of(rec, c)[o] = plane_of(A.sao_tmp, c)[o];
    }
}

void launch_backend(const HevcArgs& a, hipStream_t s) {
    const int n = a.f.mb_w * a.f.mb_h;
    hipLaunchKernelGGL(k_hevc_inter, dim3((n + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_intra_prep, dim3((n + 3) / 4), dim3(256), 0, s, a);
    if (a.f.rows_per_slice <= 4)
        hipLaunchKernelGGL(k_hevc_intra<4>, dim3(a.f.num_slices), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_hevc_intra<15>, dim3(a.f.num_slices), dim3(64 * 15), 0, s, a);
    // in-loop deblocking, then the SAO decisions on the deblocked picture (CTB syntax)
    const int cw = a.f.mb_w, ch = a.f.mb_h;
    const int nv = ch * 4 * (2 * cw - 1) + 2 * ch * 8 * (cw - 1), nh = (2 * ch - 1) * cw * 4 + 2 * (ch - 1) * cw * 8;
    if (nv > 0) hipLaunchKernelGGL(k_hevc_dbk_v, dim3((nv + 255) / 256), dim3(256), 0, s, a);
    if (nh > 0) hipLaunchKernelGGL(k_hevc_dbk_h, dim3((nh + 255) / 256), dim3(256), 0, s, a);
    const int nq = (n + 3) / 4;
    hipLaunchKernelGGL(k_hevc_sao_stats, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sao_md, dim3((n * kSaoMd + 255) / 256), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sao_row, dim3(ch), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_hevc_bins, dim3((n + 255) / 256), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_sort, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sync, dim3(a.f.num_slices), dim3(192), 0, s, a);
    hipLaunchKernelGGL(k_pc_model, dim3(a.f.mb_h, (CTX_COUNT + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_rmap, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_compose, dim3(a.f.mb_h), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_pc_code, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_merge, dim3(a.f.mb_h), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_hevc_hdr, dim3(a.f.num_slices), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_hevc_ep_copy, dim3(a.f.mb_h), dim3(64), 0, s, a);
    // the SAO output becomes the reconstruction (k_commit copies it into the reference)
    hipLaunchKernelGGL(k_hevc_sao_apply, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sao_copy, dim3(nq), dim3(256), 0, s, a);
}

}  // namespace gpu
}  // namespace hevc
}  // namespace sk
