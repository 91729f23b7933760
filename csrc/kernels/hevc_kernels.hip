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
__device__ __forceinline__ int nbm_of(bool left, bool top, bool tr) {
    return (left ? AV_L : 0) | (top ? AV_T : 0) | (left && top ? AV_TL : 0) | (tr ? AV_TR : 0);
}
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// DPP lane exchanges (VALU, no LDS round trip; the xor shuffles compile to ds_bpermute):
// quad_perm [1,0,3,2] / [2,3,0,1] are the xor-1 / xor-2 partners; once every lane of a quad
// (eight lanes) holds the same value, row_half_mirror (i <-> 7 - i) / row_mirror (i <-> 15 - i)
// reach a lane of the other quad (eight) - the same sum as the xor-4 / xor-8 partner.
__device__ __forceinline__ int dpp_x1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false); }
__device__ __forceinline__ int dpp_x2(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false); }
__device__ __forceinline__ int dpp_hm(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false); }
__device__ __forceinline__ int dpp_m(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false); }
__device__ __forceinline__ int qsum(int v) {   // over the lane's quad (4 lanes)
    v += dpp_x1(v);
    return v + dpp_x2(v);
}
__device__ __forceinline__ int rsum16(int v) {   // over the lane's row (16 lanes)
    v = qsum(v);
    v += dpp_hm(v);
    return v + dpp_m(v);
}
__device__ __forceinline__ int ror16(int v) {   // OR over the lane's row
    v |= dpp_x1(v);
    v |= dpp_x2(v);
    v |= dpp_hm(v);
    return v | dpp_m(v);
}
// 4x4 blocks in 16-lane rows (lane 4y + x): the block's values at (y, k), k = 0..3, by quad
// broadcasts, and at ((y - d) & 3, x), d = 0..3, by rotating the row 4 lanes at a time
// (row_ror: lane i reads lane i - n of its row)
template <int C> __device__ __forceinline__ int dppc(int v) { return __builtin_amdgcn_update_dpp(0, v, C, 0xF, 0xF, false); }
__device__ __forceinline__ void blk_row(int v, int (&o)[4]) {
    o[0] = dppc<0x00>(v);
    o[1] = dppc<0x55>(v);
    o[2] = dppc<0xAA>(v);
    o[3] = dppc<0xFF>(v);
}
__device__ __forceinline__ void blk_col(int v, int (&o)[4]) {
    o[0] = v;
    o[1] = dppc<0x124>(v);
    o[2] = dppc<0x128>(v);
    o[3] = dppc<0x12C>(v);
}
__device__ __forceinline__ int wsum(int v) {
    v = rsum16(v);
    v += __shfl_xor(v, 16);
    return v + __shfl_xor(v, 32);
}

// K10 per-frame cap: the coding kernels run a second time, gated, after k_rc_guard_sizes
// (f.gate = the re-code flag); they return at once unless the frame overflowed.
__device__ __forceinline__ bool second_pass_skipped(const FrameArgs& f) { return f.gate && *f.gate == 0; }

// The picture's slice layout on the CTB grid (hevc_core.h SliceMap), its unit grid, and
// the substream of a slot (CTB row cy, segment k).
__device__ __forceinline__ SliceMap smap(const HevcArgs& A) {
    return SliceMap{A.f.tasks, A.cw, A.rps, A.seg_k};
}
__device__ __forceinline__ UnitGrid ugrid(const HevcArgs& A) { return UnitGrid{A.f.mb_w, A.f.mb_h}; }
__device__ __forceinline__ size_t sub_base(const HevcArgs& A, const SliceMap& m, int cy, int k) {
    return (size_t)cy * A.sub_stride + (size_t)m.x0(cy, k) * 4 * kSubstreamCtbBytes + 64 * (size_t)k;
}
// The slice task of CTB row r.
__device__ __forceinline__ const SliceTask& ctb_task(const HevcArgs& A, int r) { return A.f.tasks[r / A.rps]; }

// Per-wave LDS working set of one CU. Sample rasters (src, pred, rec*) hold the CU's
// 384 samples: Y 16x16 (pitch 16) | Cb 8x8 | Cr 8x8 (pitch 8).
struct CuLds {
    uint8_t src[kCoefPerCu];
    uint8_t pred[kCoefPerCu];
    uint8_t recA[kCoefPerCu];    // the 16x16 TU (+ 8x8 chroma TUs)
    uint8_t recS[kCoefPerCu];    // the split tree (inter: 8x8 luma TUs + 4x4 chroma; intra: its committed reconstruction)
    uint8_t rec4[kCoefPerCu];    // 4x4 luma TUs | trials with transform skip
    uint8_t rec4t[kCoefPerCu];   // 4x4 luma TUs with transform skip | intra: the node's 8x8 trial
    int32_t a[256], b[256];      // batch intermediates (compact, TU-major)
    int16_t levA[kCoefPerCu], lev8[256], lev4[256], lev4t[256], levc[128], levct[128];
    int acc[4][32];              // per-TU sums of a batch (twin: + 16): SSE of the prediction, of the reconstruction, rate, non-zero
    long long tj[6][16];         // per-TU RD cost: 0 Y16 Cb8 Cr8, 1 Y8, 2 Y4, 3 Y4 transform skip, 4 C4, 5 C4 skip
    int tf[6][16];               // per-TU cbf, same slots
    uint8_t ref[2][68];          // intra: the TU's reference samples (raw, [1 2 1]-filtered)
    uint8_t ref4[16][17];        // intra mode decision: the sixteen 4x4 blocks' references
    uint8_t nbt[3][33];          // intra: the row above the CU per component (x = -1 .. 2N - 1)
    uint8_t nbl[3][32];          // intra: the column left of the CU (y = 0 .. 2N - 1, below-left included)
    int mlx[kMaxMergeCand], mly[kMaxMergeCand], px[2], py[2];   // inter: merge / AMVP candidates
};

// LDS copy of the 16-point DCT matrix (the 8 / 4-point ones are its rows 2k / 4k) and, at
// 256 + 4k + m, the 4x4 DST. (Read at lane-dependent positions: LDS, not __constant__.)
constexpr int kTabT = 256 + 16;
__device__ __forceinline__ void load_t16(int8_t* t) {
    for (int i = threadIdx.x; i < kTabT; i += blockDim.x)
        t[i] = i < 256 ? HEVC_T16[i >> 4][i & 15] : HEVC_DST4[(i - 256) >> 2][i & 3];
}
__device__ __forceinline__ int tx_m(const int8_t* T, int log2n, bool dst, int k, int x) {
    return dst ? (int)T[256 + 4 * k + x] : (int)T[(k << (4 - log2n)) * 16 + x];
}

// TU t of a batch: CU-raster index of its top-left sample (the pitch follows: 16 in the
// luma part, 8 in the chroma part). kind 0: luma TUs of size n in z order; 1: chroma
// TUs, the Cb ones then the Cr ones; 2: the single TU at sb; 3: the Cb TU at sb and the
// Cr TU at the same place (sb + 64).
__device__ __forceinline__ int tu_base(int kind, int log2n, int t, int sb) {
    if (kind == 2) return sb;
    if (kind == 3) return sb + 64 * t;
    const int n = 1 << log2n;
    if (kind == 0) {
        const int bx = (t & 1) | ((t >> 1) & 2), by = ((t >> 1) & 1) | ((t >> 2) & 2);
        return by * n * 16 + bx * n;
    }
    const int half = (8 >> log2n) * (8 >> log2n), c = t / half, q = t % half;
    return kCoefCb + 64 * c + (q >> 1) * n * 8 + (q & 1) * n;
}

// A batch of ntu same-size TUs coded in parallel, each exactly as hevc_cpu.cpp code_tu_1
// (forward transform / DST / transform skip, quantisation, reconstruction, RD zeroing):
// levels (compact, TU-major, raster inside the TU) into lev, the reconstruction into the
// CU raster rec, per-TU RD cost and cbf into tj / tf. Items = samples, lane-strided.
// With a twin (4x4 TUs, 2 * ntu * 16 <= 256): every TU also coded with transform skip
// into levt / rect / tjt / tft in the same passes.
__device__ void tu_batch(CuLds& L, const int8_t* T, int kind, int sb, int log2n, int ntu, bool dst, bool ts, int qp,
                         bool intra, int lam, int16_t* lev, uint8_t* rec, long long* tj, int* tf, int16_t* levt = nullptr,
                         uint8_t* rect = nullptr, long long* tjt = nullptr, int* tft = nullptr) {
    const int l = lane(), n = 1 << log2n, nn = n * n, cnt = ntu * nn;
    const bool twin = levt != nullptr;
    const int all = twin ? 2 * cnt : cnt;
    const int sh1 = log2n - 1, sh2 = log2n + 6;
    if (l < 32) L.acc[0][l] = L.acc[1][l] = L.acc[2][l] = L.acc[3][l] = 0;
    wsync();
    // forward, rows: b[t][y][u] = sum_k M[u][k] res[t][y][k] (transform skip: res << 5)
    for (int i = l; i < all; i += 64) {
        const int var = i >= cnt, ii = i - var * cnt;
        const int t = ii >> (2 * log2n), y = (ii >> log2n) & (n - 1), u = ii & (n - 1);
        const int base = tu_base(kind, log2n, t, sb), o = base + y * (base < 256 ? 16 : 8);
        const int e = (int)L.src[o + u] - (int)L.pred[o + u];
        atomicAdd(&L.acc[0][t + 16 * var], e * e);
        int v = e * 32;
        if (!(ts || var)) {
            int s = 0;
            for (int k = 0; k < n; k++) s += tx_m(T, log2n, dst, u, k) * ((int)L.src[o + k] - (int)L.pred[o + k]);
            v = (s + (1 << (sh1 - 1))) >> sh1;
        }
        L.b[i] = v;
    }
    wsync();
    // forward, columns + quantisation + dequantisation
    for (int i = l; i < all; i += 64) {
        const int var = i >= cnt, ii = i - var * cnt;
        const int t = ii >> (2 * log2n), v = (ii >> log2n) & (n - 1), u = ii & (n - 1);
        int c = L.b[i];
        if (!(ts || var)) {
            int s = 0;
            const int* bt = L.b + t * nn + u;
            for (int k = 0; k < n; k++) s += tx_m(T, log2n, dst, v, k) * bt[k * n];
            c = (s + (1 << (sh2 - 1))) >> sh2;
        }
        const int lv = quant_level(c, qp, log2n, intra);
        (var ? levt : lev)[ii] = (int16_t)lv;
        L.a[i] = dequant_level(lv, qp, log2n);
        if (lv) {
            atomicAdd(&L.acc[2][t + 16 * var], level_rate_half(lv));
            atomicOr(&L.acc[3][t + 16 * var], 1);
        }
    }
    wsync();
    // inverse, columns: b[t][y][x] = clip16((sum_j M[j][y] d[t][j][x] + 64) >> 7)
    for (int i = l; i < all; i += 64) {
        const int var = i >= cnt, ii = i - var * cnt;
        const int t = ii >> (2 * log2n), y = (ii >> log2n) & (n - 1), x = ii & (n - 1);
        int g = L.a[i];
        if (!(ts || var)) {
            int s = 0;
            const int* at = L.a + t * nn + x;
            for (int j = 0; j < n; j++) s += tx_m(T, log2n, dst, j, y) * at[j * n];
            g = sk_clip((s + 64) >> 7, -32768, 32767);
        }
        L.b[i] = g;
    }
    wsync();
    // inverse, rows + reconstruction
    for (int i = l; i < all; i += 64) {
        const int var = i >= cnt, ii = i - var * cnt;
        const int t = ii >> (2 * log2n), y = (ii >> log2n) & (n - 1), x = ii & (n - 1);
        const int base = tu_base(kind, log2n, t, sb), o = base + y * (base < 256 ? 16 : 8) + x;
        int r;
        if (ts || var) {
            r = (L.b[i] * 128 + 2048) >> 12;
        } else {
            int s = 0;
            const int* gt = L.b + t * nn + y * n;
            for (int j = 0; j < n; j++) s += tx_m(T, log2n, dst, j, x) * gt[j];
            r = (s + 2048) >> 12;
        }
        const int rv = sk_clip255((int)L.pred[o] + r);
        (var ? rect : rec)[o] = (uint8_t)rv;
        const int e = (int)L.src[o] - rv;
        atomicAdd(&L.acc[1][t + 16 * var], e * e);
    }
    wsync();
    if (l < (twin ? 2 : 1) * ntu) {   // RD zeroing (code_tu_1's rule)
        const int var = l >= ntu, t = l - var * ntu, k = t + 16 * var;
        const long long s0 = L.acc[0][k], s1 = L.acc[1][k];
        const int rate = kTuRateHalf + L.acc[2][k];
        int nz = L.acc[3][k];
        if (nz && 512 * s0 <= 512 * s1 + (long long)lam * rate) nz = 0;
        (var ? tft : tf)[t] = nz;
        (var ? tjt : tj)[t] = nz ? 512 * s1 + (long long)lam * rate : 512 * s0;
    }
    wsync();
    for (int i = l; i < all; i += 64) {   // zeroed TUs: no levels, reconstruction = prediction
        const int var = i >= cnt, ii = i - var * cnt;
        const int t = ii >> (2 * log2n);
        if ((var ? tft : tf)[t]) continue;
        const int base = tu_base(kind, log2n, t, sb);
        const int o = base + ((ii >> log2n) & (n - 1)) * (base < 256 ? 16 : 8) + (ii & (n - 1));
        (var ? levt : lev)[ii] = 0;
        (var ? rect : rec)[o] = L.pred[o];
    }
    wsync();
}

// 4x4 TUs of a batch and of its transform-skip twin: each TU keeps the skip variant when
// it codes and costs less (code_tu's rule). Returns the per-TU skip mask.
__device__ int merge_ts(CuLds& L, int kind, int sb, int ntu, int16_t* lev, uint8_t* rec, long long* tj, int* tf,
                        const int16_t* levt, const uint8_t* rect, const long long* tjt, const int* tft) {
    const int l = lane();
    int mask = 0;
    for (int t = 0; t < ntu; t++)
        if (tft[t] && tjt[t] < tj[t]) mask |= 1 << t;
    for (int i = l; i < ntu * 16; i += 64) {
        const int t = i >> 4;
        if (!((mask >> t) & 1)) continue;
        lev[i] = levt[i];
        const int base = tu_base(kind, 2, t, sb), o = base + ((i >> 2) & 3) * (base < 256 ? 16 : 8) + (i & 3);
        rec[o] = rect[o];
    }
    wsync();
    if (l < ntu && ((mask >> l) & 1)) {
        tj[l] = tjt[l];
        tf[l] = tft[l];
    }
    wsync();
    return mask;
}

// Copies the n x n block at CU-raster index o (pitch from o) from one raster to another.
__device__ __forceinline__ void blk_copy(uint8_t* dst, const uint8_t* src, int o, int n) {
    const int pitch = o < 256 ? 16 : 8;
    for (int i = lane(); i < n * n; i += 64) {
        const int k = o + (i / n) * pitch + (i % n);
        dst[k] = src[k];
    }
}

// Source samples of CU (cx, cy) into L.src; a CU raster to the rec planes.
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
__device__ __forceinline__ void store_rec(const uint8_t* rec, const FrameArgs& f, int cx, int cy) {
    const int l = lane();
    for (int i = l; i < kCoefPerCu; i += 64) {
        if (i < 256) f.rec.y[(size_t)(cy * 16 + (i >> 4)) * f.stride_y + cx * 16 + (i & 15)] = rec[i];
        else {
            const int j = i - 256, c = j >> 6, r = (j >> 3) & 7, x = j & 7;
            (c ? f.rec.v : f.rec.u)[(size_t)(cy * 8 + r) * f.stride_c + cx * 8 + x] = rec[i];
        }
    }
}

// Residual of an inter CU (hevc_cpu.cpp code_inter_residual; prediction in L.pred): all
// trees coded in parallel batches, then the RD choice. Levels to gcoef, the TU fields into
// cu; returns the raster holding the chosen reconstruction.
__device__ const uint8_t* inter_residual(CuLds& L, const int8_t* T, int qp, int16_t* gcoef, CuInfo& cu,
                                         int lam_boost, long long* Jout) {
    const int l = lane(), qpc = chroma_qp(qp), lam = rd_lambda_q8(qp + lam_boost);
    {   // Every coded TU costs at least lam * (kTuRateHalf + 5) (one level): when the CU's whole
        // prediction error is below that, every TU of every tree zeroes and the 16x16 tree wins
        // (the split one pays its flags too) - the CPU's choice, without coding the trees.
        int e2 = 0;
        for (int i = l; i < kCoefPerCu; i += 64) {
            const int e = (int)L.src[i] - (int)L.pred[i];
            e2 += e * e;
        }
        const long long sse = wsum(e2);
        if (512 * sse < (long long)lam * (kTuRateHalf + 5)) {
            *Jout = 512 * sse;
            for (int i = l; i < kCoefPerCu; i += 64) gcoef[i] = 0;
            cu.cbf = 0;
            cu.tu = cu.tuc = 0;
            cu.ycbf = 0;
            cu.tsy = 0;
            cu.tsc = 0;
            return L.pred;
        }
    }
    tu_batch(L, T, 0, 0, 4, 1, false, false, qp, false, lam, L.levA, L.recA, L.tj[0], L.tf[0]);
    tu_batch(L, T, 1, 0, 3, 2, false, false, qpc, false, lam, L.levA + kCoefCb, L.recA, L.tj[0] + 1, L.tf[0] + 1);
    tu_batch(L, T, 0, 0, 3, 4, false, false, qp, false, lam, L.lev8, L.recS, L.tj[1], L.tf[1]);
    tu_batch(L, T, 0, 0, 2, 16, false, false, qp, false, lam, L.lev4, L.rec4, L.tj[2], L.tf[2]);
    tu_batch(L, T, 0, 0, 2, 16, false, true, qp, false, lam, L.lev4t, L.rec4t, L.tj[3], L.tf[3]);
    const int tsy = merge_ts(L, 0, 0, 16, L.lev4, L.rec4, L.tj[2], L.tf[2], L.lev4t, L.rec4t, L.tj[3], L.tf[3]);
    tu_batch(L, T, 1, 0, 2, 8, false, false, qpc, false, lam, L.levc, L.recS, L.tj[4], L.tf[4]);
    tu_batch(L, T, 1, 0, 2, 8, false, true, qpc, false, lam, L.levct, L.rec4, L.tj[5], L.tf[5]);
    const int tsc = merge_ts(L, 1, 0, 8, L.levc, L.recS, L.tj[4], L.tf[4], L.levct, L.rec4, L.tj[5], L.tf[5]);
    // the decision (every lane, from LDS)
    const long long ja = L.tj[0][0] + L.tj[0][1] + L.tj[0][2];
    const int cbfa = L.tf[0][0] | (L.tf[0][1] << 1) | (L.tf[0][2] << 2);
    long long js = (long long)lam * kSplitRateHalf;
    int tuc = 0, split8 = 0, c8 = 0, c4 = 0, ly = 0;
    for (int t = 0; t < 8; t++) {
        js += L.tj[4][t];
        tuc |= L.tf[4][t] << t;
    }
    for (int q = 0; q < 4; q++) {
        const long long j8 = L.tj[1][q];
        long long j4 = (long long)lam * kSplit8RateHalf;
        for (int j = 0; j < 4; j++) {
            j4 += L.tj[2][4 * q + j];
            c4 |= L.tf[2][4 * q + j] << (4 * q + j);
        }
        c8 |= L.tf[1][q] << q;
        if (j4 < j8) split8 |= 1 << q;
        js += j4 < j8 ? j4 : j8;
        ly |= (j4 < j8) ? (c4 >> (4 * q)) & 15 : (c8 >> q) & 1;
    }
    if (js < ja && (ly | tuc)) {
        *Jout = js;
        for (int i = l; i < 256; i += 64) {
            const int q = i >> 6;
            gcoef[i] = ((split8 >> q) & 1) ? L.lev4[i] : L.lev8[i];
            if ((split8 >> q) & 1) {   // node reconstruction from the 4x4 trees
                const int o = (8 * (q >> 1) + ((i >> 3) & 7)) * 16 + 8 * (q & 1) + (i & 7);
                L.recS[o] = L.rec4[o];
            }
        }
        for (int i = l; i < 128; i += 64) gcoef[kCoefCb + i] = L.levc[i];
        cu.tu = (uint8_t)(16 | split8);
        cu.tuc = (uint8_t)tuc;
        uint16_t m = 0;
        for (int q = 0; q < 4; q++)
            m |= (uint16_t)((((split8 >> q) & 1) ? (c4 >> (4 * q)) & 15 : (((c8 >> q) & 1) ? 15 : 0)) << (4 * q));
        uint16_t u4 = 0;
        for (int q = 0; q < 4; q++)
            if ((split8 >> q) & 1) u4 |= (uint16_t)(15 << (4 * q));
        cu.ycbf = m;
        cu.cbf = (uint8_t)((m ? 1 : 0) | ((tuc & 15) ? 2 : 0) | ((tuc >> 4) ? 4 : 0));
        cu.tsy = (uint16_t)(tsy & m & u4);
        cu.tsc = (uint8_t)(tsc & tuc);
        wsync();
        return L.recS;
    }
    *Jout = ja;
    for (int i = l; i < kCoefPerCu; i += 64) gcoef[i] = L.levA[i];
    cu.cbf = (uint8_t)cbfa;
    cu.tu = cu.tuc = 0;
    cu.ycbf = (cbfa & 1) ? 0xffff : 0;
    cu.tsy = 0;
    cu.tsc = 0;
    wsync();
    return L.recA;
}

// ---------------------------------------------------------------------------
// The 32x32 TU trial of a CU32 (hevc_cpu.cpp cu32_decide: code_tu_1 of the 32x32 luma TU
// and the two 16x16 chroma TUs) on all 256 lanes of the CTB's workgroup, after the units'
// CU16 coding: residual from the units' src / pred rasters, forward DCT (rows, columns),
// quantisation, inverse, reconstruction and the RD zeroing, per TU. Storage overlays the
// units' dead working sets: A and B (1536 ints each) and the levels (1536 int16) in 256-int
// chunks of Lw[k].a.. (4 KB per unit), the reconstruction in the units' recA rasters.
struct T32Acc {
    int sse0[3], sse1[3], rate[3], nz[3];
};
static_assert(offsetof(CuLds, levct) + sizeof(int16_t) * 128 >= offsetof(CuLds, a) + 4096, "CuLds: 4 KB from a");
__device__ __forceinline__ int* t32_chunk(CuLds* Lw, int c) { return reinterpret_cast<int*>(Lw[c >> 2].a) + (c & 3) * 256; }
__device__ __forceinline__ int& t32_A(CuLds* Lw, int i) { return t32_chunk(Lw, i >> 8)[i & 255]; }
__device__ __forceinline__ int& t32_B(CuLds* Lw, int i) { return t32_chunk(Lw, 6 + (i >> 8))[i & 255]; }
__device__ __forceinline__ int16_t& t32_L(CuLds* Lw, int i) {
    return reinterpret_cast<int16_t*>(t32_chunk(Lw, 12 + (i >> 9)))[i & 511];
}
// Logical element i (luma 32x32 raster | Cb 16x16 | Cr 16x16) -> unit z and its CU raster index.
__device__ __forceinline__ void t32_where(int i, int* z, int* o) {
    if (i < kT32Cb) {
        const int y = i >> 5, x = i & 31;
        *z = (x >> 4) | ((y >> 4) << 1);
        *o = (y & 15) * 16 + (x & 15);
    } else {
        const int k = i >= kT32Cr, j = i - (k ? kT32Cr : kT32Cb), y = j >> 4, x = j & 15;
        *z = (x >> 3) | ((y >> 3) << 1);
        *o = 256 + 64 * k + (y & 7) * 8 + (x & 7);
    }
}
__device__ __forceinline__ int t32_tu(int i) { return i < kT32Cb ? 0 : (i < kT32Cr ? 1 : 2); }
__device__ int t32_res(CuLds* Lw, int i) {
    int z, o;
    t32_where(i, &z, &o);
    return (int)Lw[z].src[o] - (int)Lw[z].pred[o];
}
// Element k of thread t: i = t + 256 k; k 0..3 luma, 4 Cb, 5 Cr (TU boundaries are multiples
// of 256, so the TU is uniform per k). Sums go per wave through shuffles, then one LDS atomic.
__device__ __forceinline__ void t32_add(int* dst, int v) {
    v = wsum(v);
    if (lane() == 0 && v) atomicAdd(dst, v);
}
// Row-contiguous access: the 32 (16) entries of a TU row never straddle a 256-int chunk.
__device__ __forceinline__ const int* t32_rowA(CuLds* Lw, int i) { return &t32_A(Lw, i); }
__device__ __forceinline__ const int* t32_rowB(CuLds* Lw, int i) { return &t32_B(Lw, i); }
// Column sum over a TU of the chunked array X (A or B): sum_y M[y] X[base + y n + u], the
// chunk pointer fetched once per 256 / n rows.
template <bool IsB>
__device__ __forceinline__ int t32_colsum(CuLds* Lw, const int8_t* Mrow, int mstride, int base, int log2n, int u) {
    const int n = 1 << log2n, rpc = 256 >> log2n;
    int sum = 0;
    for (int y0 = 0; y0 < n; y0 += rpc) {
        const int* p = IsB ? &t32_B(Lw, base + y0 * n + u) : &t32_A(Lw, base + y0 * n + u);
        for (int y = 0; y < rpc; y++) sum += (int)Mrow[(y0 + y) * mstride] * p[y * n];
    }
    return sum;
}
// Returns the cbf bits; *J the trial's RD cost (every thread).
__device__ int tu32_trial(CuLds* Lw, const int8_t* T32, int qp, int lam, T32Acc& acc, long long* J) {
    const int t = threadIdx.x, qpc = chroma_qp(qp);
    if (t < 3) acc.sse0[t] = acc.sse1[t] = acc.rate[t] = acc.nz[t] = 0;
    __syncthreads();
    // the residual into B (free until the dequantised levels), the zero-residual SSE
    {
        int s0[3] = {0, 0, 0};
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int i = t + 256 * k, e = t32_res(Lw, i);
            t32_B(Lw, i) = e;
            s0[k < 4 ? 0 : k - 3] += e * e;
        }
#pragma unroll
        for (int tu = 0; tu < 3; tu++) t32_add(&acc.sse0[tu], s0[tu]);
    }
    __syncthreads();
    // forward, rows: A[tu][y][u] = (sum_x M[u][x] res[y][x] + rnd) >> sh1
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const int i = t + 256 * k, tu = k < 4 ? 0 : k - 3, log2n = tu ? 4 : 5, n = 1 << log2n;
        const int base = tu == 0 ? 0 : (tu == 1 ? kT32Cb : kT32Cr), sh1 = log2n - 1;
        const int j = i - base, y = j >> log2n, u = j & (n - 1);
        const int* rp = t32_rowB(Lw, base + y * n);
        const int8_t* Mr = T32 + (tu ? 2 * u : u) * 32;
        int sum = 0;
        for (int x = 0; x < n; x++) sum += (int)Mr[x] * rp[x];
        t32_A(Lw, i) = (sum + (1 << (sh1 - 1))) >> sh1;
    }
    __syncthreads();
    // forward, columns + quantisation + dequantisation
    {
        int rate[3] = {0, 0, 0}, nz[3] = {0, 0, 0};
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int i = t + 256 * k, tu = k < 4 ? 0 : k - 3, log2n = tu ? 4 : 5, n = 1 << log2n;
            const int base = tu == 0 ? 0 : (tu == 1 ? kT32Cb : kT32Cr), sh2 = log2n + 6, q = tu ? qpc : qp;
            const int j = i - base, v = j >> log2n, u = j & (n - 1);
            // M[v][y] for y = 0..n-1: row v of the matrix (stride 1)
            const int sum = t32_colsum<false>(Lw, T32 + (tu ? 2 * v : v) * 32, 1, base, log2n, u);
            const int lv = quant_level((sum + (1 << (sh2 - 1))) >> sh2, q, log2n, false);
            t32_L(Lw, i) = (int16_t)lv;
            // B is read by other threads' row pass only before the barrier above: free now
            t32_B(Lw, i) = dequant_level(lv, q, log2n);
            if (lv) {
                rate[k < 4 ? 0 : k - 3] += level_rate_half(lv);
                nz[k < 4 ? 0 : k - 3] = 1;
            }
        }
#pragma unroll
        for (int tu = 0; tu < 3; tu++) {
            t32_add(&acc.rate[tu], rate[tu]);
            t32_add(&acc.nz[tu], nz[tu]);
        }
    }
    __syncthreads();
    // inverse, columns: A = clip16((sum_j M[j][y] B[j][x] + 64) >> 7)
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const int i = t + 256 * k, tu = k < 4 ? 0 : k - 3, log2n = tu ? 4 : 5, n = 1 << log2n;
        const int base = tu == 0 ? 0 : (tu == 1 ? kT32Cb : kT32Cr);
        const int j = i - base, y = j >> log2n, x = j & (n - 1);
        // M[j][y] for j = 0..n-1: column y of the matrix (stride 32, or 64 for the 16-point rows)
        const int sum = acc.nz[tu] ? t32_colsum<true>(Lw, T32 + y, tu ? 64 : 32, base, log2n, x) : 0;
        t32_A(Lw, i) = sk_clip((sum + 64) >> 7, -32768, 32767);
    }
    __syncthreads();
    // inverse, rows + reconstruction (into the units' recA)
    {
        int s1[3] = {0, 0, 0};
#pragma unroll
        for (int k = 0; k < 6; k++) {
            const int i = t + 256 * k, tu = k < 4 ? 0 : k - 3, log2n = tu ? 4 : 5, n = 1 << log2n;
            const int base = tu == 0 ? 0 : (tu == 1 ? kT32Cb : kT32Cr);
            const int j = i - base, y = j >> log2n, x = j & (n - 1);
            const int* rp = t32_rowA(Lw, base + y * n);
            const int ms = tu ? 64 : 32;
            int sum = 0;
            for (int kk = 0; kk < n; kk++) sum += (int)T32[kk * ms + x] * rp[kk];
            int z, o;
            t32_where(i, &z, &o);
            const int rv = sk_clip255((int)Lw[z].pred[o] + ((sum + 2048) >> 12));
            Lw[z].recA[o] = (uint8_t)rv;
            const int e = (int)Lw[z].src[o] - rv;
            s1[k < 4 ? 0 : k - 3] += e * e;
        }
#pragma unroll
        for (int tu = 0; tu < 3; tu++) t32_add(&acc.sse1[tu], s1[tu]);
    }
    __syncthreads();
    long long jt = 0;
    int cbf = 0, keep[3];
    for (int tu = 0; tu < 3; tu++) {   // RD zeroing (code_tu_1's rule), every thread alike
        const long long s0 = acc.sse0[tu], s1 = acc.sse1[tu];
        const int rate = kTuRateHalf + acc.rate[tu];
        int nz = acc.nz[tu] != 0;
        if (nz && 512 * s0 <= 512 * s1 + (long long)lam * rate) nz = 0;
        keep[tu] = nz;
        cbf |= nz << tu;
        jt += nz ? 512 * s1 + (long long)lam * rate : 512 * s0;
    }
#pragma unroll
    for (int k = 0; k < 6; k++) {   // zeroed TUs: no levels, reconstruction = prediction
        const int i = t + 256 * k;
        if (keep[k < 4 ? 0 : k - 3]) continue;
        int z, o;
        t32_where(i, &z, &o);
        t32_L(Lw, i) = 0;
        Lw[z].recA[o] = Lw[z].pred[o];
    }
    __syncthreads();
    *J = jt;
    return cbf;
}

// K6 inter (P slices) and skip-all slices: one workgroup per CTB, wave z = the CTB's unit
// z. Phase 1: every unit as a 16x16 CU (merge / AMVP candidates of its z-scan neighbours
// on the unit motion field, quarter-pel MC, the residual trees); phase 2 (the whole
// workgroup): the CTB as one 32x32 CU instead, with a 32x32 TU trial
// (hevc_cpu.cpp code_slice_inter + cu32_decide, the same decisions).
__global__ __launch_bounds__(256) void k_hevc_inter(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ CuLds Lw[4];
    __shared__ int8_t T[kTabT];
    __shared__ int8_t T32[1024];
    __shared__ long long jw[4];
    __shared__ CuInfo cw4[4], pus[2];
    __shared__ T32Acc acc;
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int c = blockIdx.x % A.cw, r = blockIdx.x / A.cw;
    const UnitGrid ug = ugrid(A);
    const SliceMap m = smap(A);
    const int ux = 2 * c + (w & 1), uy = 2 * r + (w >> 1);
    const bool inside = ug.inside(ux, uy);
    const int idx = uy * f.mb_w + ux;
    const SliceTask t = ctb_task(A, r);
    if (t.final_action == ACT_SKIPALL) {   // block-uniform: skipped CU32 / CU16s (code_slice_skip)
        if (inside && l == 0) {
            CuInfo z;
            memset(&z, 0, sizeof(z));
            z.mode = CU_SKIP;
            z.qp = (uint8_t)t.qp;
            for (int i = 0; i < 16; i++) z.ipm[i] = 1;
            if (ug.complete(c, r)) z.c32 = kC32;
            A.cus[idx] = z;
        }
        return;
    }
    if (t.final_action != ACT_P) return;   // block-uniform
    load_t16(T);
    for (int i = threadIdx.x; i < 1024; i += 256) T32[i] = HEVC_T32[i >> 5][i & 31];
    __syncthreads();
    const int W = f.mb_w;
    auto mvf = [&](int nx, int ny, int* x, int* y) {
        *x = h264::me_qx(f.me[ny * W + nx]);
        *y = h264::me_qy(f.me[ny * W + nx]);
    };
    CuLds& L = Lw[w];
    const int lam_boost = A.f.rc->lam_boost;
    if (inside) {   // ---- phase 1 (wave-uniform)
        const PuNb nb = pu_neighbours(ug, m, mvf, 16 * ux, 16 * uy, 16, 16 * ux, 16 * uy, 16, 16, 0);
        // candidate lists in LDS (dynamically indexed: private arrays would live in scratch);
        // every lane writes the same values
        pu_merge_list(nb, PART_2Nx2N, 0, L.mlx, L.mly);
        pu_amvp_list(nb, L.px, L.py);
        wsync();
        const int mvx = h264::me_qx(f.me[idx]), mvy = h264::me_qy(f.me[idx]);   // quarter-pel (k_subpel)
        const int pic_w = f.stride_y, pic_h = f.mb_h * 16;
        load_src(L, f, ux, uy);
        {   // luma MC (hevc_core.h luma_mc_sample, separable form): the 23x23 integer window
            // into LDS (L.a as bytes, row pitch 24), horizontal 8-tap pass into L.b (23 rows x
            // 16), vertical pass into pred (lane = row l >> 2, 4 columns). L.a / L.b are free
            // until the residual batches.
            const int fx = mvx & 3, fy = mvy & 3;
            const int x0 = ux * 16 + (mvx >> 2) - 3, y0 = uy * 16 + (mvy >> 2) - 3;
            uint8_t* win = reinterpret_cast<uint8_t*>(L.a);
            int* hb = reinterpret_cast<int*>(L.lev8);   // 23 x 16 ints: L.lev8 .. L.lev4t are free too
            for (int i = l; i < 23 * 23; i += 64) {
                const int rr = i / 23, cc = i - rr * 23;
                win[rr * 24 + cc] =
                    f.ref.y[(size_t)sk_clip(y0 + rr, 0, pic_h - 1) * f.stride_y + sk_clip(x0 + cc, 0, pic_w - 1)];
            }
            wsync();
            for (int i = l; i < 23 * 16; i += 64) {
                const uint8_t* wp = win + (i >> 4) * 24 + (i & 15);
                int sm = (int)wp[3] << 6;
                if (fx) {
                    sm = 0;
#pragma unroll
                    for (int k = 0; k < 8; k++) sm += HEVC_LUMA_FILTER[fx][k] * (int)wp[k];
                }
                hb[i] = sm;
            }
            wsync();
            const int y = l >> 2;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int x = 4 * (l & 3) + k;
                int v = hb[(y + 3) * 16 + x];
                if (fy) {
                    v = 0;
#pragma unroll
                    for (int j = 0; j < 8; j++) v += HEVC_LUMA_FILTER[fy][j] * hb[(y + j) * 16 + x];
                    v >>= 6;
                }
                L.pred[y * 16 + x] = (uint8_t)sk_clip255((v + 32) >> 6);
            }
            // chroma: lane -> component l >> 5, row (l >> 2) & 7, 2 columns
            const int cc = l >> 5, rr = (l >> 2) & 7;
            const uint8_t* plane = cc ? f.ref.v : f.ref.u;
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int x = 2 * (l & 3) + k;
                L.pred[kCoefCb + cc * 64 + rr * 8 + x] = (uint8_t)chroma_mc_sample(
                    plane, f.stride_c, f.stride_c, f.mb_h * 8, ux * 8 + x, uy * 8 + rr, mvx, mvy);
            }
        }
        wsync();
        CuInfo cu;
        memset(&cu, 0, sizeof(cu));
        long long J = 0;
        const uint8_t* rec = inter_residual(L, T, t.qp, A.coefs + (size_t)idx * kCoefPerCu, cu, lam_boost, &J);
        store_rec(rec, f, ux, uy);
        if (l == 0) {
            cu.qp = (uint8_t)t.qp;
            pu_choose(cu, mvx, mvy, L.mlx, L.mly, L.px, L.py);
            if (cu.mode == CU_MERGE && !cu.cbf) cu.mode = CU_SKIP;
            for (int i = 0; i < 16; i++) cu.ipm[i] = 1;
            A.cus[idx] = cu;
            cw4[w] = cu;
            jw[w] = J;
        }
    }
    __syncthreads();
    if (!ug.complete(c, r)) return;   // ---- phase 2 (block-uniform from here)
    int mx[4], my[4];
    for (int z = 0; z < 4; z++) {
        mx[z] = cw4[z].mvx;
        my[z] = cw4[z].mvy;
    }
    const int part = cu32_part(mx, my);
    if (part < 0) return;
    if (w == 0) {   // the PUs' merge / AMVP syntax (uniform values)
        for (int pi = 0; pi < (part == PART_2Nx2N ? 1 : 2); pi++) {
            int xp, yp, pw, ph;
            pu_rect(part, pi, 32 * c, 32 * r, 32, &xp, &yp, &pw, &ph);
            const PuNb nb = pu_neighbours(ug, m, mvf, 32 * c, 32 * r, 32, xp, yp, pw, ph, pi);
            pu_merge_list(nb, part, pi, L.mlx, L.mly);
            pu_amvp_list(nb, L.px, L.py);
            wsync();
            CuInfo p;
            memset(&p, 0, sizeof(p));
            const int z = pi == 0 ? 0 : 3;
            pu_choose(p, mx[z], my[z], L.mlx, L.mly, L.px, L.py);
            if (l == 0) pus[pi] = p;
            wsync();
        }
        if (part == PART_2Nx2N && l == 0) pus[1] = pus[0];
    }
    __syncthreads();
    const int lam = rd_lambda_q8(t.qp + lam_boost);
    long long jsum = 0;
    int hsplit = 0, cbf_units = 0;
    for (int z = 0; z < 4; z++) {
        jsum += jw[z];
        hsplit += cu16_hdr_half(cw4[z]);
        cbf_units |= cw4[z].cbf;
    }
    long long j32 = 0;
    int cbf32 = 0;
    bool tu32 = false;
    if (cbf_units) {   // the 32x32 TU is tried when some unit codes a residual (cu32_decide)
        cbf32 = tu32_trial(Lw, T32, t.qp, lam, acc, &j32);
        tu32 = j32 < jsum;
    }
    const int root = tu32 ? cbf32 : cbf_units;
    const bool skip = part == PART_2Nx2N && pus[0].mode == CU_MERGE && !root;
    const long long jc = (long long)lam * cu32_hdr_half(part, pus[0], pus[1], skip) + (tu32 ? j32 : jsum);
    const long long js = (long long)lam * hsplit + jsum;
    if (jc >= js) return;
    // the CU32 replaces the four CU16s: wave z rewrites unit z
    CuInfo cu = cw4[w];
    const CuInfo& p = pus[cu32_pu_of(part, w)];
    cu.mode = skip ? CU_SKIP : p.mode;
    cu.merge_idx = p.merge_idx;
    cu.mvp_idx = p.mvp_idx;
    cu.mvdx = p.mvdx;
    cu.mvdy = p.mvdy;
    cu.c32 = (uint8_t)(kC32 | (part << 1) | (tu32 ? kC32Tu : 0));
    if (tu32) {
        cu.cbf = (uint8_t)cbf32;
        cu.tu = cu.tuc = 0;
        cu.ycbf = (cbf32 & 1) ? 0xffff : 0;
        cu.tsy = 0;
        cu.tsc = 0;
        int16_t* g = A.coefs + (size_t)idx * kCoefPerCu;
        for (int i = l; i < kCoefPerCu; i += 64) g[i] = t32_L(Lw, w * kCoefPerCu + i);
        store_rec(L.recA, f, ux, uy);
    }
    if (l == 0) A.cus[idx] = cu;
}

// ---------------------------------------------------------------------------
// Intra reference samples (8.4.4.2.2) of the n x n TU of component c at (x0, y0) in
// CU-relative component coordinates (n <= 16), availability av (AV_* bits): samples
// inside the CU from the CU raster W (nullptr: everything from the plane P, whose CU
// origin is (px0, py0)), substitution in closed form by ballot. Lane i: entry i (entry
// 64 of a 16x16 TU: lane 0's second one).
__device__ void tu_refs(const uint8_t* W, const uint8_t* P, int stride, int px0, int py0, int c, int x0, int y0,
                        int n, int av, uint8_t* out, const CuLds* nb = nullptr) {
    const int l = lane(), len = 4 * n + 1, cn = c ? 8 : 16, wb = c == 0 ? 0 : (c == 1 ? kCoefCb : kCoefCr);
    auto fetch = [&](int i, bool& ok) {
        int x, y, bit;
        if (i < 2 * n) {
            const int yy = 2 * n - 1 - i;
            x = x0 - 1;
            y = y0 + yy;
            bit = yy < n ? AV_L : AV_BL;
        } else if (i == 2 * n) {
            x = x0 - 1;
            y = y0 - 1;
            bit = AV_TL;
        } else {
            const int xx = i - 2 * n - 1;
            x = x0 + xx;
            y = y0 - 1;
            bit = xx < n ? AV_T : AV_TR;
        }
        ok = (av & bit) != 0;
        if (!ok) return 0;
        if (W && x >= 0 && y >= 0 && x < cn && y < cn) return (int)W[wb + y * cn + x];
        if (nb) return y < 0 ? (int)nb->nbt[c][x + 1] : (int)nb->nbl[c][y];   // outside the CU: prefetched
        return (int)P[(size_t)(py0 + y) * stride + px0 + x];
    };
    bool ok = false;
    const int v = l < len ? fetch(l, ok) : 0;
    const uint64_t M = __ballot(ok);
    int src = l;
    if (!ok) {
        const uint64_t below = l ? (M & ((1ull << l) - 1)) : 0ull;
        src = below ? 63 - __builtin_clzll(below) : (M ? __builtin_ctzll(M) : l);
    }
    int r = __shfl(v, src);
    if (!M) r = 128;
    if (l < len) out[l] = (uint8_t)r;
    if (len > 64) {   // entry 64 (top-right end of a 16x16 TU)
        bool ok64 = false;
        const int v64 = fetch(64, ok64);
        const int r63 = __shfl(r, 63);
        if (l == 0) out[64] = (uint8_t)(ok64 ? v64 : r63);
    }
    wsync();
}
// [1 2 1] filtering of the references (8.4.4.2.3), n <= 16.
__device__ __forceinline__ void ref_filter(const uint8_t* r, int n, uint8_t* out) {
    const int len = 4 * n + 1;
    for (int i = lane(); i < len; i += 64)
        out[i] = (i == 0 || i == len - 1) ? r[i] : (uint8_t)((r[i - 1] + 2 * r[i] + r[i + 1] + 2) >> 2);
    wsync();
}
// Prediction of the n x n TU of component c at CU-raster index o into L.pred.
__device__ __forceinline__ void tu_pred(CuLds& L, const uint8_t* ref, int c, int log2n, int mode, int o) {
    const int n = 1 << log2n, pitch = o < 256 ? 16 : 8;
    for (int i = lane(); i < n * n; i += 64)
        L.pred[o + (i >> log2n) * pitch + (i & (n - 1))] =
            (uint8_t)intra_pred_sample(ref, n, log2n, mode, c, i & (n - 1), i >> log2n);
    wsync();
}
// References + prediction of one intra TU (component c, n x n at CU-relative (x0, y0)).
__device__ void intra_tu_pred(CuLds& L, const uint8_t* W, const Planes& P, const FrameArgs& f, int cx, int cy, int c,
                              int log2n, int x0, int y0, int av, int mode) {
    const int n = 1 << log2n, cn = c ? 8 : 16;
    const uint8_t* plane = c == 0 ? P.y : (c == 1 ? P.u : P.v);
    tu_refs(W, plane, c ? f.stride_c : f.stride_y, cx * cn, cy * cn, c, x0, y0, n, av, L.ref[0], &L);
    const uint8_t* r = L.ref[0];
    if (intra_filter_flag(mode, log2n, c)) {
        ref_filter(L.ref[0], n, L.ref[1]);
        r = L.ref[1];
    }
    const int o = (c == 0 ? 0 : (c == 1 ? kCoefCb : kCoefCr)) + y0 * cn + x0;
    tu_pred(L, r, c, log2n, mode, o);
}

// The unit's outside neighbours (row above incl. the corner and the top-right unit's
// bottom row, column left incl. the below-left unit's right column) of every component
// into L.nbt / L.nbl, once per unit: the TU chain then reads its references from LDS only.
// nbm: the neighbour units' availability (AV_* bits); unavailable entries are never read.
__device__ void load_nb(CuLds& L, const Planes& P, const FrameArgs& f, int cx, int cy, int nbm) {
    for (int i = lane(); i < 147; i += 64) {
        int c, x, y;
        if (i < 33) { c = 0; x = i - 1; y = -1; }
        else if (i < 67) { c = 1 + (i - 33) / 17; x = (i - 33) % 17 - 1; y = -1; }
        else if (i < 99) { c = 0; x = -1; y = i - 67; }
        else { c = 1 + (i - 99) / 16; x = -1; y = (i - 99) % 16; }
        const int cn = c ? 8 : 16;
        const bool ok = y < 0 ? (x < 0 ? (nbm & AV_TL) != 0 : (x < cn ? (nbm & AV_T) != 0 : (nbm & AV_TR) != 0))
                              : (y < cn ? (nbm & AV_L) != 0 : (nbm & AV_BL) != 0);
        if (!ok) continue;
        const uint8_t* pl = c == 0 ? P.y : (c == 1 ? P.u : P.v);
        const int stride = c ? f.stride_c : f.stride_y;
        const uint8_t v = pl[(size_t)(cy * cn + y) * stride + cx * cn + x];
        if (y < 0) L.nbt[c][x + 1] = v;
        else L.nbl[c][y] = v;
    }
    wsync();
}

// Open-loop intra decision per unit of I slices (all units in parallel; hevc_cpu.cpp
// intra_decide): lane = (4x4 block l >> 2, row l & 3); per mode the block / 8x8 / 16x16 SADs
// by shuffles, the best mode of each, then CU16 against four CU8s (PART_2Nx2N / NxN).
__global__ __launch_bounds__(256) void k_hevc_intra_prep(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ CuLds Lw[4];
    const FrameArgs& f = A.f;
    CuLds& L = Lw[threadIdx.x >> 6];
    const int n = f.mb_w * f.mb_h;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= n) return;   // wave-uniform; no block barriers below
    const int cx = idx % f.mb_w, cy = idx / f.mb_w;
    const SliceTask t = ctb_task(A, cy >> 1);
    if (t.final_action != ACT_I) return;
    const int nbm = unit_nbm(ugrid(A), smap(A), cx, cy);
    load_src(L, f, cx, cy);
    for (int u = 0; u < 16; u++) {
        const int bx = (u & 1) | ((u >> 1) & 2), by = ((u >> 1) & 1) | ((u >> 2) & 2);
        tu_refs(nullptr, f.src.y, f.stride_y, cx * 16, cy * 16, 0, 4 * bx, 4 * by, 4, tu_avail_at(bx, by, 1, nbm), L.ref4[u]);
    }
    const int l = lane(), u = l >> 2, row = l & 3;
    const int bx = (u & 1) | ((u >> 1) & 2), by = ((u >> 1) & 1) | ((u >> 2) & 2);
    int b4 = 1, c4 = 0x7fffffff, b8 = 1, c8 = 0x7fffffff, b16 = 1, c16 = 0x7fffffff;
    for (int k = 0; k < 35; k++) {   // HEVC_INTRA_ORDER, SAD + intra_mode_bias, first minimum wins
        const int m = HEVC_INTRA_ORDER[k];
        int sad = 0;
#pragma unroll
        for (int x = 0; x < 4; x++)
            sad += sk_abs((int)L.src[(4 * by + row) * 16 + 4 * bx + x] - intra_pred_sample(L.ref4[u], 4, 2, m, 0, x, row));
        sad = qsum(sad);              // the block
        int s8 = sad + dpp_hm(sad);
        s8 += dpp_m(s8);              // the 8x8 quadrant
        int s16 = s8 + __shfl_xor(s8, 16);
        s16 += __shfl_xor(s16, 32);   // the unit
        const int bias = intra_mode_bias(m, t.qp);
        if (sad + bias < c4) { c4 = sad + bias; b4 = m; }
        if (s8 + bias < c8) { c8 = s8 + bias; b8 = m; }
        if (s16 + bias < c16) { c16 = s16 + bias; b16 = m; }
    }
    const int lam = intra_lam_sad(t.qp);
    int cn = c4 + dpp_hm(c4);   // c4 is uniform over the block's quad
    cn += dpp_m(cn);
    cn += kPenNxN * lam;
    const int nxn_q = cn < c8 ? 1 : 0;
    int cq = nxn_q ? cn : c8;
    cq += __shfl_xor(cq, 16);
    cq += __shfl_xor(cq, 32);
    const int csplit = kPenSplit * lam + cq;
    const bool split = csplit < c16;
    CuInfo cu;
    memset(&cu, 0, sizeof(cu));
    cu.mode = CU_INTRA;
    int nxn = 0;
    for (int q = 0; q < 4; q++) nxn |= __shfl(nxn_q, 16 * q) << q;
    for (int v = 0; v < 16; v++) {
        const int m4 = __shfl(b4, 4 * v), m8 = __shfl(b8, 4 * v);
        cu.ipm[v] = (uint8_t)(split ? (((nxn >> (v >> 2)) & 1) ? m4 : m8) : b16);
    }
    cu.cu8 = (uint8_t)(split ? 16 | nxn : 0);
    cu.intra_mode = cu.ipm[0];
    if (l == 0) A.cus[idx] = cu;
}

__device__ __forceinline__ long long shfl64(long long v, int src) {
    const int lo = __shfl((int)(v & 0xffffffffll), src), hi = __shfl((int)(v >> 32), src);
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// One intra 4x4 luma TU of a split node - the hot step of the TU chain (hevc_cpu.cpp
// code_slice_intra's tu(0, 2, ...): code_tu with the DST and the transform-skip trial) -
// in registers: lanes 0..15 take sample s (x = s & 3, y = s >> 2) with the DST, lanes
// 16..31 the same sample with transform skip (lanes 32..63 repeat them); transforms and
// RD sums by cross-lane shuffles instead of LDS phases. The references go through LDS
// once (the prediction reads them at sample-dependent positions). The reconstruction
// lands in W, the levels in lev; returns the cbf, *J the TU's RD cost, *ts the choice.
__device__ int intra4x4_step(CuLds& L, const int8_t* T, uint8_t* W, int bx, int by, int av, int mode, int qp, int lam,
                             int16_t* lev, long long* J, int* ts) {
    const int l = lane(), s = l & 15, var = (l >> 4) & 1;
    const int x = s & 3, y = s >> 2, o = (4 * by + y) * 16 + 4 * bx + x;
    tu_refs(W, nullptr, 0, 0, 0, 0, 4 * bx, 4 * by, 4, av, L.ref[0], &L);
    const uint8_t* ref = L.ref[0];
    const int p = intra_pred_at([&](int i) { return (int)ref[i]; }, 4, 2, mode, 0, x, y);
    const int e = (int)L.src[o] - p;
    auto M = [&](int k, int m) { return (int)T[256 + 4 * k + m]; };   // the DST (load_t16)
    // forward DST: rows t[y][u] = (sum_k M[u][k] e[y][k] + 1) >> 1, columns (+ 128) >> 8
    int t = 0, c = 0, nb[4];
    blk_row(e, nb);
#pragma unroll
    for (int k = 0; k < 4; k++) t += M(x, k) * nb[k];
    t = (t + 1) >> 1;
    blk_col(t, nb);
#pragma unroll
    for (int k = 0; k < 4; k++) c += M(y, (y - k) & 3) * nb[k];
    c = (c + 128) >> 8;
    if (var) c = e * 32;   // transform skip: the residual << 5
    const int lv = quant_level(c, qp, 2, true);
    const int d = dequant_level(lv, qp, 2);
    // inverse: columns g = clip16((sum_j M[j][y] d[j][x] + 64) >> 7), rows (sum_j M[j][x] g[y][j] + 2048) >> 12
    int g = 0, r = 0;
    blk_col(d, nb);
#pragma unroll
    for (int j = 0; j < 4; j++) g += M((y - j) & 3, y) * nb[j];
    g = sk_clip((g + 64) >> 7, -32768, 32767);
    blk_row(g, nb);
#pragma unroll
    for (int j = 0; j < 4; j++) r += M(j, x) * nb[j];
    r = (r + 2048) >> 12;
    if (var) r = (d * 128 + 2048) >> 12;
    const int rec = sk_clip255(p + r), e1 = (int)L.src[o] - rec;
    int s0 = e * e, s1 = e1 * e1, rt = level_rate_half(lv), nz = lv != 0;
    s0 = rsum16(s0);   // over the 16 lanes of the variant (rows of 16)
    s1 = rsum16(s1);
    rt = rsum16(rt);
    nz = ror16(nz);
    const int rate = kTuRateHalf + rt;
    int f = nz;
    if (f && 512ll * s0 <= 512ll * s1 + (long long)lam * rate) f = 0;   // RD zeroing (code_tu_1)
    const long long j = f ? 512ll * s1 + (long long)lam * rate : 512ll * s0;
    const int f0 = __shfl(f, 0), f1 = __shfl(f, 16);
    const long long j0 = shfl64(j, 0), j1 = shfl64(j, 16);
    const int use = (f1 && j1 < j0) ? 1 : 0;   // code_tu: transform skip when it codes and costs less
    const int fsel = use ? f1 : f0;
    const int lv_t = __shfl(lv, 16 + s), rec_t = __shfl(rec, 16 + s);
    if (l < 16) {
        lev[s] = (int16_t)(fsel ? (use ? lv_t : lv) : 0);
        W[o] = (uint8_t)(fsel ? (use ? rec_t : rec) : p);
    }
    *J = use ? j1 : j0;
    *ts = use;
    wsync();   // W for the next TU's references
    return fsel;
}

// A split node's Cb and Cr 4x4 TUs (code_tu with the DCT and the transform-skip trial), as
// intra4x4_step: lanes 0..31 Cb, 32..63 Cr, each half DCT (first 16) | transform skip.
// (ox, oy): the TUs in chroma coordinates of the CU. Levels to lev_c[0] (Cb) / lev_c[64]
// (Cr), reconstruction into W; per component cbf, RD cost and skip choice.
__device__ void intra_c4_pair(CuLds& L, const int8_t* T, uint8_t* W, int ox, int oy, int av, int mode, int qpc, int lam,
                              int16_t* lev_c, int* fc, long long* Jc, int* tsc) {
    const int l = lane(), s = l & 15, var = (l >> 4) & 1, comp = l >> 5;
    const int x = s & 3, y = s >> 2, o = (comp ? kCoefCr : kCoefCb) + (oy + y) * 8 + ox + x;
    tu_refs(W, nullptr, 0, 0, 0, 1, ox, oy, 4, av, L.ref[0], &L);
    tu_refs(W, nullptr, 0, 0, 0, 2, ox, oy, 4, av, L.ref[1], &L);
    const uint8_t* ref = L.ref[comp];
    const int p = intra_pred_at([&](int i) { return (int)ref[i]; }, 4, 2, mode, 1 + comp, x, y);
    const int e = (int)L.src[o] - p;
    auto M = [&](int k, int m) { return (int)T[(k << 2) * 16 + m]; };   // 4-point DCT rows of T16
    int t = 0, c = 0, nb[4];
    blk_row(e, nb);
#pragma unroll
    for (int k = 0; k < 4; k++) t += M(x, k) * nb[k];
    t = (t + 1) >> 1;
    blk_col(t, nb);
#pragma unroll
    for (int k = 0; k < 4; k++) c += M(y, (y - k) & 3) * nb[k];
    c = (c + 128) >> 8;
    if (var) c = e * 32;
    const int lv = quant_level(c, qpc, 2, true);
    const int d = dequant_level(lv, qpc, 2);
    int g = 0, r = 0;
    blk_col(d, nb);
#pragma unroll
    for (int j = 0; j < 4; j++) g += M((y - j) & 3, y) * nb[j];
    g = sk_clip((g + 64) >> 7, -32768, 32767);
    blk_row(g, nb);
#pragma unroll
    for (int j = 0; j < 4; j++) r += M(j, x) * nb[j];
    r = (r + 2048) >> 12;
    if (var) r = (d * 128 + 2048) >> 12;
    const int rec = sk_clip255(p + r), e1 = (int)L.src[o] - rec;
    int s0 = e * e, s1 = e1 * e1, rt = level_rate_half(lv), nz = lv != 0;
    s0 = rsum16(s0);   // over the 16 lanes of the variant (rows of 16)
    s1 = rsum16(s1);
    rt = rsum16(rt);
    nz = ror16(nz);
    const int rate = kTuRateHalf + rt;
    int f = nz;
    if (f && 512ll * s0 <= 512ll * s1 + (long long)lam * rate) f = 0;
    const long long j = f ? 512ll * s1 + (long long)lam * rate : 512ll * s0;
    const int g0 = comp * 32;
    const int f0 = __shfl(f, g0), f1 = __shfl(f, g0 + 16);
    const long long j0 = shfl64(j, g0), j1 = shfl64(j, g0 + 16);
    const int use = (f1 && j1 < j0) ? 1 : 0;
    const int fsel = use ? f1 : f0;
    const int lv_t = __shfl(lv, g0 + 16 + s), rec_t = __shfl(rec, g0 + 16 + s);
    if (!var) {
        lev_c[64 * comp + s] = (int16_t)(fsel ? (use ? lv_t : lv) : 0);
        W[o] = (uint8_t)(fsel ? (use ? rec_t : rec) : p);
    }
    // every lane returns both components' results
    fc[0] = __shfl(fsel, 0);
    fc[1] = __shfl(fsel, 32);
    Jc[0] = shfl64(use ? j1 : j0, 0);
    Jc[1] = shfl64(use ? j1 : j0, 32);
    tsc[0] = __shfl(use, 0);
    tsc[1] = __shfl(use, 32);
    wsync();
}

// One intra unit (hevc_cpu.cpp code_unit_intra): a CU16 chooses the 16x16 TU against the
// split tree, each 8x8 node's TU against its four 4x4 TUs (transform skip tried); a
// CU8-split unit codes each CU8 with its own modes (PART_2Nx2N: 8x8 TU or four 4x4,
// PART_NxN: four 4x4 TUs, one per PU); every TU is predicted from the reconstruction before
// it. `ci` holds the modes (ipm) and the CU8 structure. The committed split reconstruction
// lives in L.recS. Levels to gcoef, fields into cu; returns the chosen reconstruction.
__device__ const uint8_t* intra_cu(CuLds& L, const int8_t* T, const FrameArgs& f, int cx, int cy, int nbm,
                                   const CuInfo& ci, int qp, int16_t* gcoef, CuInfo& cu, bool reg) {
    const int l = lane(), qpc = chroma_qp(qp), lam = rd_lambda_q8(qp);
    const Planes& P = f.rec;
    const bool cu8 = (ci.cu8 & 16) != 0;
    load_nb(L, P, f, cx, cy, nbm);
    // (a) one 16x16 TU (CU16 only)
    long long ja = 0x7fffffffffffffffll;
    if (!cu8) {
        const int avc = cu_avail(nbm), m0 = ci.ipm[0];
        intra_tu_pred(L, nullptr, P, f, cx, cy, 0, 4, 0, 0, avc, m0);
        intra_tu_pred(L, nullptr, P, f, cx, cy, 1, 3, 0, 0, avc, m0);
        intra_tu_pred(L, nullptr, P, f, cx, cy, 2, 3, 0, 0, avc, m0);
        tu_batch(L, T, 0, 0, 4, 1, false, false, qp, true, lam, L.levA, L.recA, L.tj[0], L.tf[0]);
        tu_batch(L, T, 1, 0, 3, 2, false, false, qpc, true, lam, L.levA + kCoefCb, L.recA, L.tj[0] + 1, L.tf[0] + 1);
        ja = L.tj[0][0] + L.tj[0][1] + L.tj[0][2];
    }
    // (b) four nodes / CU8s, reconstruction committed into W = L.recS
    uint8_t* W = L.recS;
    long long jb = (long long)lam * kSplitRateHalf;
    int split8 = 0, c8 = 0, c4 = 0, tuc = 0, tsy = 0, tsc = 0;
    for (int q = 0; q < 4; q++) {
        const int av = tu_avail(q, nbm), ox = 8 * (q & 1), oy = 8 * (q >> 1), o8 = oy * 16 + ox;
        const int mq = ci.ipm[4 * q], nxn = cu8 && ((ci.cu8 >> q) & 1);
        long long j8 = 0x7fffffffffffffffll;
        if (!nxn) {
            intra_tu_pred(L, W, P, f, cx, cy, 0, 3, ox, oy, av, mq);
            tu_batch(L, T, 2, o8, 3, 1, false, false, qp, true, lam, L.lev8 + 64 * q, L.rec4t, L.tj[1] + q, L.tf[1] + q);
            j8 = L.tj[1][q];
        }
        long long j4 = (long long)lam * kSplit8RateHalf;
        for (int j = 0; j < 4; j++) {
            const int bx = 2 * (q & 1) + (j & 1), by = 2 * (q >> 1) + (j >> 1), t4 = 4 * q + j, o4 = 4 * by * 16 + 4 * bx;
            const int m4 = ci.ipm[t4];
            if (reg) {   // registers (intra4x4_step)
                long long jt;
                int tsb;
                const int f4 = intra4x4_step(L, T, W, bx, by, tu_avail_at(bx, by, 1, nbm), m4, qp, lam, L.lev4 + 16 * t4,
                                             &jt, &tsb);
                tsy |= tsb << t4;
                j4 += jt;
                c4 |= f4 << t4;
                continue;
            }
            intra_tu_pred(L, W, P, f, cx, cy, 0, 2, 4 * bx, 4 * by, tu_avail_at(bx, by, 1, nbm), m4);
            tu_batch(L, T, 2, o4, 2, 1, true, false, qp, true, lam, L.lev4 + 16 * t4, W, L.tj[2] + t4, L.tf[2] + t4,
                     L.lev4t + 16 * t4, L.rec4, L.tj[3] + t4, L.tf[3] + t4);
            const int mm = merge_ts(L, 2, o4, 1, L.lev4 + 16 * t4, W, L.tj[2] + t4, L.tf[2] + t4, L.lev4t + 16 * t4, L.rec4,
                                    L.tj[3] + t4, L.tf[3] + t4);
            tsy |= mm << t4;
            j4 += L.tj[2][t4];
            c4 |= L.tf[2][t4] << t4;
        }
        if (!nxn) c8 |= L.tf[1][q] << q;
        if (j4 < j8) {
            split8 |= 1 << q;
            jb += j4;
        } else {
            blk_copy(W, L.rec4t, o8, 8);
            tsy &= ~(15 << (4 * q));
            jb += j8;
            wsync();
        }
        // the node's Cb and Cr 4x4 TUs (slots q, q + 4), the CU8's / CU16's chroma mode
        if (reg) {   // registers (intra_c4_pair)
            int fcc[2], tcc[2];
            long long jcc[2];
            intra_c4_pair(L, T, W, ox / 2, oy / 2, av, mq, qpc, lam, L.levc + 16 * q, fcc, jcc, tcc);
#pragma unroll
            for (int cc = 0; cc < 2; cc++) {
                const int t = q + 4 * cc;
                tsc |= tcc[cc] << t;
                jb += jcc[cc];
                tuc |= fcc[cc] << t;
            }
            continue;
        }
        const int ocb = kCoefCb + (oy / 2) * 8 + ox / 2;
        intra_tu_pred(L, W, P, f, cx, cy, 1, 2, ox / 2, oy / 2, av, mq);
        intra_tu_pred(L, W, P, f, cx, cy, 2, 2, ox / 2, oy / 2, av, mq);
        int16_t* lc = L.levct + 64;   // scratch pair: Cb / Cr levels of this node (compact), copied below
        int16_t* lct = L.levct + 96;
        tu_batch(L, T, 3, ocb, 2, 2, false, false, qpc, true, lam, lc, W, L.tj[4] + 8, L.tf[4] + 8, lct, L.rec4,
                 L.tj[5] + 8, L.tf[5] + 8);
        const int mc = merge_ts(L, 3, ocb, 2, lc, W, L.tj[4] + 8, L.tf[4] + 8, lct, L.rec4, L.tj[5] + 8, L.tf[5] + 8);
        for (int i = l; i < 32; i += 64) L.levc[16 * (q + 4 * (i >> 4)) + (i & 15)] = lc[i];
        for (int cc = 0; cc < 2; cc++) {
            const int t = q + 4 * cc;
            tsc |= ((mc >> cc) & 1) << t;
            jb += L.tj[4][8 + cc];
            tuc |= L.tf[4][8 + cc] << t;
        }
        wsync();
    }
    if (jb < ja) {
        for (int i = l; i < 256; i += 64) gcoef[i] = ((split8 >> (i >> 6)) & 1) ? L.lev4[i] : L.lev8[i];
        for (int i = l; i < 128; i += 64) gcoef[kCoefCb + i] = L.levc[i];
        cu.tu = (uint8_t)(16 | split8);
        cu.tuc = (uint8_t)tuc;
        uint16_t m = 0;
        for (int q = 0; q < 4; q++)
            m |= (uint16_t)((((split8 >> q) & 1) ? (c4 >> (4 * q)) & 15 : (((c8 >> q) & 1) ? 15 : 0)) << (4 * q));
        cu.ycbf = m;
        cu.cbf = (uint8_t)((m ? 1 : 0) | ((tuc & 15) ? 2 : 0) | ((tuc >> 4) ? 4 : 0));
        cu.tsy = (uint16_t)tsy;
        cu.tsc = (uint8_t)tsc;
        wsync();
        return W;
    }
    const int cbfa = L.tf[0][0] | (L.tf[0][1] << 1) | (L.tf[0][2] << 2);
    for (int i = l; i < kCoefPerCu; i += 64) gcoef[i] = L.levA[i];
    cu.tu = cu.tuc = 0;
    cu.cbf = (uint8_t)cbfa;
    cu.ycbf = (cbfa & 1) ? 0xffff : 0;
    cu.tsy = 0;
    cu.tsc = 0;
    wsync();
    return L.recA;
}

// Codes intra unit (ux, uy) (its decisions from k_hevc_intra_prep) and commits it.
__device__ void intra_unit(const HevcArgs& A, CuLds& L, const int8_t* T, int ux, int uy, int qp) {
    const FrameArgs& f = A.f;
    const int idx = uy * f.mb_w + ux, l = lane();
    const int nbm = unit_nbm(ugrid(A), smap(A), ux, uy);
    CuInfo cu = A.cus[idx];   // mode, cu8, ipm from k_hevc_intra_prep
    load_src(L, f, ux, uy);
    wsync();
    const uint8_t* rec = intra_cu(L, T, f, ux, uy, nbm, cu, qp, A.coefs + (size_t)idx * kCoefPerCu, cu, A.reg_steps != 0);
    store_rec(rec, f, ux, uy);
    if (l == 0) {
        cu.qp = (uint8_t)qp;
        A.cus[idx] = cu;
        f.me[idx].mvx = 0;
        f.me[idx].mvy = 0;
        f.me[idx].ref = 0;
        f.me[idx].fx = f.me[idx].fy = 0;
    }
    // this unit's reconstruction (global memory) is the next one's neighbour
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    wsync();
}

// I slices: one workgroup per slice, wave w = CTB row w of the slice, CTB x coded at
// step x + 2w (the top-right CTB is one step older: WPP / intra availability order), its
// units in z order.
template <int MAXR>
__global__ __launch_bounds__(64 * MAXR) void k_hevc_intra(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ CuLds Lw[MAXR];
    __shared__ int8_t T[kTabT];
    const FrameArgs& f = A.f;
    const SliceTask t = f.tasks[blockIdx.x];
    if (t.final_action != ACT_I || A.seg_k > 1) return;   // block-uniform; split rows: k_hevc_intra_seg
    load_t16(T);
    __syncthreads();
    const int w = threadIdx.x >> 6;
    CuLds& L = Lw[w];
    const UnitGrid ug = ugrid(A);
    const int r0 = t.first_row >> 1, rows = ((t.first_row + t.num_rows + 1) >> 1) - r0;
    const int steps = A.cw + 2 * (rows - 1);
    const int r = r0 + w;
    __builtin_amdgcn_s_setprio(3);
    for (int step = 0; step < steps; step++) {
        const int c = step - 2 * w;
        if (w < rows && c >= 0 && c < A.cw)
            for (int z = 0; z < 4; z++) {
                const int ux = 2 * c + (z & 1), uy = 2 * r + (z >> 1);
                if (ug.inside(ux, uy)) intra_unit(A, L, T, ux, uy, t.qp);
            }
        __syncthreads();   // this step's reconstruction is visible to the next step's neighbours
    }
}

// I slices cut into row segments (SliceMap, seg_k > 1): one wave per segment, its CTBs
// left to right (units in z order); no top neighbours, so the segments of all rows run at
// once (a 4K key frame: 816 chains of 40 units instead of 34 workgroups of 124 steps).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_hevc_intra_seg(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ CuLds Lw[4];
    __shared__ int8_t T[kTabT];
    load_t16(T);
    __syncthreads();   // the only block barrier: waves run independent segments below
    const int w = threadIdx.x >> 6;
    const int slot = blockIdx.x * 4 + w;
    if (slot >= A.ch * A.seg_k) return;
    const SliceMap m = smap(A);
    const int r = slot / A.seg_k, k = slot - r * A.seg_k;
    if (!m.split(r)) return;
    const SliceTask t = ctb_task(A, r);
    const UnitGrid ug = ugrid(A);
    CuLds& L = Lw[w];
    __builtin_amdgcn_s_setprio(3);
    for (int c = m.x0(r, k); c < m.x1(r, k); c++)
        for (int z = 0; z < 4; z++) {
            const int ux = 2 * c + (z & 1), uy = 2 * r + (z >> 1);
            if (ug.inside(ux, uy)) intra_unit(A, L, T, ux, uy, t.qp);
        }
}

// ---------------------------------------------------------------------------
// Unit syntax -> bin entries (hevc_cpu.cpp binarize_slice: SAO of the CTB at its first
// unit, code_unit, end_of_slice_segment_flag / end_of_subset_one_bit after its last): one
// wave per unit. The CU syntax runs wave-uniform (lane 0 stores); each TU's residual runs
// sub-block-parallel, lane j = sub-block j of the scan: every lane derives its sub-block's
// coded_sub_block_flag neighbours and entering greater1 state from ballots / shuffles, counts
// its entries, and writes them at its offset in coding order (descending j) after a wave
// scan. The same code_last / code_sb as the CPU's serial code_residual: identical bins.
__device__ __forceinline__ uint64_t wor64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)v, o), hi = __shfl_xor((uint32_t)(v >> 32), o);
        v |= ((uint64_t)hi << 32) | lo;
    }
    return v;
}
struct WaveBinBuf {
    static constexpr bool kWave = true;
    uint16_t* p;
    int n;   // wave-uniform
    __device__ __forceinline__ void ctx(int c, int b) {
        if (lane() == 0) p[n] = (uint16_t)(((b & 1) << 8) | c);
        n++;
    }
    __device__ __forceinline__ void term(int b) {
        if (lane() == 0) p[n] = (uint16_t)(((b & 1) << 8) | CTX_TERM);
        n++;
    }
    __device__ __forceinline__ void bypass(uint32_t v, int nb) {
        if (lane() == 0) {
            BinBuf t{p, n};
            t.bypass(v, nb);
        }
        n += (nb + 7) >> 3;
    }
    template <class C>
    __device__ void residual(C c, int log2n, int cidx, int scan, int ts, int lo, int hi) {
        if (log2n == 2) {   // one sub-block: lane 0 alone, serially (no ballots, scans or second pass)
            int cnt = 0;
            if (lane() == 0) {
                BinBuf b{p, n};
                code_residual_serial(b, c, log2n, cidx, scan, ts, lo, hi);
                cnt = b.n - n;
            }
            n += __shfl(cnt, 0);
            return;
        }
        const int j = lane(), n4 = 1 << log2n, sbw = n4 >> 2, nsb = sbw * sbw;
        int sr = 0, xs = 0, ys = 0;
        Sb4 s{0, 0, 0, 0};
        if (j < nsb) {
            sr = sb_scan_raster(log2n, scan, j);
            xs = sr % sbw;
            ys = sr / sbw;
            s = load_sb(c, n4, xs, ys);
        }
        const bool nz = j < nsb && s.nz();
        const uint64_t M = __ballot(nz);
        if (!M) return;   // callers only code TUs with cbf = 1
        const int last_i = 63 - __builtin_clzll(M);
        const int last_n = __shfl(nz ? sb_last_pos(s, scan) : 0, last_i);
        const int i0 = last_i < hi ? last_i : hi;
        if (i0 < lo) return;   // a piece above the last sub-block
        if (i0 == last_i) code_last(*this, log2n, cidx, scan, ts, last_i, last_n);
        const uint64_t cs = wor64(nz ? 1ull << sr : 0ull);   // coded_sub_block_flags, raster
        const int right = (xs + 1 < sbw) ? (int)((cs >> (sr + 1)) & 1) : 0;
        const int below = (ys + 1 < sbw) ? (int)((cs >> (sr + sbw)) & 1) : 0;
        // the greater1 state entering sub-block j: that of the nearest sub-block above j
        // (coded before it) holding a level
        const int g = nz ? sb_g1(s, scan) : 0;
        const uint64_t above = M & ~((2ull << j) - 1);   // j = 63: 2 << 63 wraps to 0, mask 0
        const int c1 = __shfl(g, above ? __builtin_ctzll(above) : j);
        const bool act = j >= lo && j <= i0;
        BinCount bc;
        if (act) code_sb(bc, s, log2n, cidx, scan, j, last_i, last_n, xs, ys, right, below, above == 0, c1);
        int incl = bc.n;   // inclusive prefix over lanes 0..j
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(incl, o);
            if (j >= o) incl += t;
        }
        const int total = __shfl(incl, 63);
        if (act) {
            BinBuf wb{p, n + total - incl};   // after the entries of the lanes above j
            code_sb(wb, s, log2n, cidx, scan, j, last_i, last_n, xs, ys, right, below, above == 0, c1);
        }
        n += total;
    }
};

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_hevc_bins(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const FrameArgs& f = A.f;
    const int n = f.mb_w * f.mb_h;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= n) return;   // wave-uniform
    const int W = f.mb_w;
    const int ux = idx % W, uy = idx / W, c = ux >> 1, r = uy >> 1;
    const SliceTask t = ctb_task(A, r);
    const bool p_slice = t.final_action != ACT_I;
    const SliceMap m = smap(A);
    const UnitGrid ug = ugrid(A);
    UnitCtx u;
    u.z = (ux & 1) | ((uy & 1) << 1);
    u.first = u.z == 0;
    u.complete = ug.complete(c, r);
    u.left = ug.avail(m, ux, uy, ux - 1, uy);
    u.top = ug.avail(m, ux, uy, ux, uy - 1);
    u.row0 = (uy & 1) == 0;
    u.p_slice = p_slice;
    const CuInfo& cu = A.cus[idx];
    const size_t i0 = (size_t)2 * r * W + 2 * c;   // the CTB's unit z0
    WaveBinBuf w{A.bins + (size_t)idx * kCuBinCap, 0};
    if (u.first) sao_bins(w, A.sao[r * A.cw + c], m.left(c, r), m.top(c, r));   // CTB-level SAO syntax
    // neighbours and the CU32's units are read in place (no private copies: no scratch)
    code_unit(w, u, cu, A.cus + idx - 1, A.cus + idx - W, A.coefs + (size_t)idx * kCoefPerCu,
              Ctb4{A.cus + i0, A.coefs + i0 * kCoefPerCu, W});
    bool last = true;   // the CTB's last unit in coding order
    for (int k = u.z + 1; k < 4; k++) last &= !ug.inside(2 * c + (k & 1), 2 * r + (k >> 1));
    if (last) {
        const int r1 = ((t.first_row + t.num_rows + 1) >> 1) - 1;   // the slice's last CTB row
        if (m.split(r)) {   // each row segment is a slice: end_of_slice_segment_flag at its end
            w.term(c + 1 == m.x1(r, m.seg(c, r)));
        } else {
            w.term(r == r1 && c == A.cw - 1);
            if (r != r1 && c == A.cw - 1) w.term(1);   // end_of_subset_one_bit closes the row's substream
        }
    }
    if (lane() == 0) A.bin_n[idx] = w.n;
}

// Lane `ln` (wave-uniform) of `v` takes the uniform value `x`: v_writelane_b32 with the
// lane index in M0 (one SGPR read per VALU op on gfx9; no compiler builtin for it).
__device__ __forceinline__ int writelane(int x, int ln, int v) {
    asm("s_nop 0\n\tv_writelane_b32 %0, %1, m0"
        : "+v"(v)
        : "s"(__builtin_amdgcn_readfirstlane(x)), "{m0}"(__builtin_amdgcn_readfirstlane(ln)));
    return v;
}

// WPP context states at each CTB row start of a slice (9.3.2.4: the states after the
// second CTB of the row above). Thread c owns context c and replays only that context's
// bins of the two CTBs' chunks (their units), from k_pc_sort's per-context lists: the
// chains run in parallel and each is a few entries long.
__global__ __launch_bounds__(192) void k_hevc_sync(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ uint8_t nlps[64];
    const FrameArgs& f = A.f;
    const SliceTask t = f.tasks[blockIdx.x];
    const int c = threadIdx.x;
    if (c < 64) nlps[c] = CABAC_NEXT_LPS[c];
    __syncthreads();
    if (c >= CTX_COUNT) return;
    const UnitGrid ug = ugrid(A);
    const int RC = 2 * f.mb_w;   // coff row stride (chunks)
    const int it = t.final_action == ACT_I ? 0 : 1;
    const uint8_t init = ctx_init_state(HEVC_CTX_INIT[it][c], t.qp);
    const int K = A.seg_k, r0 = t.first_row >> 1, nr = ((t.first_row + t.num_rows + 1) >> 1) - r0;
    if (smap(A).split(r0)) {   // every row segment is a slice: initial states
        for (int i = 0; i < nr * K; i++) A.sync[((size_t)r0 * K + i) * CTX_COUNT + c] = init;
        return;
    }
    uint32_t st = init;
    A.sync[(size_t)r0 * K * CTX_COUNT + c] = init;
    for (int rr = 1; rr < nr; rr++) {
        const int prev = r0 + rr - 1;
        if (A.cw >= 2) {
            const uint16_t* co = A.coff + ((size_t)prev * kPcCtxOff + c) * RC;
            const int jn = ug.ctb_chunk0(prev, 2);
            for (int j = 0; j < jn; j++) {
                const uint16_t* sp = A.srt + (size_t)ug.chunk_unit(prev, j) * kCuBinCap;
                const int hi = co[RC + j];
                for (int k = co[j]; k < hi; k++) {
                    const uint32_t bin = sp[k] & 1u, mps = st & 1u, s6 = st >> 1;
                    st = bin == mps ? (((s6 < 62 ? s6 + 1 : 62) << 1) | mps)
                                    : (((uint32_t)nlps[s6] << 1) | (s6 == 0 ? mps ^ 1u : mps));
                }
            }
        } else {
            st = init;
        }
        A.sync[(size_t)(r0 + rr) * K * CTX_COUNT + c] = (uint8_t)st;
    }
}

// ---------------------------------------------------------------------------
// Chunk-parallel substream coding (codec/hevc_pcabac.h has the derivation and the host
// model): k_pc_sort -> k_pc_model -> k_pc_rmap -> k_pc_compose -> k_pc_code ->
// k_pc_merge. Chunk = unit (the units of a CTB row in coding order, UnitGrid::chunk_unit),
// so every phase but the per-row composition and merge runs one wave per unit or per (CTB
// row, context). Same bytes as CabacEncoder (hevc_core.h).
constexpr int kPcMaxRowChunks = 1024;   // units per CTB row (8K width); alloc_hevc checks it
constexpr int kPcMaxRowCtb = 512;       // CTBs per row (SAO row pass)

// One wave per CTB: stable counting sort of its context bins by context index.
__global__ __launch_bounds__(256) void k_pc_sort(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
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
    // coff is [CTB row][context][chunk]: k_pc_model and k_hevc_sync read one context's
    // offsets along a row as one contiguous run
    const int uy = idx / f.mb_w, ux = idx - uy * f.mb_w, RC = 2 * f.mb_w;
    uint16_t* co = A.coff + (size_t)(uy >> 1) * kPcCtxOff * RC + ugrid(A).unit_chunk(ux, uy);
#pragma unroll
    for (int k = 0; k < 3; k++) {
        if (3 * l + k < kPcCtxOff) {
            cnt[3 * l + k] = run;
            co[(size_t)(3 * l + k) * RC] = (uint16_t)run;
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

// One wave per (CTB row, context, slice group): the context's state chain along the
// row's chunks, from its WPP start state; each context bin is rewritten in place as a
// modelled entry (LPS state, is-LPS). The chunks holding the context are listed with the
// prefix of their counts; the chain itself runs as up to 64 speculative segments, one per
// lane (below).
constexpr int kPcModelZ = 4;   // k_pc_model workgroups per (row, context group)
__global__ __launch_bounds__(256) void k_pc_model(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ uint2 lst_s[4][kPcMaxRowChunks + 1];   // (chunk | lo << 16, chain position of its first entry)
    __shared__ uint8_t nl_s[4][64];                // CABAC_NEXT_LPS
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int cy = blockIdx.x, c = blockIdx.y * 4 + w;
    if (c >= CTX_COUNT) return;
    const SliceMap m = smap(A);
    const UnitGrid ug = ugrid(A);
    const int RC = 2 * f.mb_w;
    uint8_t* nl = nl_s[w];
    nl[l] = CABAC_NEXT_LPS[l];
    // the row's slices k = z, z + kPcModelZ, ... (a split key-frame row: its segments'
    // short chains, a few per wave; a grid of every possible slot launched tens of
    // thousands of LDS-heavy workgroups that exit at once on the P frames)
    for (int k = blockIdx.z; k < m.nseg(cy); k += kPcModelZ) {
    const int slot = cy * A.seg_k + k;
    const int xa = ug.ctb_chunk0(cy, m.x0(cy, k));
    const int xb = m.x1(cy, k) < A.cw ? ug.ctb_chunk0(cy, m.x1(cy, k)) : ug.row_chunks(cy);
    uint2* L = lst_s[w];
    const uint64_t lt = (1ull << l) - 1;
    int n = 0, tot = 0;
    for (int g = xa; g < xb; g += 64) {
        const int cx = g + l;
        int lo = 0, cnt = 0;
        if (cx < xb) {
            const uint16_t* co = A.coff + ((size_t)cy * kPcCtxOff + c) * RC + cx;
            lo = co[0];
            cnt = co[RC] - lo;
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
    if (tot == 0) continue;
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readfirstlane(A.sync[(size_t)slot * CTX_COUNT + c]);
    // The chain is cut into up to 64 segments, lane = segment (>= 32 entries each).
    // Pass 1 runs every segment from a guessed start state; CABAC states forget their
    // start quickly (MPS runs saturate, LPS steps contract), so segment j-1's end state
    // from the guess is almost always segment j's true start. Pass 2 runs from those
    // starts and writes the modelled entries; a start that does not match the true end
    // of the segment before it is corrected and its segment re-run (loop until none).
    const int seglen = tot > 64 * A.pc_seg ? (tot + 63) / 64 : A.pc_seg;
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
                cu[j] = (uint32_t)ug.chunk_unit(cy, (int)(it.x & 0xffffu));
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
    wsync();   // L is rebuilt for the next slice of the row
    }
}

// One wave per CTB: the chunk's range map. Lane l follows the start ranges 256 + 4l .. +3
// through the chunk's entries (bypass runs and terminating bins shift all of them alike).
__global__ __launch_bounds__(256) void k_pc_rmap(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
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
// lookup each (a readlane); the maps of the next 16 chunks are in flight.
__global__ __launch_bounds__(64) void k_pc_compose(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const FrameArgs& f = A.f;
    const int slot = blockIdx.x, l = lane();
    const SliceMap m = smap(A);
    const int cy = slot / A.seg_k, k = slot - cy * A.seg_k;
    if (k >= m.nseg(cy)) return;
    // the segment's chunks as a row of their own: chunk j0 + d = unit ug.chunk_unit(cy, j0 + d)
    const UnitGrid ug = ugrid(A);
    const int j0 = ug.ctb_chunk0(cy, m.x0(cy, k));
    const int nw = (m.x1(cy, k) < A.cw ? ug.ctb_chunk0(cy, m.x1(cy, k)) : ug.row_chunks(cy)) - j0;
    auto unit = [&](int d) { return ug.chunk_unit(cy, j0 + d); };
    constexpr int D = 16;
    uint4 buf[D];
#pragma unroll
    for (int d = 0; d < D; d++)
        buf[d] = reinterpret_cast<const uint4*>(A.rmap + (size_t)unit(d < nw ? d : nw - 1) * 256)[l];
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
                        const int u = unit((cx & ~63) + l);
                        A.cu_r[u] = (uint16_t)vr;
                        A.cu_t[u] = (uint32_t)vt;
                    }
                }
                r = val & 511u;
                T += val >> 9;
            }
            const int nx = cx + D < nw ? cx + D : nw - 1;
            buf[d] = reinterpret_cast<const uint4*>(A.rmap + (size_t)unit(nx) * 256)[l];
        }
    }
    if (l == 0) A.row_bits[slot] = T;
}

// One wave per CTB: the chunk coded from V = 0 (PcCoder, scalar state) and fully
// flushed; bytes gathered in a VGPR (lane = 4 bytes) and stored every 256: the exclusive
// ones into the row substream, the last two into the chunk's tail.
__global__ __launch_bounds__(256) void k_pc_code(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int idx = blockIdx.x * 4 + w;
    if (idx >= f.mb_w * f.mb_h) return;
    const int uy = idx / f.mb_w, ux = idx - uy * f.mb_w, cy = uy >> 1, cx = ux >> 1;
    const SliceMap m = smap(A);
    const UnitGrid ug = ugrid(A);
    const int k = m.seg(cx, cy), slot = cy * A.seg_k + k;
    const int j = ug.unit_chunk(ux, uy);
    const int jend = m.x1(cy, k) < A.cw ? ug.ctb_chunk0(cy, m.x1(cy, k)) : ug.row_chunks(cy);
    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)A.cu_t[idx]);
    const uint32_t tn = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(j + 1 < jend ? A.cu_t[ug.chunk_unit(cy, j + 1)] : A.row_bits[slot]));
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)A.cu_r[idx]);
    const int g0 = (int)(t0 >> 3), nex = (int)(tn >> 3) - g0;
    uint8_t* out = A.sub + sub_base(A, m, cy, k) + g0;
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

// Emulation prevention over 256 bytes per wave step: lane l holds bytes i0 .. i0 + 3 (word
// w, little-endian; bytes at or past n read as 1). Byte i is preceded by an inserted 0x03
// iff it is <= 3 and the zero run before it has even length >= 2 (the sequential rule,
// given a non-zero byte before the piece). Returns the lane's insertion mask (bit j: before
// byte i0 + j); *excl = insertions of the lanes before it, *tot = of the step; last_nz
// carries the last non-zero position across steps.
__device__ __forceinline__ int ep_step(uint32_t w, int i0, int n, int& last_nz, int* excl, int* tot) {
    const int l = lane();
    int lane_last = -1;
#pragma unroll
    for (int j = 0; j < 4; j++)
        if ((w >> (8 * j)) & 255u) lane_last = i0 + j;
    int p = lane_last;   // inclusive max-scan of non-zero positions
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int q = __shfl_up(p, d);
        if (l >= d) p = max(p, q);
    }
    int prev = __shfl_up(p, 1);
    if (l == 0) prev = -1;
    prev = max(prev, last_nz);
    int m = 0, c = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int i = i0 + j, b = (int)((w >> (8 * j)) & 255u), z = i - 1 - prev;
        if (i < n && b <= 3 && z >= 2 && (z & 1) == 0) {
            m |= 1 << j;
            c++;
        }
        if (b) prev = i;
    }
    int inc = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int q = __shfl_up(inc, d);
        if (l >= d) inc += q;
    }
    *excl = inc - c;
    *tot = __shfl(inc, 63);
    last_nz = max(last_nz, __shfl(p, 63));
    return m;
}
// Word wi of a substream of n bytes (4-byte aligned base), bytes at or past n as 1.
__device__ __forceinline__ uint32_t ep_word(const uint8_t* in, int wi, int n) {
    const int i = 4 * wi;
    if (i >= n) return 0x01010101u;
    uint32_t w = *reinterpret_cast<const uint32_t*>(in + i);
    if (i + 4 > n) w = (w & (0xffffffffu >> (8 * (i + 4 - n)))) | (0x01010101u << (8 * (n - i)));
    return w;
}

// One wave per CTB row: adds every chunk's tail into the substream (a 256-byte window
// of it in a VGPR; carries run toward the start), writes the rbsp stop bit, then counts
// the emulation-prevention bytes (same rule as k_hevc_ep_copy).
__global__ __launch_bounds__(64) void k_pc_merge(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const FrameArgs& f = A.f;
    const int slot = blockIdx.x, l = lane();
    const SliceMap m = smap(A);
    const int cy = slot / A.seg_k, k = slot - cy * A.seg_k;
    if (k >= m.nseg(cy)) {   // unused slot: no substream (k_rc_account sums every slot)
        if (l == 0) A.sub_size[slot] = A.sub_esc[slot] = 0;
        return;
    }
    const UnitGrid ug = ugrid(A);
    const int j0 = ug.ctb_chunk0(cy, m.x0(cy, k));
    const int nw = (m.x1(cy, k) < A.cw ? ug.ctb_chunk0(cy, m.x1(cy, k)) : ug.row_chunks(cy)) - j0;
    const uint32_t T = (uint32_t)__builtin_amdgcn_readfirstlane((int)A.row_bits[slot]);
    const int excl = (int)(T >> 3), nbytes = excl + 2;
    uint8_t* out = A.sub + sub_base(A, m, cy, k);
    int wb = 0;
    uint32_t win = 0;
    // bytes excl, excl + 1 (past the chunks' exclusive bytes) start as zero: cleared here so
    // that a window reloaded after tails were added there (and stored) reads them back
    if (l == 0) {
        out[excl] = 0;
        out[excl + 1] = 0;
    }
    __threadfence();
    auto load_win = [&]() __attribute__((always_inline)) {
        const int q = wb + 4 * l;
        uint32_t v = 0;
        if (q + 4 <= nbytes) {
            for (int k = 0; k < 4; k++) v |= (uint32_t)out[q + k] << (8 * k);
        } else {
            for (int k = 0; k < 4; k++)
                if (q + k < nbytes) v |= (uint32_t)out[q + k] << (8 * k);
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
    for (int g = 0; g < nw; g += 64) {
        const int cx = g + l;   // chunk j0 + cx of the segment
        int p_l = 0, t_l = 0;
        if (cx < nw) {
            const int u = ug.chunk_unit(cy, j0 + cx);
            p_l = (int)((cx + 1 < nw ? A.cu_t[ug.chunk_unit(cy, j0 + cx + 1)] : T) >> 3);
            t_l = (int)((uint32_t)A.tail[2 * u] | ((uint32_t)A.tail[2 * u + 1] << 8));
        }
        const int mm = nw - g < 64 ? nw - g : 64;
        for (int j = 0; j < mm; j++) {
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
    for (int base = 0; base < size; base += 256) {
        const int wi = (base >> 2) + l;
        int ex, tot;
        ep_step(ep_word(out, wi, size), 4 * wi, size, last_nz, &ex, &tot);
        ins_total += tot;
    }
    if (l == 0) {
        A.sub_size[slot] = size;
        A.sub_esc[slot] = size + ins_total;
        if (A.dbg && k == 0) {
            A.dbg[4 * cy + 0] = 0;
            A.dbg[4 * cy + 1] = T;
            A.dbg[4 * cy + 2] = (unsigned long long)size;
            A.dbg[4 * cy + 3] = 0;
        }
    }
}

// Slice header + NAL prefix per slice; substream offsets for k_hevc_ep_copy. A split
// intra slice (SliceMap) is one slice NAL per row segment, laid out back to back in the
// slice's output slot: lane j writes segment j's header, a scan places them.
constexpr int kMaxSegsPerSlice = 256;
__global__ __launch_bounds__(64) void k_hevc_hdr(HevcArgs A) {
    __shared__ uint8_t hdr[1024];
    __shared__ int esc[256];
    __shared__ int offs[kMaxSegsPerSlice + 1];
    __shared__ uint8_t shdr[64][48];
    const FrameArgs& f = A.f;
    const int s = blockIdx.x;
    const SliceTask t = f.tasks[s];
    const int l = lane();
    const SliceMap m = smap(A);
    bool idr = true;
    for (int i = l; i < f.num_slices; i += 64) idr &= f.tasks[i].final_action == ACT_I && f.tasks[i].idr_on_intra;
    idr = __syncthreads_and(idr);
    const int r0 = t.first_row >> 1, nr = ((t.first_row + t.num_rows + 1) >> 1) - r0;   // CTB rows
    auto seg_header = [&](int cy, int k, uint8_t* buf) {   // header RBSP of a row segment
        for (int i = 0; i < 48; i++) buf[i] = 0;
        SliceHeader h;
        h.address = cy * A.cw + m.x0(cy, k);
        h.first_slice = h.address == 0;
        h.idr = idr;
        h.address_bits = A.addr_bits;
        h.slice_type = 2;
        h.poc_lsb = t.frame_num & ((1 << kLog2MaxPocLsb) - 1);
        h.qp_delta = t.qp - 26;
        h.num_entry = 0;
        h.entry = nullptr;
        return write_slice_header(buf, h);
    };
    if (m.split(r0)) {
        const int K = A.seg_k, nseg = nr * K;
        int run = 0;
        for (int base = 0; base < nseg; base += 64) {   // pass 1: NAL lengths -> offsets
            const int j = base + l;
            int len = 0;
            if (j < nseg) {
                const int cy = r0 + j / K, k = j % K;
                const int hn = seg_header(cy, k, shdr[l]);
                len = 6 + ep_escape(shdr[l], hn, nullptr) + A.sub_esc[cy * K + k];
            }
            int inc = len;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int v = __shfl_up(inc, o);
                if (l >= o) inc += v;
            }
            if (j < nseg) offs[j] = run + inc - len;
            run += __shfl(inc, 63);
        }
        __syncthreads();
        const int total = run;
        const bool fits = total <= A.out_slot;
        uint8_t* o = fits ? A.out_host + (size_t)s * A.out_slot : A.out_dev + (size_t)s * A.out_dev_slot;
        for (int base = 0; base < nseg; base += 64) {   // pass 2: NAL prefixes and headers
            const int j = base + l;
            if (j < nseg) {
                const int cy = r0 + j / K, k = j % K;
                const int hn = seg_header(cy, k, shdr[l]);
                uint8_t* d = o + offs[j];
                d[0] = 0; d[1] = 0; d[2] = 0; d[3] = 1;
                d[4] = (uint8_t)((idr ? kNalIdrWRadl : kNalTrailR) << 1);
                d[5] = 1;
                const int hesc = ep_escape(shdr[l], hn, d + 6);
                A.row_off[cy * K + k] = offs[j] + 6 + hesc;
            }
        }
        if (l == 0) __hip_atomic_store(A.out_size + s, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    for (int i = l; i < 1024; i += 64) hdr[i] = 0;
    for (int i = l; i < nr; i += 64) esc[i] = A.sub_esc[(r0 + i) * A.seg_k];
    __syncthreads();
    if (l == 0) {
        SliceHeader h;
        h.first_slice = s == 0;
        h.idr = idr;
        h.address = r0 * A.cw;
        h.address_bits = A.addr_bits;
        h.slice_type = t.final_action == ACT_I ? 2 : 1;
        h.poc_lsb = t.frame_num & ((1 << kLog2MaxPocLsb) - 1);
        h.qp_delta = t.qp - 26;
        h.num_entry = nr - 1;
        h.entry = esc;
        const int hn = write_slice_header(hdr, h);
        const int hesc = ep_escape(hdr, hn, nullptr);
        int total = 6 + hesc;
        int off = total;
        for (int r = 0; r < nr; r++) {
            A.row_off[(r0 + r) * A.seg_k] = off;
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

// Emulation prevention + copy of one slot's substream (a row, or a row segment), wave-parallel
// over 256-byte steps (ep_step): byte i of the substream is preceded by an inserted 0x03 iff it
// is <= 3 and the zero run before it has even length >= 2 (equivalent to the sequential rule;
// the previous piece ends in a non-zero byte).
__global__ __launch_bounds__(64) void k_hevc_ep_copy(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int slot = blockIdx.x;
    const SliceMap m = smap(A);
    const int cy = slot / A.seg_k, k = slot - cy * A.seg_k;
    if (k >= m.nseg(cy)) return;
    const int s = cy / A.rps;
    const int total = __hip_atomic_load(A.out_size + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const bool fits = total <= A.out_slot;
    uint8_t* o = (fits ? A.out_host + (size_t)s * A.out_slot : A.out_dev + (size_t)s * A.out_dev_slot) + A.row_off[slot];
    const uint8_t* in = A.sub + sub_base(A, m, cy, k);
    const int n = A.sub_size[slot];
    const int l = lane();
    int last_nz = -1;   // the last non-zero byte before the current step (-1: none yet,
                        // the byte before the substream is non-zero)
    int opos = 0;
    uint32_t w = ep_word(in, l, n);
    for (int base = 0; base < n; base += 256) {
        const int wi = (base >> 2) + l;
        const uint32_t wn = ep_word(in, wi + 64, n);   // the next step's word in flight
        int ex, tot;
        const int m = ep_step(w, 4 * wi, n, last_nz, &ex, &tot);
        int at = 4 * wi + opos + ex;   // output position of byte 4 wi (before its own insertions)
#pragma unroll
        for (int j = 0; j < 4; j++) {
            if (4 * wi + j >= n) break;
            if ((m >> j) & 1) o[at++] = 3;
            o[at++] = (uint8_t)((w >> (8 * j)) & 255u);
        }
        opos += tot;
        w = wn;
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
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const h264::gpu::FrameArgs& f = A.f;
    const int cw = f.mb_w, ch = f.mb_h, ne = cw - 1, nel = 2 * cw - 1;   // units
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int nl = ch * 4 * nel, nc = ch * 8 * ne;
    const SliceMap m = smap(A);
    if (e < nl) {
        const int x = 8 * (1 + e % nel), seg = e / nel;
        if (!(x & 8) && !m.same_u((x >> 4) - 1, seg >> 2, x >> 4, seg >> 2)) return;   // slice boundary
        dbk_luma_edge(f.rec.y, f.stride_y, A.cus, cw, true, x, 4 * seg);
    } else if (e < nl + 2 * nc) {
        const int k0 = e - nl, plane = k0 / nc, k = k0 % nc;
        const int cx = 1 + k % ne, line = k / ne, cy = line >> 3;
        const CuInfo p = A.cus[cy * cw + cx - 1], q = A.cus[cy * cw + cx];
        if (cu_intra_edge(p, q) && m.same_u(cx - 1, cy, cx, cy))
            dbk_chroma_line((plane ? f.rec.v : f.rec.u) + (size_t)line * f.stride_c + cx * 8, 1, (p.qp + q.qp + 1) >> 1);
    }
}

__global__ __launch_bounds__(256) void k_hevc_dbk_h(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const h264::gpu::FrameArgs& f = A.f;
    const int cw = f.mb_w, ch = f.mb_h, ne = ch - 1, nel = 2 * ch - 1;   // units
    if (nel <= 0) return;
    const int e = blockIdx.x * 256 + threadIdx.x;
    const int nl = nel * cw * 4, nc = ne * cw * 8;
    const SliceMap m = smap(A);
    if (e < nl) {
        const int y = 8 * (1 + e / (cw * 4)), x4 = e % (cw * 4);
        if (!(y & 8) && !m.same_u(x4 >> 2, (y >> 4) - 1, x4 >> 2, y >> 4)) return;   // slice boundary
        dbk_luma_edge(f.rec.y, f.stride_y, A.cus, cw, false, y, 4 * x4);
    } else if (e < nl + 2 * nc) {
        const int k0 = e - nl, plane = k0 / nc, k = k0 % nc;
        const int cy = 1 + k / (cw * 8), col = k % (cw * 8), cx = col >> 3;
        if (!m.same_u(cx, cy - 1, cx, cy)) return;
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
// Sample i (0..1535) of CTB (cx, cy): component and plane coordinates; false when it lies
// outside the picture (the partial CTBs of the last row / column).
constexpr int kCtbSamples = 1536;
__device__ __forceinline__ bool ctb_sample(const HevcArgs& A, int i, int cx, int cy, int* c, int* x, int* y) {
    if (i < 1024) {
        *c = 0; *x = cx * 32 + (i & 31); *y = cy * 32 + (i >> 5);
        return *x < A.f.mb_w * 16 && *y < A.f.mb_h * 16;
    }
    const int j = i - 1024;
    *c = 1 + (j >> 8); *x = cx * 16 + (j & 15); *y = cy * 16 + ((j >> 4) & 15);
    return *x < A.f.mb_w * 8 && *y < A.f.mb_h * 8;
}
__device__ __forceinline__ SaoPlane sao_plane_of(const HevcArgs& A, int c) {
    const int n = c ? 16 : 32, u = c ? 8 : 16;
    return SaoPlane{A.f.mb_w * u, A.f.mb_h * u, n, smap(A)};
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_hevc_sao_stats(HevcArgs A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ SaoStats Sw[4][3];
    __shared__ SaoTables Tw[4];
    const FrameArgs& f = A.f;
    const int w = threadIdx.x >> 6, l = lane();
    const int idx = blockIdx.x * 4 + w;
    if (idx >= A.cw * A.ch) return;   // wave-uniform; no block barriers below
    const int cx = idx % A.cw, cy = idx / A.cw;
    const SliceTask t = ctb_task(A, cy);
    SaoStats* st = Sw[w];
    int32_t* z = reinterpret_cast<int32_t*>(st);
    for (int i = l; i < 3 * kSaoStatsInts; i += 64) z[i] = 0;
    wsync();
    if (t.final_action == ACT_P || t.final_action == ACT_I) {
        for (int i = l; i < kCtbSamples; i += 64) {
            int c, x, y;
            if (!ctb_sample(A, i, cx, cy, &c, &x, &y)) continue;
            const SaoPlane pl = sao_plane_of(A, c);
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
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const FrameArgs& f = A.f;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= A.cw * A.ch * kSaoMd) return;
    const int idx = t / kSaoMd, j = t - idx * kSaoMd, cx = idx % A.cw;
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
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ long long md[kPcMaxRowCtb * kSaoMd];
    __shared__ SaoParams own[kPcMaxRowCtb];
    __shared__ long long cost[kPcMaxRowCtb];
    __shared__ uint16_t sel[kPcMaxRowCtb];
    __shared__ uint8_t fl[kPcMaxRowCtb];
    const FrameArgs& f = A.f;
    const int cy = blockIdx.x, l = threadIdx.x, W = A.cw;
    const size_t o = (size_t)cy * W;
    const SliceMap m = smap(A);
    for (int i = l; i < W * kSaoMd; i += 64) md[i] = A.sao_md[o * kSaoMd + i];
    for (int i = l; i < W; i += 64) {
        own[i] = A.sao_own[o + i];
        cost[i] = A.sao_cost[o + i];
        fl[i] = sao_row_flags(m, cy, i);
    }
    __syncthreads();
    if (l == 0) {   // the decision chain is sequential along the row
        const SliceTask t = ctb_task(A, cy);
        sao_row_decide(md, own, cost, W, t.qp, fl, sel);
    }
    __syncthreads();
    for (int x = l; x < W; x += 64) sao_row_apply_sel(own, sel[x], A.sao + o + x);
}

__device__ __forceinline__ bool sao_any(const SaoParams& p) { return (p.type[0] | p.type[1] | p.type[2]) != 0; }

// The filter (8.7.3) of the CTBs SAO changes, from the deblocked picture into sao_tmp:
// one wave per CTB; k_hevc_sao_copy then writes those CTBs back (after every CTB has
// read its deblocked neighbours).
__global__ __launch_bounds__(256) void k_hevc_sao_apply(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= A.cw * A.ch) return;
    const SaoParams p = A.sao[idx];
    if (!sao_any(p)) return;
    const int cx = idx % A.cw, cy = idx / A.cw;
    for (int i = lane(); i < kCtbSamples; i += 64) {
        int c, x, y;
        if (!ctb_sample(A, i, cx, cy, &c, &x, &y)) continue;
        const int stride = c ? f.stride_c : f.stride_y;
        plane_of(A.sao_tmp, c)[(size_t)y * stride + x] =
            (uint8_t)sao_apply_sample(p, c, sao_plane_of(A, c), plane_of(f.rec, c), stride, x, y);
    }
}
__global__ __launch_bounds__(256) void k_hevc_sao_copy(HevcArgs A) {
    const FrameArgs& f = A.f;
    const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (idx >= A.cw * A.ch) return;
    if (!sao_any(A.sao[idx])) return;
    const int cx = idx % A.cw, cy = idx / A.cw;
    Planes rec = f.rec;
    for (int i = lane(); i < kCtbSamples; i += 64) {
        int c, x, y;
        if (!ctb_sample(A, i, cx, cy, &c, &x, &y)) continue;
        const size_t o = (size_t)y * (c ? f.stride_c : f.stride_y) + x;
        plane_of(rec, c)[o] = plane_of(A.sao_tmp, c)[o];
    }
}

// CU coding, deblocking, SAO decisions and the CABAC substreams: everything the coded
// size depends on (the K10 guard re-runs it, gated).
static void launch_code(const HevcArgs& a, hipStream_t s) {
    const int n = a.f.mb_w * a.f.mb_h, nc = a.cw * a.ch;   // units, CTBs
    hipLaunchKernelGGL(k_hevc_inter, dim3(nc), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_intra_prep, dim3((n + 3) / 4), dim3(256), 0, s, a);
    if (a.rps <= 4)
        hipLaunchKernelGGL(k_hevc_intra<4>, dim3(a.f.num_slices), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_hevc_intra<15>, dim3(a.f.num_slices), dim3(64 * 15), 0, s, a);
    const int slots = a.ch * a.seg_k;   // substream slots (SliceMap)
    if (a.seg_k > 1) hipLaunchKernelGGL(k_hevc_intra_seg, dim3((slots + 3) / 4), dim3(256), 0, s, a);
    // in-loop deblocking, then the SAO decisions on the deblocked picture (CTB syntax)
    const int cw = a.f.mb_w, ch = a.f.mb_h;
    const int nv = ch * 4 * (2 * cw - 1) + 2 * ch * 8 * (cw - 1), nh = (2 * ch - 1) * cw * 4 + 2 * (ch - 1) * cw * 8;
    if (nv > 0) hipLaunchKernelGGL(k_hevc_dbk_v, dim3((nv + 255) / 256), dim3(256), 0, s, a);
    if (nh > 0) hipLaunchKernelGGL(k_hevc_dbk_h, dim3((nh + 255) / 256), dim3(256), 0, s, a);
    const int nq = (n + 3) / 4, ncq = (nc + 3) / 4;
    hipLaunchKernelGGL(k_hevc_sao_stats, dim3(ncq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sao_md, dim3((nc * kSaoMd + 255) / 256), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sao_row, dim3(a.ch), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_hevc_bins, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_sort, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sync, dim3(a.f.num_slices), dim3(192), 0, s, a);
    hipLaunchKernelGGL(k_pc_model, dim3(a.ch, (CTX_COUNT + 3) / 4, sk_min(a.seg_k, kPcModelZ)), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_rmap, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_compose, dim3(slots), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_pc_code, dim3(nq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_pc_merge, dim3(slots), dim3(64), 0, s, a);
}

void launch_backend(const HevcArgs& a, hipStream_t s, int* redo) {
    const int nc = a.cw * a.ch;
    launch_code(a, s);
    if (redo) {   // K10 CBR per-frame cap: payload = the substream bytes (as k_rc_account)
        HevcArgs b = a;
        b.f.gate = redo;
        for (int r = 0; r < h264::rc_max_recodes(1); r++) {
            h264::gpu::launch_rc_guard_sizes(a.f, a.sub_size, a.ch * a.seg_k, redo, r > 0, s);
            launch_code(b, s);
        }
    }
    hipLaunchKernelGGL(k_hevc_hdr, dim3(a.f.num_slices), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_hevc_ep_copy, dim3(a.ch * a.seg_k), dim3(64), 0, s, a);
    // the SAO output becomes the reconstruction (k_commit copies it into the reference)
    const int ncq = (nc + 3) / 4;
    hipLaunchKernelGGL(k_hevc_sao_apply, dim3(ncq), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_hevc_sao_copy, dim3(ncq), dim3(256), 0, s, a);
}

}  // namespace gpu
}  // namespace hevc
}  // namespace sk
