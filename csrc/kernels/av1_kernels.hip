// gfx950 (CDNA4) kernels of the AV1 back end (codec/av1_core.h semantics, bit-exact
// with the CPU reference codec/av1_cpu.cpp):
//   k_av1_setup        frame type (any intra slice -> key frame) and qindex
//   k_av1_intra_modes  key frames: open-loop intra mode per block, one wave per 16x16 unit
//   k_av1_intra_rec    key frames: reconstruction wavefront, one workgroup per tile (intra
//                      prediction never crosses a tile edge), anti-diagonal steps x + y
//   k_av1_inter        inter frames: motion compensation (8-tap / 4-tap sub-pel chroma),
//                      transform, quantisation, reconstruction, one wave per unit
//   k_av1_merge        inter frames: static 32x32 / 64x64 merging, one wave per superblock
//   k_av1_modes        inter frames: reference-MV stack -> NEAREST / NEAR / GLOBAL / NEWMV
//   k_av1_tokens       block syntax -> token lists, one wave per 16x16 unit (coefficients lane-parallel)
//   k_av1_tok_scan/copy  per-tile token streams in coding order
//   k_av1_cdf          CDF adaptation, 16 context partitions per tile in parallel ->
//                      per-symbol interval words
//   k_av1_ec_map/link/emit/bytes  the arithmetic coder, parallel over token blocks:
//                      speculative rng per block (128 candidate states), block chaining,
//                      big-integer accumulation of low, carries -> host-mapped tile bytes
//   k_av1_lf           in-loop deblocking (codec/av1_lf.h), one launch per plane and pass
//   k_av1_cdef         CDEF (codec/av1_cdef.h), one wave per 8x8, from a copy of the deblocked picture
//   k_av1_finish       padding rows of the reconstruction, slice actions for k_commit
// Transforms: forward DCT as LDS matrix products (lanes = output coefficients),
// inverse as the normative butterflies, lane = row / column of a transform block.
#include <cstring>
#include <vector>

#include "av1_gpu.h"

namespace sk {
namespace av1 {
namespace gpu {

using h264::ACT_I;
using h264::ACT_NONE;
using h264::ACT_P;
using h264::ACT_SKIPALL;
using h264::SliceTask;
using h264::gpu::FrameArgs;

__device__ __forceinline__ int lane() { return threadIdx.x & 63; }
// K10 per-frame cap: the coding kernels run a second time, gated, after k_rc_guard_sizes
// (f.gate = the re-code flag); they return at once unless the frame overflowed.
__device__ __forceinline__ bool second_pass_skipped(const FrameArgs& f) { return f.gate && *f.gate == 0; }
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

// Forward DCT bases in LDS: [0] 4-point at 0, 8-point at 16, 16-point at 80.
struct FdctLds {
    int16_t k[16 + 64 + 256];
};
__device__ __forceinline__ const int16_t* fdct_k(const FdctLds& F, int log2n) {
    return F.k + (log2n == 2 ? 0 : (log2n == 3 ? 16 : 80));
}
__device__ __forceinline__ void load_fdct(FdctLds& F) {
    for (int i = threadIdx.x; i < 336; i += blockDim.x) {
        const int log2n = i < 16 ? 2 : (i < 80 ? 3 : 4);
        const int base = log2n == 2 ? 0 : (log2n == 3 ? 16 : 80);
        const int n = 1 << log2n, j = i - base;
        F.k[i] = (int16_t)fdct_basis(log2n, j / n, j % n);
    }
}

// One block's working set: luma n x n at 0, U at 256, V at 320 (raster per plane).
struct BlkLds {
    uint8_t src[384];
    uint8_t pred[384];
    int32_t a[384];
    int32_t b[384];
    int16_t lv[384];     // quantised levels (raster per plane) before tail trimming
    int16_t lv2[384];    // IDTX levels of the same residual (the transform-type decision)
    long long jreg;      // intra: the luma J of the cheaper transform type (palette decision)
    IntraEdge e[3];      // intra edges of Y, U, V
};
// Tile of a unit position (mi r, c).
__device__ __forceinline__ TileRect tile_of(const Av1Geo& g, int r, int c) {
    const int tc = (c >> 4) / g.tile_w_sb, tr = (r >> 4) / g.tile_h_sb;
    return tile_rect(g, tr * g.tile_cols + tc);
}

__device__ __forceinline__ long long wsum64(long long v) {
    int lo = (int)(v & 0xffffffffll), hi = (int)(v >> 32);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const unsigned lo2 = (unsigned)__shfl_xor(lo, o), hi2 = (unsigned)__shfl_xor(hi, o);
        const unsigned long long a = ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
        const unsigned long long b = ((unsigned long long)hi2 << 32) | lo2;
        const unsigned long long c = a + b;
        lo = (int)(unsigned)c;
        hi = (int)(c >> 32);
    }
    return (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// Tail trimming of levels lv (raster, n = 1 << ln), lanes over scan positions
// l + 64 k (av1_core.h trim_tail): nonzero masks by ballot, each lane's previous
// nonzero scan position from them, the cut at the last level trim_keep keeps
// (wave-uniform; -1: nothing kept). apply: zero the levels past the cut.
__device__ int trim_cut_wave(int16_t* lv, int ln, bool apply) {
    const int l = lane(), nn2 = 1 << (2 * ln), nw = (nn2 + 63) >> 6;
    uint64_t mk[4];
    int lvk[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int sidx = l + 64 * k;
        lvk[k] = k < nw && sidx < nn2 ? (int)lv[default_scan(ln, sidx)] : 0;
        mk[k] = __ballot(lvk[k] != 0);
    }
    int cut = -1, last_before = -1;   // last_before: the last non-zero position of the earlier groups
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint64_t below = l ? (mk[k] & ((1ull << l) - 1)) : 0ull;
        const int prev = below ? 64 * k + 63 - __builtin_clzll(below) : last_before;
        const uint64_t keep = __ballot(lvk[k] != 0 && trim_keep(lvk[k], l + 64 * k, prev));
        if (keep) cut = 64 * k + 63 - __builtin_clzll(keep);
        if (mk[k]) last_before = 64 * k + 63 - __builtin_clzll(mk[k]);
    }
    if (apply)
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int sidx = l + 64 * k;
            if (k < nw && sidx < nn2 && sidx > cut && lvk[k]) lv[default_scan(ln, sidx)] = 0;
        }
    return cut;
}

// Rate (half bits, av1_core.h tx_bits2 / tx_eob_bits2) of levels lv (raster, n = 1 << ln).
__device__ int rate2_wave(const int16_t* lv, int ln) {
    const int l = lane(), nn2 = 1 << (2 * ln), nw = (nn2 + 63) >> 6;
    int lvk[4], eob = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int sidx = l + 64 * k;
        lvk[k] = k < nw && sidx < nn2 ? (int)lv[default_scan(ln, sidx)] : 0;
        const uint64_t m = __ballot(lvk[k] != 0);
        if (m) eob = 64 * k + 64 - __builtin_clzll(m);
    }
    int r = 0;
#pragma unroll
    for (int k = 0; k < 4; k++)
        if (l + 64 * k < eob) r += tx_bits2(lvk[k]);
    return wsum(r) + tx_eob_bits2(eob);
}

// Transform, quantisation and reconstruction of one block held in L (src, pred):
// luma n = 1 << log2n, chroma n / 2. The transform type is DCT_DCT or IDTX by RD cost
// (the CPU encoder's quant_block rule: inter blocks over the three planes, intra blocks
// luma only, chroma DCT_DCT). Writes levels to gl (3 planes), the reconstruction into
// L.pred, and returns the per-plane level summaries (cul | dc << 6) packed as bytes
// 0..2, bit 24 = any nonzero, bit 25 = IDTX.
__device__ uint32_t code_block_wave(BlkLds& L, const FdctLds& F, int log2n, int qidx, bool intra, int16_t* gy,
                                    int16_t* gu, int16_t* gv) {
    const int l = lane();
    const int n = 1 << log2n, nn = n * n, cn = n >> 1, cnn = cn * cn;
    const int qd = dc_q(qidx), qa = ac_q(qidx);
    // plane p element i: luma [0, nn), U [256, 256 + cnn), V [320, 320 + cnn)
    auto base = [&](int p) { return p == 0 ? 0 : (p == 1 ? 256 : 320); };
    int e2 = 0;   // the residual's SSE: J of coding nothing (inter RD skip)
    for (int p = 0; p < 3; p++) {
        const int m = p ? cnn : nn, o = base(p);
        for (int i = l; i < m; i += 64) {
            const int e = (int)L.src[o + i] - (int)L.pred[o + i];
            L.a[o + i] = e;
            e2 += e * e;
        }
    }
    const long long jz = 256ll * wsum(e2);
    wsync();
    // forward stage 1 (columns): b[k][j] = (sum_m K[k][m] a[m][j] + 512) >> 10
    for (int p = 0; p < 3; p++) {
        const int ln = p ? log2n - 1 : log2n, sz = 1 << ln, o = base(p);
        const int16_t* K = fdct_k(F, ln);
        for (int i = l; i < sz * sz; i += 64) {
            const int k = i >> ln, j = i & (sz - 1);
            int s = 0;
            for (int m2 = 0; m2 < sz; m2++) s += (int)K[k * sz + m2] * L.a[o + m2 * sz + j];
            L.b[o + i] = (s + 512) >> 10;
        }
    }
    wsync();
    // forward stage 2 (rows) + quantisation, DCT levels to L.lv and IDTX levels (8 x the
    // residual, still in L.a) to L.lv2, with both squared coefficient errors per plane
    // transform type: J per plane (av1_core.h tx_rd_cost) summed over the decision planes
    long long jd = 0, ji = 0;
    const int np = intra ? 1 : 3;   // planes in the decision
    for (int p = 0; p < 3; p++) {
        const int ln = p ? log2n - 1 : log2n, sz = 1 << ln, o = base(p);
        const int16_t* K = fdct_k(F, ln);
        long long ed = 0, ei = 0;
        for (int i = l; i < sz * sz; i += 64) {
            const int k = i >> ln, lc = i & (sz - 1);
            // |sum| <= |t|_2 |K|_2 < 2^31 (orthonormal Q13 rows, |t| <= 8 * 255 * sqrt(N)):
            // the 32-bit sum equals av1_core.h fwd_transform's 64-bit one
            int s = 0;
            for (int j = 0; j < sz; j++) s += L.b[o + k * sz + j] * (int)K[lc * sz + j];
            const int32_t c = (s + (s >= 0 ? 4096 : 4095)) >> 13;
            const int q = i == 0 ? qd : qa;
            const int lv = quantize(c, q, intra);
            L.lv[o + i] = (int16_t)lv;
            const long long e = (long long)c - dequant(lv, q);
            ed += e * e;
            if (p < np) {
                const int32_t ci = 8 * L.a[o + i];
                const int li = quantize(ci, q, intra);
                L.lv2[o + i] = (int16_t)li;
                const long long e2 = (long long)ci - dequant(li, q);
                ei += e2 * e2;
            }
        }
        const long long dp = wsum64(ed), ip = wsum64(ei);
        if (p < np) {
            wsync();   // the plane's levels, for the rate estimates
            jd += tx_rd_cost(4 * dp, rate2_wave(L.lv + o, ln), qa);
            ji += tx_rd_cost(4 * ip, rate2_wave(L.lv2 + o, ln), qa);
        }
    }
    wsync();
    // intra: the luma J of the cheaper transform type, through LDS (an out-pointer kept jd /
    // ji live across the inter kernel too: 256 VGPRs, occupancy 1)
    if (intra && l == 0) L.jreg = jd < ji ? jd : ji;
    bool idtx;
    {
        if (intra) {
            // luma keeps a level under IDTX
            int anyl = 0;
            for (int i = l; i < nn; i += 64) anyl |= L.lv2[i];
            idtx = ji < jd && __ballot(anyl != 0) != 0;
        } else {
            // IDTX only where the DCT codes something and the luma keeps levels after trimming
            bool dct_codes = false;
            for (int p = 0; p < 3; p++) dct_codes |= trim_cut_wave(L.lv + base(p), p ? log2n - 1 : log2n, false) >= 0;
            idtx = dct_codes && ji < jd && trim_cut_wave(L.lv2, log2n, false) >= 0;
        }
    }
    wsync();
    if (idtx)
        for (int p = 0; p < np; p++) {
            const int m = p ? cnn : nn, o = base(p);
            for (int i = l; i < m; i += 64) L.lv[o + i] = L.lv2[o + i];
        }
    // inter RD skip (av1_cpu.cpp inter_block): nothing coded when the levels do not pay
    if (!intra && jz <= (idtx ? ji : jd))
        for (int p = 0; p < 3; p++) {
            const int m = p ? cnn : nn, o = base(p);
            for (int i = l; i < m; i += 64) L.lv[o + i] = 0;
        }
    wsync();
    // inter blocks: tail trimming of the chosen levels
    if (!intra)
        for (int p = 0; p < 3; p++) trim_cut_wave(L.lv + base(p), p ? log2n - 1 : log2n, true);
    wsync();
    // dequantisation, level summaries
    int nzm = 0;
    uint32_t cul = 0;
    for (int p = 0; p < 3; p++) {
        const int ln = p ? log2n - 1 : log2n, sz = 1 << ln, o = base(p);
        int16_t* g = p == 0 ? gy : (p == 1 ? gu : gv);
        int sum = 0, nz = 0, first = 0;
        for (int i = l; i < sz * sz; i += 64) {
            const int q = i == 0 ? qd : qa;
            const int lv = L.lv[o + i];
            g[i] = (int16_t)lv;
            if (i == 0) first = lv;
            sum += lv < 0 ? -lv : lv;
            nz |= lv;
            L.a[o + i] = dequant(lv, q);
        }
        sum = wsum(sum);
        const bool any = __ballot(nz != 0) != 0;
        if (any) nzm |= 1 << p;
        const int lv0 = __shfl(first, 0);
        const int dc = lv0 < 0 ? 1 : (lv0 > 0 ? 2 : 0);
        const uint32_t summ = any ? (uint32_t)(sk_min(sum, 63) | (dc << 6)) : 0u;
        cul |= summ << (8 * p);
    }
    wsync();
    // inverse: rows (lane = row of one plane's block), then columns
    const int rows_y = n, rows_c = cn;
    {
        const int p = l < rows_y ? 0 : (l < rows_y + rows_c ? 1 : (l < rows_y + 2 * rows_c ? 2 : 3));
        if (p < 3) {
            const int ln = p ? log2n - 1 : log2n, sz = 1 << ln, o = base(p);
            const int i = p == 0 ? l : (p == 1 ? l - rows_y : l - rows_y - rows_c);
            const int rs = ln == 2 ? 0 : (ln == 3 ? 1 : 2);
            int32_t t[16];
#pragma unroll
            for (int j = 0; j < 16; j++) t[j] = j < sz ? L.a[o + i * sz + j] : 0;
            if (idtx && p < np)
#pragma unroll
                for (int j = 0; j < 16; j++) t[j] = iidentity(t[j], ln);
            else if (ln == 2) idct4(t);
            else if (ln == 3) idct8(t);
            else idct16(t);
#pragma unroll
            for (int j = 0; j < 16; j++)
                if (j < sz) {
                    const int32_t v = rs ? (t[j] + (1 << (rs - 1))) >> rs : t[j];
                    L.b[o + i * sz + j] = sk_clip(v, -32768, 32767);
                }
        }
    }
    wsync();
    {
        const int p = l < rows_y ? 0 : (l < rows_y + rows_c ? 1 : (l < rows_y + 2 * rows_c ? 2 : 3));
        if (p < 3) {
            const int ln = p ? log2n - 1 : log2n, sz = 1 << ln, o = base(p);
            const int j = p == 0 ? l : (p == 1 ? l - rows_y : l - rows_y - rows_c);
            int32_t t[16];
#pragma unroll
            for (int i = 0; i < 16; i++) t[i] = i < sz ? L.b[o + i * sz + j] : 0;
            if (idtx && p < np)
#pragma unroll
                for (int i = 0; i < 16; i++) t[i] = iidentity(t[i], ln);
            else if (ln == 2) idct4(t);
            else if (ln == 3) idct8(t);
            else idct16(t);
#pragma unroll
            for (int i = 0; i < 16; i++)
                if (i < sz) {
                    const int k = o + i * sz + j;
                    L.pred[k] = (uint8_t)sk_clip255((int)L.pred[k] + ((t[i] + 8) >> 4));
                }
        }
    }
    wsync();
    return cul | (nzm ? (1u << 24) : 0u) | (idtx && nzm ? (1u << 25) : 0u);   // no levels: DCT_DCT
}

// Block loads / stores (luma n at (x, y); chroma n/2 at (x/2, y/2)).
__device__ __forceinline__ void load_src_blk(BlkLds& L, const FrameArgs& f, int x, int y, int n) {
    const int l = lane(), cn = n >> 1;
    for (int i = l; i < n * n; i += 64) L.src[i] = f.src.y[(size_t)(y + i / n) * f.stride_y + x + i % n];
    for (int i = l; i < 2 * cn * cn; i += 64) {
        const int p = i / (cn * cn), j = i % (cn * cn);
        const uint8_t* P = p ? f.src.v : f.src.u;
        L.src[(p ? 320 : 256) + j] = P[(size_t)((y >> 1) + j / cn) * f.stride_c + (x >> 1) + j % cn];
    }
}
__device__ __forceinline__ void store_rec_blk(const BlkLds& L, const FrameArgs& f, int x, int y, int n) {
    const int l = lane(), cn = n >> 1;
    for (int i = l; i < n * n; i += 64) f.rec.y[(size_t)(y + i / n) * f.stride_y + x + i % n] = L.pred[i];
    for (int i = l; i < 2 * cn * cn; i += 64) {
        const int p = i / (cn * cn), j = i % (cn * cn);
        uint8_t* P = p ? f.rec.v : f.rec.u;
        P[(size_t)((y >> 1) + j / cn) * f.stride_c + (x >> 1) + j % cn] = L.pred[(p ? 320 : 256) + j];
    }
}

// Motion-compensated prediction of an n x n block (§7.11.3.4 without scaling), separably
// through LDS (every sample of the block shares the filter phases): the (n + 7)^2 reference
// window into win (bytes), the horizontal pass into h (ints, (n + 7) rows x n), the vertical
// pass into out (pitch n): h = (sum_tt tap * ref + 4) >> 3, out = clip((sum_rr tap * h + 1024)
// >> 11). P: plane; (px0, py0): the block in the plane; mv in 1/8 luma pel; ss: chroma shift;
// f4: 4-tap filters (blocks 4 wide / high).
__device__ void mc_block(const uint8_t* P, int stride, int last_x, int last_y, int px0, int py0, int n, int mv_row,
                         int mv_col, int ss, int f4, uint8_t* win, int* h, uint8_t* out) {
    const int l = lane();
    const int dx = (2 * mv_col) >> ss, dy = (2 * mv_row) >> ss;
    const int fx = dx & 15, fy = dy & 15, ix0 = px0 + (dx >> 4), iy0 = py0 + (dy >> 4);
    if (fx == 0 && fy == 0) {
        for (int i = l; i < n * n; i += 64)
            out[i] = P[(size_t)sk_clip(iy0 + i / n, 0, last_y) * stride + sk_clip(ix0 + i % n, 0, last_x)];
        return;
    }
    const int wn = n + 7;
    for (int i = l; i < wn * wn; i += 64) {
        const int r = i / wn, c = i - r * wn;
        win[i] = P[(size_t)sk_clip(iy0 - 3 + r, 0, last_y) * stride + sk_clip(ix0 - 3 + c, 0, last_x)];
    }
    wsync();
    for (int i = l; i < wn * n; i += 64) {
        const int r = i / n, c = i - r * n;
        const uint8_t* w = win + r * wn + c;
        int s1 = 0;
#pragma unroll
        for (int tt = 0; tt < 8; tt++) s1 += subpel_tap(f4, fx, tt) * (int)w[tt];
        h[i] = (s1 + 4) >> 3;
    }
    wsync();
    for (int i = l; i < n * n; i += 64) {
        const int r = i / n, c = i - r * n;
        int s2 = 0;
#pragma unroll
        for (int rr = 0; rr < 8; rr++) s2 += subpel_tap(f4, fy, rr) * h[(r + rr) * n + c];
        out[i] = (uint8_t)sk_clip255((s2 + 1024) >> 11);
    }
    wsync();
}

// Per-block side outputs: cells and level contexts.
__device__ __forceinline__ void set_cells(const Av1Args& A, int r, int c, int bsl, const BlkInfo& b) {
    const int n8 = (1 << bsl) >> 1;
    for (int i = lane(); i < n8 * n8; i += 64) {
        const int ry = (r >> 1) + i / n8, cx = (c >> 1) + i % n8;
        if (ry < A.geo.r8 && cx < A.geo.c8) A.blk[(size_t)ry * A.geo.c8 + cx] = b;
    }
}
__device__ __forceinline__ void set_lctx(const Av1Args& A, int p, int x4, int y4, int n4, uint8_t v) {
    const int W = A.lctx_w[p], H = p ? A.geo.mi_rows >> 1 : A.geo.mi_rows;
    for (int i = lane(); i < n4 * n4; i += 64) {
        const int yy = y4 + i / n4, xx = x4 + i % n4;
        if (yy < H && xx < W) A.lctx[p][(size_t)yy * W + xx] = v;
    }
}
__device__ __forceinline__ int16_t* lev_ptr(const Av1Args& A, int r, int c, int bsl, int p) {
    int16_t* u = A.lev + ((size_t)(r >> 2) * A.f.mb_w + (c >> 2)) * kLevPerUnit;
    if (bsl >= 2) return u + (p == 0 ? 0 : (p == 1 ? 256 : 320));
    const int k = ((r >> 1) & 1) * 2 + ((c >> 1) & 1);
    return u + (p == 0 ? 64 * k : (p == 1 ? 256 + 16 * k : 320 + 16 * k));
}

// Blocks of a unit: one 16x16 (returns -1), or the inside 8x8s in Z order at frame edges
// (returns their count; 0 outside the frame). unit_block: the k-th of them (no arrays:
// dynamically indexed private arrays would live in scratch).
__device__ __forceinline__ int unit_blocks(const Av1Geo& g, int ur, int uc) {
    const int r = ur * 4, c = uc * 4;
    if (r >= g.mi_rows || c >= g.mi_cols) return 0;
    if (r + 2 < g.mi_rows && c + 2 < g.mi_cols) return -1;
    int n = 0;
    for (int q = 0; q < 4; q++) n += (r + (q >> 1) * 2 < g.mi_rows && c + (q & 1) * 2 < g.mi_cols) ? 1 : 0;
    return n;
}
__device__ __forceinline__ void unit_block(const Av1Geo& g, int ur, int uc, int k, int& r, int& c) {
    r = ur * 4;
    c = uc * 4;
    int n = 0;
    for (int q = 0; q < 4; q++) {
        const int rr = ur * 4 + (q >> 1) * 2, cc = uc * 4 + (q & 1) * 2;
        if (rr < g.mi_rows && cc < g.mi_cols) {
            if (n == k) {
                r = rr;
                c = cc;
            }
            n++;
        }
    }
}

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_av1_setup(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const FrameArgs& f = A.f;
    const int ns = f.num_slices;
    bool key = false;
    for (int s = threadIdx.x; s < ns; s += 256) key |= f.tasks[s].final_action == ACT_I;
    key = __syncthreads_or(key);
    if (key)
        for (int s = threadIdx.x; s < ns; s += 256) {
            f.tasks[s].final_action = ACT_I;
            f.tasks_host[s].final_action = ACT_I;
        }
    if (threadIdx.x == 0) {
        // K10: the frame's fractional QP under CRF / CBR (slices dither on H.264 / HEVC)
        const int qidx = f.rc->mode == h264::RC_CQP ? A.qidx_of_qp[sk_clip(f.tasks[0].qp, 0, 51)]
                                                    : frame_qidx(A.qidx_of_qp, f.rc->cur_qpf);
        const int lvl = lf_level_for(ac_q(qidx), key);   // av1_lf.h, the host encoder's choice
        A.frame[0] = key;
        A.frame[1] = qidx;
        A.frame[2] = lvl;
        A.frame_host[0] = key;
        A.frame_host[1] = qidx;
        A.frame_host[2] = lvl;
    }
}

// Key frames: intra mode per block from the source edges (one wave per unit).
__global__ __launch_bounds__(256) void k_av1_intra_modes(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ IntraEdge E[4];
    __shared__ uint32_t pal_seen[4][8];
    __shared__ uint8_t pal_map[4][256], pal_col[4][8];
    if (!A.frame[0]) return;
    const FrameArgs& f = A.f;
    const Av1Geo& g = A.geo;
    const int w = threadIdx.x >> 6, l = lane();
    const int u = blockIdx.x * 4 + w;
    if (u >= f.mb_w * f.mb_h) return;
    const int ux = u % f.mb_w, uy = u / f.mb_w;
    int nb = unit_blocks(g, uy, ux);
    const int bsl = nb < 0 ? 2 : 1;
    if (nb < 0) nb = 1;
    for (int k = 0; k < nb; k++) {
        int r, c;
        unit_block(g, uy, ux, k, r, c);
        const int log2n = bsl + 2, n = 1 << log2n;
        const TileRect t = tile_of(g, r, c);
        const bool au = inside(t, r - 1, c), al = inside(t, r, c - 1);
        if (l == 0) intra_edges(f.src.y, f.stride_y, c * 4, r * 4, n, au, al, g.mi_cols * 4 - 1, g.mi_rows * 4 - 1, E[w]);
        wsync();
        const int dc = intra_dc(E[w], log2n);
        const uint8_t cand[7] = {DC_PRED, V_PRED, H_PRED, SMOOTH_PRED, SMOOTH_V_PRED, SMOOTH_H_PRED, PAETH_PRED};
        int best = DC_PRED, best_cost = 1 << 30;
        for (int m = 0; m < 7; m++) {
            int sad = 0;
            for (int i = l; i < n * n; i += 64) {
                const int pr = cand[m] == DC_PRED ? dc : intra_pred_px(E[w], cand[m], log2n, i / n, i % n);
                sad += sk_abs((int)f.src.y[(size_t)(r * 4 + i / n) * f.stride_y + c * 4 + i % n] - pr);
            }
            sad = wsum(sad);
            const int cost = sad + (cand[m] == DC_PRED ? 0 : n * 2);
            if (cost < best_cost) {
                best_cost = cost;
                best = cand[m];
            }
        }
        BlkInfo b{};
        b.bsl = (uint8_t)bsl;
        b.mode = (uint8_t)best;
        b.uv_mode = DC_PRED;
        // palette candidate (source only, so decided here in parallel rather than in the
        // reconstruction wavefront): the block's distinct luma values, its colours into
        // the palette cells, palette_rate2 for k_av1_intra_rec's RD comparison
        if (A.palette && r + (1 << bsl) <= g.mi_rows && c + (1 << bsl) <= g.mi_cols) {
            uint32_t* seen = pal_seen[w];
            uint8_t* map = pal_map[w];
            uint8_t* col = pal_col[w];
            if (l < 8) seen[l] = 0u;
            wsync();
            for (int i = l; i < n * n; i += 64) {
                const int v = f.src.y[(size_t)(r * 4 + i / n) * f.stride_y + c * 4 + i % n];
                atomicOr(&seen[v >> 5], 1u << (v & 31));
            }
            wsync();
            const int k = wsum(l < 8 ? __builtin_popcount(seen[l]) : 0);
            if (k >= 2 && k <= kPalMax) {
                if (l == 0) {
                    int q = 0;
                    for (int v = 0; v < 256; v++)
                        if ((seen[v >> 5] >> (v & 31)) & 1) col[q++] = (uint8_t)v;
                    for (; q < 8; q++) col[q] = 0;
                }
                wsync();
                for (int i = l; i < n * n; i += 64)
                    map[i] = (uint8_t)palette_index(col, k, f.src.y[(size_t)(r * 4 + i / n) * f.stride_y + c * 4 + i % n]);
                wsync();
                int r2 = 0;
                for (int i = l; i < n * n; i += 64) r2 += palette_rate2_px(map, n, i / n, i % n, k);
                r2 = wsum(r2) + palette_rate2_head(k);
                const int n8 = (1 << bsl) >> 1;
                for (int i = l; i < n8 * n8 * 8; i += 64) {
                    const int cell = i >> 3, ry = (r >> 1) + cell / n8, cx = (c >> 1) + cell % n8;
                    A.pal[((size_t)ry * g.c8 + cx) * 8 + (i & 7)] = col[i & 7];
                }
                if (l == 0) A.pal_rate[(size_t)(r >> 1) * g.c8 + (c >> 1)] = r2;
                b.pad1 = (uint8_t)k;
            }
            wsync();
        }
        set_cells(A, r, c, bsl, b);
        wsync();
    }
}

// Reconstruction of one intra block (mode from the cells) by one wave.
__device__ void intra_rec_block(const Av1Args& A, BlkLds& L, const FdctLds& F, int r, int c, int bsl, int qidx) {
    const FrameArgs& f = A.f;
    const Av1Geo& g = A.geo;
    const int l = lane(), log2n = bsl + 2, n = 1 << log2n, cn = n >> 1;
    const int x = c * 4, y = r * 4;
    const TileRect t = tile_of(g, r, c);
    const bool au = inside(t, r - 1, c), al = inside(t, r, c - 1);
    BlkInfo b = A.blk[(size_t)(r >> 1) * g.c8 + (c >> 1)];
    IntraEdge* E = L.e;
    if (l == 0) {
        intra_edges(f.rec.y, f.stride_y, x, y, n, au, al, g.mi_cols * 4 - 1, g.mi_rows * 4 - 1, E[0]);
        intra_edges(f.rec.u, f.stride_c, x >> 1, y >> 1, cn, au, al, g.mi_cols * 2 - 1, g.mi_rows * 2 - 1, E[1]);
        intra_edges(f.rec.v, f.stride_c, x >> 1, y >> 1, cn, au, al, g.mi_cols * 2 - 1, g.mi_rows * 2 - 1, E[2]);
    }
    load_src_blk(L, f, x, y, n);
    wsync();
    const int dcy = intra_dc(E[0], log2n), dcu = intra_dc(E[1], log2n - 1), dcv = intra_dc(E[2], log2n - 1);
    for (int i = l; i < n * n; i += 64)
        L.pred[i] = (uint8_t)(b.mode == DC_PRED ? dcy : intra_pred_px(E[0], b.mode, log2n, i / n, i % n));
    for (int i = l; i < cn * cn; i += 64) {
        L.pred[256 + i] = (uint8_t)dcu;
        L.pred[320 + i] = (uint8_t)dcv;
    }
    wsync();
    uint32_t s = code_block_wave(L, F, log2n, qidx, true, lev_ptr(A, r, c, bsl, 0), lev_ptr(A, r, c, bsl, 1),
                                 lev_ptr(A, r, c, bsl, 2));
    const long long jreg = L.jreg;
    b.tx_type = (int16_t)((s >> 25) & 1 ? TX_IDTX : TX_DCT_DCT);
    // palette candidate from k_av1_intra_modes (colours already in the palette cells):
    // exact palette of the source luma vs the transform path (av1_cpu.cpp intra_block)
    const int kc = b.pad1;
    b.pad1 = 0;
    b.pal_n = 0;
    if (kc && tx_rd_cost(0, A.pal_rate[(size_t)(r >> 1) * g.c8 + (c >> 1)], ac_q(qidx)) < jreg) {
        b.pal_n = (uint8_t)kc;
        b.mode = DC_PRED;
        b.tx_type = TX_DCT_DCT;
        int16_t* gy = lev_ptr(A, r, c, bsl, 0);
        for (int i = l; i < n * n; i += 64) {
            gy[i] = 0;
            L.pred[i] = L.src[i];
        }
        s &= ~0xffu;   // no luma levels: the summary and the skip flag come from chroma
        s = (s & ~(1u << 24)) | ((s & 0xffff00u) ? (1u << 24) : 0u);
        wsync();
    }
    store_rec_blk(L, f, x, y, n);
    b.flags = (s >> 24) & 1 ? 0 : 2;
    set_cells(A, r, c, bsl, b);
    const int n4 = 1 << bsl;
    set_lctx(A, 0, c, r, n4, (uint8_t)(s & 0xff));
    set_lctx(A, 1, c >> 1, r >> 1, n4 >> 1, (uint8_t)((s >> 8) & 0xff));
    set_lctx(A, 2, c >> 1, r >> 1, n4 >> 1, (uint8_t)((s >> 16) & 0xff));
    wsync();
}

// Key frames: one workgroup (16 waves) per tile; unit (x, y) of the tile at step x + y.
__global__ __launch_bounds__(1024) void k_av1_intra_rec(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ BlkLds Lw[16];
    __shared__ FdctLds F;
    if (!A.frame[0]) return;
    const Av1Geo& g = A.geo;
    const int t = blockIdx.x;
    const TileRect tr = tile_rect(g, t);
    load_fdct(F);
    __syncthreads();
    const int w = threadIdx.x >> 6;
    const int ux0 = tr.mi_col0 >> 2, uy0 = tr.mi_row0 >> 2;
    const int uw = (tr.mi_col1 - tr.mi_col0 + 3) >> 2, uh = (tr.mi_row1 - tr.mi_row0 + 3) >> 2;
    const int qidx = A.frame[1];
    const int steps = uw + uh - 1;
    for (int s = 0; s < steps; s++) {
        for (int y = w; y < uh; y += 16) {
            const int x = s - y;
            if (x < 0 || x >= uw) continue;
            int nb = unit_blocks(g, uy0 + y, ux0 + x);
            const int bsl = nb < 0 ? 2 : 1;
            if (nb < 0) nb = 1;
            for (int k = 0; k < nb; k++) {
                int r, c;
                unit_block(g, uy0 + y, ux0 + x, k, r, c);
                intra_rec_block(A, Lw[w], F, r, c, bsl, qidx);
            }
        }
        __syncthreads();
    }
}

// Inter frames: one wave per unit, vector from the front end's motion search.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_av1_inter(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ BlkLds Lw[4];
    __shared__ FdctLds F;
    if (A.frame[0]) return;
    const FrameArgs& f = A.f;
    const Av1Geo& g = A.geo;
    load_fdct(F);
    __syncthreads();
    const int w = threadIdx.x >> 6, l = lane();
    const int u = blockIdx.x * 4 + w;
    if (u >= f.mb_w * f.mb_h) return;
    BlkLds& L = Lw[w];
    const int ux = u % f.mb_w, uy = u / f.mb_w;
    const SliceTask t = f.tasks[uy / f.rows_per_slice];
    const h264::MeResult me = f.me[u];
    const bool moving = t.final_action == ACT_P;
    const int mv_row = moving ? 8 * me.mvy : 0, mv_col = moving ? 8 * me.mvx : 0;
    const int qidx = A.frame[1];
    int nb = unit_blocks(g, uy, ux);
    const int bsl = nb < 0 ? 2 : 1;
    if (nb < 0) nb = 1;
    const int lxc = ((g.W + 1) >> 1) - 1, lyc = ((g.H + 1) >> 1) - 1;
    for (int k = 0; k < nb; k++) {
        int r, c;
        unit_block(g, uy, ux, k, r, c);
        const int log2n = bsl + 2, n = 1 << log2n, cn = n >> 1;
        const int x = c * 4, y = r * 4;
        load_src_blk(L, f, x, y, n);
        // prediction (mc_block: window in L.lv, horizontal pass in L.a; both free until
        // code_block_wave)
        uint8_t* win = reinterpret_cast<uint8_t*>(L.lv);
        mc_block(f.ref.y, f.stride_y, g.W - 1, g.H - 1, x, y, n, mv_row, mv_col, 0, n <= 4, win, L.a, L.pred);
        mc_block(f.ref.u, f.stride_c, lxc, lyc, x >> 1, y >> 1, cn, mv_row, mv_col, 1, cn <= 4, win, L.a, L.pred + 256);
        mc_block(f.ref.v, f.stride_c, lxc, lyc, x >> 1, y >> 1, cn, mv_row, mv_col, 1, cn <= 4, win, L.a, L.pred + 320);
        wsync();
        const uint32_t s = code_block_wave(L, F, log2n, qidx, false, lev_ptr(A, r, c, bsl, 0),
                                           lev_ptr(A, r, c, bsl, 1), lev_ptr(A, r, c, bsl, 2));
        store_rec_blk(L, f, x, y, n);
        BlkInfo b{};
        b.bsl = (uint8_t)bsl;
        b.flags = (uint8_t)(1 | ((s >> 24) & 1 ? 0 : 2));
        b.tx_type = (int16_t)((s >> 25) & 1 ? TX_IDTX : TX_DCT_DCT);
        b.mv_row = (int16_t)mv_row;
        b.mv_col = (int16_t)mv_col;
        b.mode = GLOBALMV;
        set_cells(A, r, c, bsl, b);
        const int n4 = 1 << bsl;
        set_lctx(A, 0, c, r, n4, (uint8_t)(s & 0xff));
        set_lctx(A, 1, c >> 1, r >> 1, n4 >> 1, (uint8_t)((s >> 8) & 0xff));
        set_lctx(A, 2, c >> 1, r >> 1, n4 >> 1, (uint8_t)((s >> 16) & 0xff));
        wsync();
    }
}

// Static merging per superblock: lane = 8x8 cell of the SB (8 x 8 cells).
__global__ __launch_bounds__(64) void k_av1_merge(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    if (A.frame[0]) return;
    const Av1Geo& g = A.geo;
    const int sb = blockIdx.x, sr = sb / g.sb_cols, sc = sb % g.sb_cols;
    const int l = lane(), cy = sr * 8 + (l >> 3), cx = sc * 8 + (l & 7);
    const bool in = cy < g.r8 && cx < g.c8;
    for (int lvl = 3; lvl <= 4; lvl++) {
        const int sz = 1 << lvl, half = sz >> 1, cells = sz >> 1;
        // region of this lane
        const int r = (cy & ~(cells - 1)) * 2, c = (cx & ~(cells - 1)) * 2;
        // the merged block lies inside the picture (no partially outside 32x32 / 64x64)
        const bool fits = r + sz <= g.mi_rows && c + sz <= g.mi_cols;
        const BlkInfo b0 = A.blk[(size_t)(r >> 1) * g.c8 + (c >> 1)];
        const BlkInfo me = in ? A.blk[(size_t)cy * g.c8 + cx] : b0;
        const bool ok_me = !in || (blk_skip(me) && me.mv_row == b0.mv_row && me.mv_col == b0.mv_col);
        // all lanes of the region must agree: reduce over the region's lanes
        const uint64_t bad = __ballot(!ok_me);
        uint64_t mask = 0;
        for (int k = 0; k < 64; k++) {
            const int ky = sr * 8 + (k >> 3), kx = sc * 8 + (k & 7);
            if ((ky & ~(cells - 1)) * 2 == r && (kx & ~(cells - 1)) * 2 == c) mask |= 1ull << k;
        }
        wsync();
        if (fits && !(bad & mask) && in) {
            BlkInfo m = b0;
            m.bsl = (uint8_t)lvl;
            A.blk[(size_t)cy * g.c8 + cx] = m;
        }
        wsync();
        __threadfence_block();
    }
}

// Inter modes from the MV stack: one lane per 8x8 cell, block origins only.
__global__ __launch_bounds__(256) void k_av1_modes(Av1Args A) {
    __shared__ MvStack stk[256];
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    if (A.frame[0]) return;
    const Av1Geo& g = A.geo;
    const int cell = blockIdx.x * 256 + threadIdx.x;
    if (cell >= g.c8 * g.r8) return;
    const int y8 = cell / g.c8, x8 = cell % g.c8;
    const BlkInfo b = A.blk[cell];
    const int n8 = (1 << b.bsl) >> 1;
    if ((y8 & (n8 - 1)) || (x8 & (n8 - 1))) return;
    const int r = y8 * 2, c = x8 * 2;
    const TileRect t = tile_of(g, r, c);
    MvStack& s = stk[threadIdx.x];   // LDS: a per-lane stack indexed at run time would live in scratch
    const BlkGrid grid{A.blk, g.c8};
    find_mv_stack(s, grid, t, g.mi_rows, g.mi_cols, r, c, b.bsl, DecodedBefore{r, c});
    int mode, idx = 0;
    if (b.mv_row == 0 && b.mv_col == 0) mode = GLOBALMV;
    else if (b.mv_row == s.mv[0][0] && b.mv_col == s.mv[0][1]) mode = NEARESTMV;
    else if (s.n >= 2 && b.mv_row == s.mv[1][0] && b.mv_col == s.mv[1][1]) {
        mode = NEARMV;
        idx = 1;
    } else mode = NEWMV;
    for (int yy = 0; yy < n8; yy++)
        for (int xx = 0; xx < n8; xx++)
            if (y8 + yy < g.r8 && x8 + xx < g.c8) {
                BlkInfo& d = A.blk[(size_t)(y8 + yy) * g.c8 + x8 + xx];
                d.mode = (uint8_t)mode;
                d.flags = (uint8_t)((d.flags & 0x0f) | (idx << 4));
            }
}

// Block syntax -> tokens, one wave per 16x16 unit. The syntax above the coefficients
// (partitions, modes, vectors) is short and runs wave-uniform (lane 0 stores); the
// coefficients of every transform block are tokenised lane-parallel by the
// WaveTokenSink overload of code_coeffs below.
struct WaveTokenSink {
    uint32_t* p;
    int n, cap;
    uint32_t pend;
    int pend_n;
    uint32_t* bits;   // this wave's LDS bit buffer (256 words) for the sign / Golomb run
    __device__ __forceinline__ void push(uint32_t t) {
        if (n < cap && lane() == 0) p[n] = t;
        n++;
    }
    __device__ __forceinline__ void flush() {
        if (pend_n) push(tok_lit(pend, pend_n));
        pend = 0;
        pend_n = 0;
    }
    __device__ __forceinline__ void sym(int off, int n2, int v) {
        flush();
        push(tok_sym(off, n2, v));
    }
    __device__ __forceinline__ void bit(int b) {
        pend = (pend << 1) | (uint32_t)(b & 1);
        if (++pend_n == 24) flush();
    }
    __device__ __forceinline__ void lits(uint32_t v, int nbits) {
        for (int i = nbits - 1; i >= 0; i--) bit((v >> i) & 1);
    }
    __device__ __forceinline__ void gather(int off, bool bottom_out, int v) {
        flush();
        push(tok_gather(off, bottom_out, v));
    }
};

// Number of coeff_br tokens of a level magnitude a (code_coeffs: up to 4 groups of 3).
__device__ __forceinline__ int br_count(int a) {
    if (a <= 2) return 0;
    int level = 3, k = 0;
    for (int idx = 0; idx < 4; idx++) {
        const int br = sk_min(a - level, 3);
        k++;
        level += br;
        if (br < 3) break;
    }
    return k;
}

// Lane-parallel code_coeffs (codec/av1_core.h): the same tokens in the same order.
// Every coefficient's base / range contexts depend only on the level array (its
// neighbours lie on later anti-diagonals, already coded in the reverse scan), so lanes
// take scan positions s = l + 64 k, place their tokens by a suffix sum over the reverse
// scan, and pack the forward-scan sign / Golomb bits through LDS into 24-bit literals.
__device__ __forceinline__ int code_coeffs_regs(WaveTokenSink& w, const CdfContext& cx, const int16_t* lev, int txs,
                                                int plane, CoefCtx cc, bool is_inter, int intra_dir, int qidx,
                                                int tx_type) {
    const int l = lane();
    const int log2n = txs + 2, n = 1 << log2n, nn = n * n, nw = (nn + 63) >> 6;
    const int ptype = plane > 0;
    int lv[4], pos[4];
    int eob = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int sidx = l + 64 * k;
        pos[k] = k < nw && sidx < nn ? default_scan(log2n, sidx) : 0;
        lv[k] = k < nw && sidx < nn ? (int)lev[pos[k]] : 0;
        const uint64_t m = __ballot(lv[k] != 0);
        if (m) eob = 64 * k + 64 - __builtin_clzll(m);
    }
    w.sym(cdf_off(cx, cx.txb_skip[txs][cc.txb_skip]), 2, eob == 0);
    if (eob == 0) return 0;
    if (plane == 0 && qidx > 0) {
        const int sym = tx_type == TX_IDTX ? 0 : 1;
        if (is_inter) w.sym(cdf_off(cx, cx.inter_tx_set3[txs]), 2, sym);
        else w.sym(cdf_off(cx, cx.intra_tx_set2[txs][intra_dir]), 5, sym);
    }
    const int eob_multi = 2 * log2n - 4;
    const int eob_pt = eob_pt_of(eob);
    switch (eob_multi) {
        case 0: w.sym(cdf_off(cx, cx.eob_pt_16[ptype][0]), 5, eob_pt - 1); break;
        case 2: w.sym(cdf_off(cx, cx.eob_pt_64[ptype][0]), 7, eob_pt - 1); break;
        default: w.sym(cdf_off(cx, cx.eob_pt_256[ptype][0]), 9, eob_pt - 1); break;
    }
    if (eob_pt >= 3) {
        const int off = eob - ((1 << (eob_pt - 2)) + 1);
        const int sh = eob_pt - 3;
        w.sym(cdf_off(cx, cx.eob_extra[txs][ptype][eob_pt - 3]), 2, (off >> sh) & 1);
        for (int i = 1; i < eob_pt - 2; i++) w.bit((off >> (sh - i)) & 1);
    }
    w.flush();   // the coefficient symbols follow (each sym flushes; keep n exact for the offsets)
    // ---- base levels + ranges, reverse scan: tokens of position s at n + (tokens of s' > s)
    int cnt[4], tot = 0, hi[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int sidx = l + 64 * k;
        cnt[k] = sidx < eob ? 1 + br_count(lv[k] < 0 ? -lv[k] : lv[k]) : 0;
    }
    // suffix sums: chunk totals (uniform), then within a chunk the lanes above
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        int x = cnt[k];   // inclusive suffix scan over lanes (lane 63 first)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_down(x, o);
            if (l + o < 64) x += y;
        }
        hi[k] = tot + x - cnt[k];   // tokens of chunks above + lanes above in this chunk
        tot += __shfl(x, 0);
    }
    auto qv = [&](int rr, int c2) -> int {   // min(level, 15) of a later-coded neighbour (0 outside)
        if (rr >= n || c2 >= n) return 0;
        const int a = sk_abs((int)lev[(rr << log2n) + c2]);
        return a < 15 ? a : 15;
    };
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int c = l + 64 * k;
        if (c >= eob) continue;
        const int a = sk_abs(lv[k]), pz = pos[k];
        const int row = pz >> log2n, col = pz & (n - 1);
        int o = w.n + hi[k];
        uint32_t t;
        if (c == eob - 1) {
            const int ctx = c == 0 ? 0 : (c <= nn / 8 ? 1 : (c <= nn / 4 ? 2 : 3));
            t = tok_sym(cdf_off(cx, cx.coeff_base_eob[txs][ptype][ctx]), 3, sk_min(a, 3) - 1);
        } else {
            int mag = sk_min(qv(row, col + 1), 3) + sk_min(qv(row + 1, col), 3) + sk_min(qv(row + 1, col + 1), 3) +
                      sk_min(qv(row, col + 2), 3) + sk_min(qv(row + 2, col), 3);
            int ctx = sk_min((mag + 1) >> 1, 4);
            if (row == 0 && col == 0) ctx = 0;
            else {
                const int rm = sk_min(row, 4), cm = sk_min(col, 4);
                int ofs;
                if (txs == TX_4X4) {
                    constexpr uint8_t t4[5][5] = {{0, 1, 6, 6, 0}, {1, 6, 6, 21, 0}, {6, 6, 21, 21, 0},
                                                  {6, 21, 21, 21, 0}, {0, 0, 0, 0, 0}};
                    ofs = t4[rm][cm];
                } else {
                    constexpr uint8_t t8[5][5] = {{0, 1, 6, 6, 21}, {1, 6, 6, 21, 21}, {6, 6, 21, 21, 21},
                                                  {6, 21, 21, 21, 21}, {21, 21, 21, 21, 21}};
                    ofs = t8[rm][cm];
                }
                ctx += ofs;
            }
            t = tok_sym(cdf_off(cx, cx.coeff_base[txs][ptype][ctx]), 4, sk_min(a, 3));
        }
        if (o < w.cap) w.p[o] = t;
        o++;
        if (a > 2) {
            int mag = qv(row, col + 1) + qv(row + 1, col) + qv(row + 1, col + 1);
            mag = sk_min((mag + 1) >> 1, 6);
            const int ctx = pz == 0 ? mag : ((row < 2 && col < 2) ? mag + 7 : mag + 14);
            const int cdf = cdf_off(cx, cx.coeff_br[sk_min(txs, TX_32X32)][ptype][ctx]);
            int level = 3;
            for (int idx = 0; idx < 4; idx++) {
                const int br = sk_min(a - level, 3);
                if (o < w.cap) w.p[o] = tok_sym(cdf, 4, br);
                o++;
                level += br;
                if (br < 3) break;
            }
        }
    }
    w.n += tot;
    // ---- signs and Golomb remainders, forward scan: dc_sign symbol, then one bit run
    const int l0 = (int)lev[0];
    if (l0 != 0) w.sym(cdf_off(cx, cx.dc_sign[ptype][cc.dc_sign]), 2, l0 < 0);
    int nb[4], bsum = 0, cul = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int c = l + 64 * k, a = sk_abs(lv[k]);
        nb[k] = 0;
        if (c < eob && a) {
            nb[k] = c > 0 ? 1 : 0;
            if (a > 14) nb[k] += 2 * (31 - __builtin_clz((uint32_t)(a - 14))) + 1;
            cul += a;
        }
    }
    for (int i = l; i < 256; i += 64) w.bits[i] = 0u;
    wsync();
    int base = 0, boff[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {   // exclusive prefix over the forward scan
        int x = nb[k];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (l >= o) x += y;
        }
        boff[k] = base + x - nb[k];
        base += __shfl(x, 63);
    }
    bsum = base;
    auto put_bits = [&](int off, uint32_t v, int cntb) {   // cntb <= 32 bits, MSB first, at bit offset off
        for (int i = 0; i < cntb; i++)
            if ((v >> (cntb - 1 - i)) & 1) atomicOr(&w.bits[(off + i) >> 5], 0x80000000u >> ((off + i) & 31));
    };
#pragma unroll
    for (int k = 0; k < 4; k++) {
        if (!nb[k]) continue;
        const int a = sk_abs(lv[k]), c = l + 64 * k;
        int off = boff[k];
        if (c > 0) {
            put_bits(off, lv[k] < 0 ? 1u : 0u, 1);
            off++;
        }
        if (a > 14) {
            const uint32_t x = (uint32_t)(a - 14);
            const int len = 31 - __builtin_clz(x);
            off += len;                          // len zero bits
            put_bits(off, x, len + 1);           // the leading one and the len low bits
        }
    }
    wsync();
    // 24-bit literal tokens, the remainder stays pending (flushed by the next symbol)
    const int full = bsum / 24, rem = bsum - 24 * full;
    auto chunk = [&](int start, int cntb) -> uint32_t {
        uint32_t v = 0;
        for (int i = 0; i < cntb; i++) v = (v << 1) | ((w.bits[(start + i) >> 5] >> (31 - ((start + i) & 31))) & 1u);
        return v;
    };
    for (int j = l; j < full; j += 64) {
        const int o = w.n + j;
        if (o < w.cap) w.p[o] = tok_lit(chunk(24 * j, 24), 24);
    }
    w.n += full;
    w.pend = rem ? chunk(24 * full, rem) : 0u;
    w.pend_n = rem;
    wsync();
    const int dcc = l0 == 0 ? 0 : (l0 < 0 ? 1 : 2);
    return sk_min(wsum(cul), 63) | (dcc << 6);
}

// code_coeffs is too large to inline at its nine call sites, and a sink passed by
// reference to a call lives in scratch memory (on both sides of the call). The call takes
// the sink by value and returns it, so it stays in registers in the caller and the callee.
struct SinkResult {
    WaveTokenSink w;
    int r;
};
__device__ __noinline__ SinkResult code_coeffs_call(WaveTokenSink w, const CdfContext& cx, const int16_t* lev, int txs,
                                                    int plane, CoefCtx cc, bool is_inter, int intra_dir, int qidx,
                                                    int tx_type) {
    const int r = code_coeffs_regs(w, cx, lev, txs, plane, cc, is_inter, intra_dir, qidx, tx_type);
    return SinkResult{w, r};
}
__device__ __forceinline__ int code_coeffs(WaveTokenSink& w, const CdfContext& cx, const int16_t* lev, int txs, int plane,
                                           CoefCtx cc, bool is_inter, int intra_dir, int qidx, int tx_type = TX_DCT_DCT) {
    const SinkResult res = code_coeffs_call(w, cx, lev, txs, plane, cc, is_inter, intra_dir, qidx, tx_type);
    w = res.w;
    return res.r;
}

// Lane-parallel palette_tokens (codec/av1_core.h code_palette_tokens): every sample's
// colour context depends only on the index map, so lanes rank their samples at once and
// store each token at its anti-diagonal position.
__device__ void code_palette_tokens(WaveTokenSink& w, const CdfContext& cx, const FrameView& v, int r, int c, int bsl,
                                    int k) {
    const int l = lane(), n = 4 << bsl;
    const uint8_t* col = v.pal_at(r, c);
    uint8_t* map = (uint8_t*)w.bits;   // the wave's LDS bit buffer (1 KB), unused here
    for (int i = l; i < n * n; i += 64)
        map[i] = (uint8_t)palette_index(col, k, v.src_y[(size_t)(r * 4 + i / n) * v.stride_y + c * 4 + i % n]);
    wsync();
    code_ns(w, k, map[0]);
    w.flush();
    for (int i = l; i < n * n; i += 64) {
        if (i == 0) continue;
        const int y = i / n, x = i % n, d = x + y;
        // samples before (y, x) in the scan: the diagonals before d, then the ones of d
        // with a larger column (the scan runs j from the top-right end down)
        const int before = d < n ? d * (d + 1) / 2 : n * n - (2 * n - 1 - d) * (2 * n - d) / 2;
        const int jmax = d < n ? d : n - 1;
        const int o = w.n + before + (jmax - x) - 1;
        uint32_t order;
        const int ctx = palette_color_context(map, n, y, x, k, &order);
        if (o < w.cap) w.p[o] = tok_sym(cdf_off(cx, cx.palette_y_color[k - 2][ctx]), k, palette_rank(order, k, map[i]));
    }
    w.n += n * n - 1;
    wsync();
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_av1_tokens(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ uint32_t bits_w[4][256];
    __shared__ MvStack stk_w[4];
    const int w = threadIdx.x >> 6;
    const int u = blockIdx.x * 4 + w;
    const FrameArgs& f = A.f;
    if (u >= f.mb_w * f.mb_h) return;
    const Av1Geo& g = A.geo;
    FrameView v;
    v.stk = &stk_w[w];
    v.geo = g;
    v.blk = A.blk;
    v.lev = A.lev;
    for (int p = 0; p < 3; p++) {
        v.lctx[p] = A.lctx[p];
        v.lctx_w[p] = A.lctx_w[p];
    }
    v.unit_w = f.mb_w;
    v.qidx = A.frame[1];
    v.key = A.frame[0];
    v.screen = A.frame[0] && A.palette;
    v.pal = A.pal;
    v.src_y = f.src.y;
    v.stride_y = f.stride_y;
    const int ux = u % f.mb_w, uy = u / f.mb_w;
    WaveTokenSink sink{A.tok + (size_t)u * kTokCap, 0, kTokCap, 0u, 0, bits_w[w]};
    const TileRect t = tile_of(g, uy * 4, ux * 4);
    code_unit(sink, AV1_DEFAULT_CDF[0], v, t, ux, uy);
    sink.flush();
    if (lane() == 0) A.tok_n[u] = sink.n;
}

// Tile token streams: the unit slots of each tile concatenated in coding order, so
// the coder reads one contiguous stream. k_av1_tok_scan: per-unit offsets (one
// workgroup per tile, block scan); k_av1_tok_copy: one wave per unit.
__global__ __launch_bounds__(256) void k_av1_tok_scan(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ int wsum_s[4];
    __shared__ int run_s;
    const Av1Geo& g = A.geo;
    const int t = blockIdx.x, tid = threadIdx.x, l = lane(), w = tid >> 6;
    const TileRect tr = tile_rect(g, t);
    const int U = tile_units(tr);
    if (tid == 0) run_s = 0;
    __syncthreads();
    for (int b0 = 0; b0 < U; b0 += 256) {
        const int i = b0 + tid;
        int u = -1, cnt = 0, ux, uy;
        if (i < U) {
            tile_unit(g, tr, i, &ux, &uy);
            if (ux * 4 < g.mi_cols && uy * 4 < g.mi_rows) {
                u = uy * A.f.mb_w + ux;
                cnt = sk_min(A.tok_n[u], kTokCap);
            }
        }
        int x = cnt;   // inclusive wave scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (l >= o) x += y;
        }
        if (l == 63) wsum_s[w] = x;
        __syncthreads();
        int pre = run_s;
        for (int k = 0; k < w; k++) pre += wsum_s[k];
        if (u >= 0) A.tok_off[u] = pre + x - cnt;
        __syncthreads();
        if (tid == 0) run_s += wsum_s[0] + wsum_s[1] + wsum_s[2] + wsum_s[3];
        __syncthreads();
    }
    if (tid == 0) A.tile_ntok[t] = run_s;
}

__global__ __launch_bounds__(256) void k_av1_tok_copy(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const Av1Geo& g = A.geo;
    const int u = blockIdx.x * 4 + (threadIdx.x >> 6), l = lane();
    if (u >= A.f.mb_w * A.f.mb_h) return;
    const int ux = u % A.f.mb_w, uy = u / A.f.mb_w;
    const int t = (uy / 4 / g.tile_h_sb) * g.tile_cols + ux / 4 / g.tile_w_sb;
    const int n = sk_min(A.tok_n[u], kTokCap);
    const uint32_t* s = A.tok + (size_t)u * kTokCap;
    uint32_t* d = A.tokc + (size_t)t * A.tile_tok_cap + A.tok_off[u];
    for (int i = l; i < n; i += 64) d[i] = s[i];
}

// Entropy coding in two phases.
//
// k_av1_cdf (phase A): the CDF adaptation, parallel over contexts. Each tile's CDF
// slots are split over kEcParts waves by a hash of the slot offset; every wave scans
// the tile's whole token stream in 64-token batches, takes the symbols of its own
// contexts in order (ballot + find-first-set) and, with the tile's CDFs in its LDS,
// adapts them lane-parallel (lane i: cdf[i], lane N: the counter). Per symbol it
// writes the interval word the coder needs:
//   [9:0] (32768 - cdf[s]) >> 6 (0 for the last symbol)   [19:10] (32768 - cdf[s-1]) >> 6
//   [24:20] N - s   [25] s > 0
// Literal tokens are copied as their own word (bits 31:30 = 01).
// Phase B (k_av1_ec_*, below k_av1_cdf): the arithmetic coder over the interval words
// and literal bits, parallel over token blocks. Bit-exact with SymbolCoder (av1_ec.h).
constexpr int kEcParts = 16;

__device__ __forceinline__ uint32_t sgpr(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, i); }
__device__ __forceinline__ int ec_owner(uint32_t off) { return (int)((off * 0x9E3779B1u) >> 28) & (kEcParts - 1); }
__device__ __forceinline__ uint32_t ec_word(uint32_t clo, uint32_t chi, int n, int s) {
    const uint32_t fh = s < n - 1 ? (32768u - chi) >> kProbShift : 0u;
    const uint32_t fl = s > 0 ? (32768u - clo) >> kProbShift : 0u;
    return fh | fl << 10 | (uint32_t)(n - s) << 20 | (s > 0 ? 1u << 25 : 0u);
}

// Tokens per compaction chunk: 16 loads per lane in flight, then this wave's tokens of
// the chunk (about 1 / kEcParts of them, plus the literals for partition 0) in LDS.
constexpr int kChunk = 1024;

// update_cdf of one CDF entry in one dependent step: towards 32768 (target 32768) or
// towards 0 (target (1 << rate) - 1, which makes the arithmetic shift round the way
// c - (c >> rate) does); equal to both forms for every c in [0, 32768].
__device__ __forceinline__ int cdf_step(int c, int target, int rate) { return c + ((target - c) >> rate); }

__global__ __launch_bounds__(64) void k_av1_cdf(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ CdfContext cx;
    __shared__ uint32_t wst[64];     // words of the gathered booleans of the sub-batch
    __shared__ uint16_t cap[64][66]; // per token of the sub-batch: the CDF row before its update (padded: conflict-free column reads)
    __shared__ uint32_t ctok[kChunk], cpos[kChunk];   // this wave's tokens of the chunk, in order, and their stream positions
    const int t = blockIdx.x / kEcParts, part = blockIdx.x % kEcParts, L = threadIdx.x;
    {
        const uint16_t* src = (const uint16_t*)&AV1_DEFAULT_CDF[coef_qctx(A.frame[1])];
        uint16_t* d16 = (uint16_t*)&cx;
        for (int i = L; i < (int)(sizeof(CdfContext) / 2); i += 64) d16[i] = src[i];
    }
    __syncthreads();
    uint16_t* cdfs = (uint16_t*)&cx;
    const int ntok = A.tile_ntok[t], last = A.tile_tok_cap - 1;
    const uint32_t* tk = A.tokc + (size_t)t * A.tile_tok_cap;
    uint32_t* pw = A.pw + (size_t)t * A.tile_tok_cap;
    // The CDF of the context adapted last stays in a register (lane j: cdf[j]; its
    // counter and adaptation rate in scalars) and goes back to LDS only when another
    // context comes up: the hot contexts (the zero-level context of 16x16 luma blocks
    // can be half of a tile's symbols) adapt in registers with no LDS round trip. The
    // serial loop does only what the next symbol depends on - the lane-parallel update
    // of the row - and leaves the row it started from in cap[token]; the interval words
    // are built after the loop, one lane per token. Every wave first compacts its own
    // tokens of a chunk (ballot + prefix count), so the serial batches hold only them and
    // each word is stored once, at its stream position.
    // A run of consecutive tokens in the cached context with its counter saturated
    // (`hot`) takes a tight loop with no context or counter checks, and the update is one
    // dependent step per entry (cdf_step).
    int cache_off = -1, cache_n = 0, cnt = 0, rate = 0, rbase = 0;
    uint32_t cache = 0;
    uint32_t hot = ~0u;   // token bits (kind, N, slot) of the cached context once its counter saturated
    auto evict = [&]() {
        if (cache_off >= 0) {
            if (L < cache_n - 1) {
                cdfs[cache_off + L] = (uint16_t)cache;
            } else if (L == cache_n) {
                cdfs[cache_off + L] = (uint16_t)cnt;
            }
        }
        cache_off = -1;
    };
    auto sub = [&](int b, int nown) {   // own tokens b .. b + 63 of the chunk
        const bool valid = b + L < nown;
        const uint32_t tv = valid ? ctok[b + L] : (1u << 30);
        const uint32_t kind = tv >> 30;   // literal tokens are their own word (partition 0's)
        const uint32_t sv = (tv >> 22) & 15;   // the symbol of a symbol token
        uint64_t m = __ballot(valid && kind != 1);
        int i = m ? __builtin_ctzll(m) : 0;
        uint32_t tt = sgpr(rdlane(tv, i));
        while (m) {
            if ((tt & 0xFC3FFFFFu) == hot) {
                // a run of consecutive tokens in the cached context, its counter saturated:
                // a tight loop (no context checks, no counter updates)
                const uint64_t above = __ballot((tv & 0xFC3FFFFFu) == hot) >> i;
                const int e = i + (~above ? __builtin_ctzll(~above) : 64);
                m = e >= 64 ? 0ull : m & (~0ull << e);
                const int lo = (1 << rate) - 1;
                for (int j = i; j < e; j++) {
                    const int sj = (int)sgpr(rdlane(sv, j));
                    cap[j][L] = (uint16_t)cache;
                    cache = (uint32_t)cdf_step((int)cache, L >= sj ? 32768 : lo, rate);
                }
            } else {
                asm volatile("s_bitset0_b64 %0, %1" : "+s"(m) : "s"(i));   // m &= m - 1 in one SALU op
                if ((tt >> 30) == 0) {
                    const int off = (int)(tt & 0x3fffff);
                    const int n = (int)((tt >> 26) & 15) + 1;
                    const int s = (int)((tt >> 22) & 15);
                    if (off != cache_off) {
                        evict();
                        cache_off = off;
                        cache_n = n;
                        rbase = 3 + (n > 3 ? 2 : (n > 1 ? 1 : 0));
                        cache = L <= n ? (uint32_t)cdfs[off + L] : 0u;
                        cnt = (int)sgpr(rdlane(cache, n));
                        rate = (int)sgpr((uint32_t)(rbase + (cnt > 15) + (cnt > 31)));
                    }
                    cap[i][L] = (uint16_t)cache;
                    // update_cdf, branch-free: lanes >= s move towards 32768, the others to 0
                    // (lanes >= N-1 are never written back; the counter lives in cnt)
                    cache = (uint32_t)cdf_step((int)cache, L >= s ? 32768 : (1 << rate) - 1, rate);
                    if (cnt < 32) {
                        cnt++;
                        rate = (int)sgpr((uint32_t)(rbase + (cnt > 15) + (cnt > 31)));
                    }
                } else {   // gathered boolean: reads a partition CDF from LDS
                    evict();
                    uint16_t c2[3];   // split_or_horz / split_or_vert (read-only CDF)
                    gather_partition_cdf(cdfs + (tt & 0x3fffff), ((tt >> 29) & 1) == 0, c2);
                    const uint32_t c0 = sgpr(c2[0]);
                    const int v = (int)((tt >> 28) & 1);
                    if (L == 0) wst[i] = ec_word(c0, v ? 32768u : c0, 2, v);
                }
                hot = sgpr(cache_off >= 0 && cnt >= 32 ? (uint32_t)cache_off | (uint32_t)(cache_n - 1) << 26 : ~0u);
            }
            if (m) {
                i = __builtin_ctzll(m);
                tt = sgpr(rdlane(tv, i));
            }
        }
        wsync();
        uint32_t out = tv;   // literal
        if (kind == 0) {
            const int n = (int)((tv >> 26) & 15) + 1, s = (int)((tv >> 22) & 15);
            const uint32_t chi = s < n - 1 ? (uint32_t)cap[L][s] : 0u, clo = s > 0 ? (uint32_t)cap[L][s - 1] : 0u;
            out = ec_word(clo, chi, n, s);
        } else if (kind != 1) {
            out = wst[L];
        }
        if (valid) pw[cpos[b + L]] = out;
        wsync();
    };
    uint32_t v[kChunk / 64];
    auto load = [&](int c0) {
#pragma unroll
        for (int j = 0; j < kChunk / 64; j++) v[j] = tk[sk_min(c0 + 64 * j + L, last)];
    };
    load(0);
    for (int c0 = 0; c0 < ntok; c0 += kChunk) {
        int nown = 0;
#pragma unroll
        for (int j = 0; j < kChunk / 64; j++) {
            const int i = c0 + 64 * j + L;
            const uint32_t tv = v[j];
            const bool mine = i < ntok && ((tv >> 30) == 1 ? part == 0 : ec_owner(tv & 0x3fffff) == part);
            const uint64_t m = __ballot(mine);
            const int k = nown + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (mine) {
                ctok[k] = tv;
                cpos[k] = (uint32_t)i;
            }
            nown += __builtin_popcountll(m);
        }
        wsync();
        load(c0 + kChunk);   // the next chunk's loads fly during the serial pass
        for (int b = 0; b < nown; b += 64) sub(b, nown);
    }
}

// ---------------------------------------------------------------------------
// Phase B: the arithmetic coder, parallel over token blocks (no per-tile serial pass).
//
// The coder state is (low, rng). rng alone evolves serially, and at every token that
// "resets" it - a symbol with s > 0 (interval bounds u, v from rng >> 8 only) or a
// literal whose first bit is 1 (split from rng >> 8 only) - the next rng depends on
// the 7 bits of rng >> 8 (128 values in [32768, 65535]), not on the whole state.
// low is a sum: symbol i adds a_i = r_i - u_i at bit position P_i = (total shift after
// i), so the tile is one big integer V = sum a_i << P_i, finished as
// V' = ((V + 0x3fff) & ~0x3fff) | 0x4000 and emitted as its top 8N bits with
// N = (D + 8) >> 3 (D = total shift): byte j holds bits [D + 7 - 8j, D + 15 - 8j).
// (Equal to SymbolCoder in codec/av1_ec.h, carries included; tests/test_av1_entropy.py.)
//
//   k_av1_ec_map   blocks of ~kEcBlk tokens, each starting at a resetting token: every
//                  lane runs the block from two candidate states (rng >> 8 = 128 + l and
//                  192 + l) -> per candidate the exit rng and the block's shift count
//   k_av1_ec_link  one wave per tile chains the block maps (LDS-free readlane lookups)
//                  -> each block's true entry rng and shift prefix; tile sizes
//   k_av1_ec_emit  each block re-run from its true entry, scalar state: a_i into V's
//                  64-bit words (coalesced per word, one atomic per word and block)
//   k_av1_ec_bytes per tile: carries of V (carry-lookahead scan), rounding, bytes ->
//                  host-mapped output at the tiles' prefix offsets
constexpr int kEcBlk = 512;      // nominal tokens per block
constexpr int kEcGrid = 1024;    // workgroups (4 waves) of the block-parallel kernels

__device__ __forceinline__ bool ec_resets(uint32_t w) {
    if ((w >> 30) == 1) return (w >> ((w >> 25) & 31)) & 1;   // literal: its first (top) bit
    return (w >> 25) & 1;                                        // symbol: s > 0
}
// Block size of this frame: at least kEcBlk, larger when the frame would need more
// than max_blocks maps. Lane t < tiles: the tile's block count; returns the total,
// incl = inclusive prefix over lanes.
__device__ __forceinline__ int ec_blocks(const Av1Args& A, int tiles, int* bsz, int* incl, int* ntok_l) {
    const int l = lane();
    const int nt = l < tiles ? A.tile_ntok[l] : 0;
    const int tot = wsum(nt);
    int b = kEcBlk;
    const int need = (tot + A.ec_max_blocks - tiles - 1) / sk_max(A.ec_max_blocks - tiles, 1);
    if (need > b) b = (need + 63) & ~63;
    int n = l < tiles ? (nt + b - 1) / b : 0;
    if (l < tiles && n == 0) n = 1;
    int x = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (l >= o) x += y;
    }
    *bsz = b;
    *incl = x;
    *ntok_l = nt;
    return __shfl(x, 63);
}
__device__ int ec_first_reset(const uint32_t* pw, int i, int ntok) {
    for (; i < ntok; i += 64) {
        const int k = i + lane();
        const bool r = k < ntok && ec_resets(pw[k < ntok ? k : 0]);
        const uint64_t m = __ballot(r);
        if (m) return i + __builtin_ctzll(m);
    }
    return ntok;
}
// One symbol / literal bit on a per-lane rng (VALU): returns r2 (before normalisation).
__device__ __forceinline__ uint32_t ec_sym_r2(uint32_t r, uint32_t w) {
    const uint32_t r8 = r >> 8, ns4 = ((w >> 20) & 31) * kMinProb;
    const uint32_t v = ((r8 * (w & 1023)) >> (7 - kProbShift)) + ns4 - kMinProb;
    const uint32_t u = (w >> 25) & 1 ? ((r8 * ((w >> 10) & 1023)) >> (7 - kProbShift)) + ns4 : r;
    return u - v;
}
__device__ __forceinline__ void ec_norm(uint32_t& r, uint32_t& D, uint32_t r2) {
    const uint32_t d = (uint32_t)__builtin_clz(r2) - 16;
    r = r2 << d;
    D += d;
}
__device__ __forceinline__ void ec_step(uint32_t& r, uint32_t& D, uint32_t w) {
    if ((w >> 30) == 1) {
        const int nb = (int)((w >> 25) & 31) + 1;
        for (int k = nb - 1; k >= 0; k--) {
            const uint32_t split = ((r >> 8) << 7) + kMinProb;
            ec_norm(r, D, (w >> k) & 1 ? split : r - split);
        }
    } else {
        ec_norm(r, D, ec_sym_r2(r, w));
    }
}

__global__ __launch_bounds__(256) void k_av1_ec_map(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const int tiles = A.geo.tile_cols * A.geo.tile_rows, l = lane();
    int bsz, incl, ntl;
    const int total = ec_blocks(A, tiles, &bsz, &incl, &ntl);
    const int nw = gridDim.x * 4;
    for (int g = (int)sgpr(blockIdx.x * 4 + (threadIdx.x >> 6)); g < total; g += nw) {
        const int t = __popcll(__ballot(l < tiles && incl <= g));
        const int b = g - (t ? __shfl(incl, t - 1) : 0);
        const int ntok = __shfl(ntl, t);
        const uint32_t* pw = A.pw + (size_t)t * A.tile_tok_cap;
        const int s = b == 0 ? 0 : ec_first_reset(pw, b * bsz, ntok);
        const int e = (b + 1) * bsz >= ntok ? ntok : ec_first_reset(pw, (b + 1) * bsz, ntok);
        if (l == 0) A.ecblk[g] = make_int4(s, e, 0, 0);
        // block 0 starts from the coder's initial state; the others from every candidate
        uint32_t ra = b == 0 ? 0x8000u : (uint32_t)(128 + l) << 8, rb = b == 0 ? 0x8000u : (uint32_t)(192 + l) << 8;
        uint32_t da = 0, db = 0;
        for (int i0 = s; i0 < e; i0 += 64) {
            const uint32_t wv = pw[sk_min(i0 + l, e - 1)];
            const int m = sk_min(64, e - i0);
            for (int j = 0; j < m; j++) {
                const uint32_t w = rdlane(wv, j);
                ec_step(ra, da, w);
                ec_step(rb, db, w);
            }
        }
        uint2* mp = A.ecmap + (size_t)g * 128;
        mp[l] = make_uint2(ra, da);
        mp[64 + l] = make_uint2(rb, db);
    }
}

__global__ __launch_bounds__(64) void k_av1_ec_link(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const int tiles = A.geo.tile_cols * A.geo.tile_rows, l = lane(), t = blockIdx.x;
    int bsz, incl, ntl;
    ec_blocks(A, tiles, &bsz, &incl, &ntl);
    const int g0 = t ? __shfl(incl, t - 1) : 0, nb = __shfl(incl, t) - g0;
    const uint2 m0 = A.ecmap[(size_t)g0 * 128];
    uint32_t r = sgpr(m0.x), D = sgpr(m0.y);
    if (l == 0) {
        A.ecblk[g0].z = 0x8000;
        A.ecblk[g0].w = 0;
    }
    constexpr int kG = 16;   // block maps prefetched per group: lane l holds entries l and 64 + l
    for (int bb = 1; bb < nb; bb += kG) {
        uint2 ma[kG], mb[kG];
        int se = 0;
#pragma unroll
        for (int k = 0; k < kG; k++) {
            const int g = g0 + sk_min(bb + k, nb - 1);
            ma[k] = A.ecmap[(size_t)g * 128 + l];
            mb[k] = A.ecmap[(size_t)g * 128 + 64 + l];
        }
        if (l < kG && bb + l < nb) {
            const int4 bi = A.ecblk[g0 + bb + l];
            se = bi.x < bi.y;
        }
        const uint64_t nonempty = __ballot(se);
#pragma unroll
        for (int k = 0; k < kG; k++) {
            if (bb + k >= nb) continue;
            const int g = g0 + bb + k;
            if (l == 0) {
                A.ecblk[g].z = (int)r;
                A.ecblk[g].w = (int)D;
            }
            if ((nonempty >> k) & 1) {   // empty blocks pass the state through
                const int idx = (int)(r >> 8) - 128;
                const uint32_t er = idx < 64 ? rdlane(ma[k].x, idx) : rdlane(mb[k].x, idx - 64);
                const uint32_t ed = idx < 64 ? rdlane(ma[k].y, idx) : rdlane(mb[k].y, idx - 64);
                r = sgpr(er);
                D = sgpr(D + ed);
            }
        }
    }
    // V: bits [0, D + 48) as 64-bit partial sums of 32-bit digits
    const int nwords = (int)(D >> 5) + 3, nbytes = (int)((D + 8) >> 3);
    const bool fits = nwords <= A.ec_vcap && nbytes <= A.tile_cap;
    if (l == 0) A.tile_bits[t] = fits ? (int)D : -1;
    if (fits) {
        unsigned long long* V = A.ecv + (size_t)t * A.ec_vcap;
        for (int i = l; i < nwords; i += 64) V[i] = 0ull;
    }
}

__global__ __launch_bounds__(256) void k_av1_ec_emit(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    const int tiles = A.geo.tile_cols * A.geo.tile_rows, l = lane();
    int bsz, incl, ntl;
    const int total = ec_blocks(A, tiles, &bsz, &incl, &ntl);
    const int nw = gridDim.x * 4;
    for (int g = (int)sgpr(blockIdx.x * 4 + (threadIdx.x >> 6)); g < total; g += nw) {
        const int t = __popcll(__ballot(l < tiles && incl <= g));
        const int Dt = A.tile_bits[t];
        if (Dt < 0) continue;   // tile over capacity: reported by k_av1_ec_bytes
        const int4 bi = A.ecblk[g];
        const int s = sgpr(bi.x), e = sgpr(bi.y);
        const uint32_t* pw = A.pw + (size_t)t * A.tile_tok_cap;
        unsigned long long* V = A.ecv + (size_t)t * A.ec_vcap;
        uint32_t r = sgpr(bi.z);
        int x = Dt - bi.w;   // bit position of the next add
        x = (int)sgpr((uint32_t)x);
        int cw = 1 << 30;    // word of accA (accB: cw + 1)
        unsigned long long accA = 0, accB = 0;
        auto flush = [&](int w, unsigned long long v) {
            if (v && l == 0) atomicAdd(V + w, v);
        };
        auto put = [&](uint32_t add) {
            const int k = x >> 5;
            const unsigned long long v = (unsigned long long)add << (x & 31);
            if (k != cw) {
                if (k == cw - 1) {
                    flush(cw + 1, accB);
                    accB = accA;
                } else {
                    flush(cw, accA);
                    flush(cw + 1, accB);
                    accB = 0;
                }
                accA = 0;
                cw = k;
            }
            accA += v & 0xffffffffull;
            accB += v >> 32;
        };
        for (int i0 = s; i0 < e; i0 += 64) {
            const uint32_t wv = pw[sk_min(i0 + l, e - 1)];
            const int m = sk_min(64, e - i0);
            for (int j = 0; j < m; j++) {
                const uint32_t w = sgpr(rdlane(wv, j));
                r = sgpr(r);
                x = (int)sgpr((uint32_t)x);
                if ((w >> 30) == 1) {
                    const int nb = (int)((w >> 25) & 31) + 1;
                    for (int k = nb - 1; k >= 0; k--) {
                        const uint32_t split = ((r >> 8) << 7) + kMinProb;
                        uint32_t r2 = r - split;
                        if ((w >> k) & 1) {
                            put(r - split);
                            r2 = split;
                        }
                        const int d = __builtin_clz(r2) - 16;
                        r = r2 << d;
                        x -= d;
                    }
                } else {
                    const uint32_t r8 = r >> 8, ns4 = ((w >> 20) & 31) * kMinProb;
                    const uint32_t v = ((r8 * (w & 1023)) >> (7 - kProbShift)) + ns4 - kMinProb;
                    uint32_t u = r;
                    if ((w >> 25) & 1) {
                        u = ((r8 * ((w >> 10) & 1023)) >> (7 - kProbShift)) + ns4;
                        put(r - u);
                    }
                    const uint32_t r2 = u - v;
                    const int d = __builtin_clz(r2) - 16;
                    r = r2 << d;
                    x -= d;
                }
            }
        }
        flush(cw, accA);
        flush(cw + 1, accB);
    }
}

__global__ __launch_bounds__(256) void k_av1_ec_bytes(Av1Args A) {
    if (second_pass_skipped(A.f)) return;   // K10: no re-code this frame
    __shared__ uint32_t wg_s[4], wp_s[4];
    __shared__ int off_s, carry_s;
    const int t = blockIdx.x, tid = threadIdx.x, l = lane(), w = tid >> 6;
    const int tiles = A.geo.tile_cols * A.geo.tile_rows;
    const int D = A.tile_bits[t];
    if (tid == 0) {
        int off = 0;
        for (int k = 0; k < t; k++) {
            const int dk = A.tile_bits[k];
            off += dk < 0 ? 0 : (dk + 8) >> 3;
        }
        const int n = D < 0 ? -1 : (D + 8) >> 3;
        A.tile_size[t] = n;
        A.out_size_host[t] = (n >= 0 && off + n <= A.out_cap) ? n : -1;
        off_s = off;
        carry_s = 0;
    }
    __syncthreads();
    const int off = off_s;
    if (D < 0 || off + ((D + 8) >> 3) > A.out_cap) return;
    (void)tiles;
    const unsigned long long* V = A.ecv + (size_t)t * A.ec_vcap;
    uint32_t* F = A.ecf + (size_t)t * A.ec_vcap;
    const int nwords = (D >> 5) + 3, N = (D + 8) >> 3;
    // a_k = lo(V_k) + hi(V_k-1) (+ 0x3fff rounding at k = 0) < 2^33; b_k = lo(a_k) + hi(a_k-1) <= 2^32
    auto a_of = [&](int k) -> unsigned long long {
        if (k < 0) return 0ull;
        return (V[k] & 0xffffffffull) + (k ? V[k - 1] >> 32 : 0ull) + (k == 0 ? 0x3fffull : 0ull);
    };
    for (int w0 = 0; w0 < nwords; w0 += 1024) {
        unsigned long long bk[4];
        uint32_t G = 0, P = 1;   // carry generate / propagate over this thread's 4 words
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int k = w0 + 4 * tid + q;
            bk[q] = k < nwords ? (a_of(k) & 0xffffffffull) + (a_of(k - 1) >> 32) : 0ull;
            const uint32_t g = (uint32_t)(bk[q] >> 32), p = bk[q] == 0xffffffffull;
            G = g | (p & G);
            P = P & p;
        }
        // exclusive scan of (G, P) over the workgroup, lower words first
        uint32_t eg = G, ep = P;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t ug = __shfl_up(eg, o), up = __shfl_up(ep, o);
            if (l >= o) {
                eg = eg | (ep & ug);
                ep = ep & up;
            }
        }
        if (l == 63) {
            wg_s[w] = eg;
            wp_s[w] = ep;
        }
        __syncthreads();
        uint32_t c = carry_s;   // carry into wave w's first word
        for (int k = 0; k < w; k++) c = wg_s[k] | (wp_s[k] & c);
        {   // into this thread: the inclusive scan of the lanes below
            const uint32_t pg = __shfl_up(eg, 1), pp = __shfl_up(ep, 1);
            if (l > 0) c = pg | (pp & c);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int k = w0 + 4 * tid + q;
            if (k < nwords) F[k] = (uint32_t)(bk[q] + c);
            c = (uint32_t)((bk[q] + c) >> 32);
        }
        __syncthreads();
        if (tid == 255) carry_s = c;
        __syncthreads();
    }
    if (tid == 0) F[0] = (F[0] & ~0x3fffu) | 0x4000u;
    __syncthreads();
    uint8_t* out = A.out_host + off;
    for (int j = tid; j < N; j += 256) {
        const int p = D + 7 - 8 * j, k = p >> 5;
        const unsigned long long v = (unsigned long long)F[k] | ((unsigned long long)(k + 1 < nwords ? F[k + 1] : 0u) << 32);
        out[j] = (uint8_t)(v >> (p & 31));
    }
}

// Rows below the picture repeat its last row (the reference clamp AV1's MC reads),
// and every slice's reconstruction becomes the reference: static slices (coded as
// zero-motion skips) become ACT_P with zero vectors, so k_commit copies rec -> ref (the
// loop filter and CDEF may have touched their rows) and gives them a zero MV field.
// In-loop deblocking (av1_lf.h lf_edge), one launch per (plane, pass): one thread per
// MI edge position (4 lines), every edge of a pass independent of the others.
__global__ __launch_bounds__(256) void k_av1_lf(Av1Args A, int plane, int pass) {
    const int lvl = A.frame[2];
    if (lvl == 0) return;
    const Av1Geo& g = A.geo;
    const int ss = plane ? 1 : 0;
    const int cols = (g.mi_cols + ss) >> ss, rows = (g.mi_rows + ss) >> ss;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= cols * rows) return;
    const int r = (t / cols) << ss, c = (t % cols) << ss;
    const LfFrame lf{A.blk, g.c8, g.mi_rows, g.mi_cols, g.W, g.H, {lvl, lvl, lvl, lvl}};
    const FrameArgs& f = A.f;
    uint8_t* buf = plane == 0 ? f.rec.y : (plane == 1 ? f.rec.u : f.rec.v);
    lf_edge(lf, plane, pass, r, c, buf, plane ? f.stride_c : f.stride_y);
}

// CDEF (av1_cdef.h): one wave per 8x8 block, lane = luma pixel. The direction's line
// sums are accumulated with LDS atomics (integer, order-independent), lane 0 turns them
// into the direction, then every lane filters its luma pixel and lanes 0..31 the 4x4 Cb /
// Cr pixels, reading the deblocked copy in cdef_in and writing f.rec.
__global__ __launch_bounds__(256) void k_av1_cdef(Av1Args A) {
    __shared__ int part[4][8][15];
    __shared__ int dirvar[4][2];
    __shared__ long long cost[4][8];
    const Av1Geo& g = A.geo;
    const int w = threadIdx.x >> 6, l = lane();
    const int cols = g.mi_cols >> 1, rows = g.mi_rows >> 1;
    const int b = blockIdx.x * 4 + w;
    if (b >= cols * rows) return;   // wave-uniform; no block barriers below
    const int r = (b / cols) * 2, c = (b % cols) * 2;
    const CdefParams p = cdef_choose(A.frame[1], ac_q(A.frame[1]));
    if (!cdef_on(p) || !cdef_sb_on(A.blk, g, r & ~15, c & ~15) || blk_skip(A.blk[(size_t)(r >> 1) * g.c8 + (c >> 1)]))
        return;
    const FrameArgs& f = A.f;
    int* pw = &part[w][0][0];
    for (int k = l; k < 8 * 15; k += 64) pw[k] = 0;
    wsync();
    const int i = l >> 3, j = l & 7;
    const int x = (int)A.cdef_in.y[(size_t)(r * 4 + i) * f.stride_y + c * 4 + j] - 128;
#pragma unroll
    for (int d = 0; d < 8; d++) atomicAdd(&part[w][d][cdef_partial_index(d, i, j)], x);
    wsync();
    if (l < 8) cost[w][l] = cdef_dir_cost(part[w], l);   // one direction per lane
    wsync();
    if (l == 0) {
        int var = 0;
        dirvar[w][0] = cdef_pick_dir(cost[w], &var);
        dirvar[w][1] = var;
    }
    wsync();
    const int ydir = dirvar[w][0], var = dirvar[w][1];
    int pri, dir;
    cdef_luma_setup(p, ydir, var, &pri, &dir);
    const int out = cdef_filter_px(A.cdef_in.y, f.stride_y, 0, c * 4, r * 4, i, j, pri, p.y_sec, p.damping, dir,
                                   g.mi_rows, g.mi_cols);
    f.rec.y[(size_t)(r * 4 + i) * f.stride_y + c * 4 + j] = (uint8_t)out;
    if (l < 32) {   // Cb (lanes 0..15) / Cr (16..31): 4x4 pixel l & 15
        const int pl = l >> 4, ci = (l & 15) >> 2, cj = l & 3;
        const uint8_t* in = pl ? A.cdef_in.v : A.cdef_in.u;
        uint8_t* o = pl ? f.rec.v : f.rec.u;
        const int udir = p.uv_pri == 0 ? 0 : ydir;   // Cdef_Uv_Dir is the identity for 4:2:0
        o[(size_t)(r * 2 + ci) * f.stride_c + c * 2 + cj] = (uint8_t)cdef_filter_px(
            in, f.stride_c, 1, c * 2, r * 2, ci, cj, p.uv_pri, p.uv_sec, p.damping - 1, udir, g.mi_rows, g.mi_cols);
    }
}

__global__ __launch_bounds__(256) void k_av1_finish(Av1Args A) {
    const FrameArgs& f = A.f;
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int H = A.geo.H, Hc = (H + 1) >> 1;
    if (x < f.stride_y)
        for (int y = H; y < f.mb_h * 16; y++) f.rec.y[(size_t)y * f.stride_y + x] = f.rec.y[(size_t)(H - 1) * f.stride_y + x];
    if (x < f.stride_c)
        for (int y = Hc; y < f.mb_h * 8; y++) {
            f.rec.u[(size_t)y * f.stride_c + x] = f.rec.u[(size_t)(Hc - 1) * f.stride_c + x];
            f.rec.v[(size_t)y * f.stride_c + x] = f.rec.v[(size_t)(Hc - 1) * f.stride_c + x];
        }
    if (blockIdx.x == 0)
        for (int s = threadIdx.x; s < f.num_slices; s += 256) {
            const int fa = f.tasks[s].final_action;
            if (fa == ACT_NONE || fa == ACT_SKIPALL) {   // coded as zero-motion skips
                f.tasks[s].final_action = ACT_P;
                f.tasks_host[s].final_action = ACT_P;
                const int j0 = f.tasks[s].first_row * f.mb_w, j1 = j0 + f.tasks[s].num_rows * f.mb_w;
                for (int j = j0; j < j1; j++) f.me[j].mvx = f.me[j].mvy = 0;
            }
        }
}

static void launch_ec(const Av1Args& a, int tiles, hipStream_t s) {
    hipLaunchKernelGGL(k_av1_ec_map, dim3(kEcGrid), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_ec_link, dim3(tiles), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_av1_ec_emit, dim3(kEcGrid), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_ec_bytes, dim3(tiles), dim3(256), 0, s, a);
}

void ec_buffers(int tiles, int tile_bytes, int* max_blocks, int* vcap) {
    *max_blocks = 16384 + tiles;
    *vcap = tile_bytes / 4 + 8;
}

// Block decisions, reconstruction and the arithmetic-coded tiles: everything the coded
// size depends on (the K10 guard re-runs it, gated).
static void launch_code(const Av1Args& a, hipStream_t s) {
    const int n = a.f.mb_w * a.f.mb_h;
    const int tiles = a.geo.tile_cols * a.geo.tile_rows;
    hipLaunchKernelGGL(k_av1_setup, dim3(1), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_intra_modes, dim3((n + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_intra_rec, dim3(tiles), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(k_av1_inter, dim3((n + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_merge, dim3(a.geo.sb_cols * a.geo.sb_rows), dim3(64), 0, s, a);
    hipLaunchKernelGGL(k_av1_modes, dim3((a.geo.c8 * a.geo.r8 + 255) / 256), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_tokens, dim3((n + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_tok_scan, dim3(tiles), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_tok_copy, dim3((n + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_cdf, dim3(tiles * kEcParts), dim3(64), 0, s, a);
    launch_ec(a, tiles, s);
}

void launch_backend(const Av1Args& a, hipStream_t s, int* redo) {
    const int tiles = a.geo.tile_cols * a.geo.tile_rows;
    launch_code(a, s);
    if (redo) {   // K10 CBR per-frame cap: payload = the tile bytes (as k_rc_account)
        Av1Args b = a;
        b.f.gate = redo;
        for (int r = 0; r < h264::rc_max_recodes(2, a.geo.W * a.geo.H); r++) {
            h264::gpu::launch_rc_guard_sizes(a.f, a.tile_size, tiles, redo, r > 0, s);
            launch_code(b, s);
        }
    }
    for (int p = 0; p < 3; p++) {   // in-loop deblocking of the reconstruction, plane by plane
        const int ss = p ? 1 : 0;
        const int cnt = ((a.geo.mi_cols + ss) >> ss) * ((a.geo.mi_rows + ss) >> ss);
        for (int pass = 0; pass < 2; pass++) hipLaunchKernelGGL(k_av1_lf, dim3((cnt + 255) / 256), dim3(256), 0, s, a, p, pass);
    }
    // CDEF reads the deblocked picture: a copy, then the filter writes the reconstruction
    const size_t ny = (size_t)a.f.stride_y * a.f.mb_h * 16, nc = (size_t)a.f.stride_c * a.f.mb_h * 8;
    (void)hipMemcpyAsync(a.cdef_in.y, a.f.rec.y, ny, hipMemcpyDeviceToDevice, s);
    (void)hipMemcpyAsync(a.cdef_in.u, a.f.rec.u, nc, hipMemcpyDeviceToDevice, s);
    (void)hipMemcpyAsync(a.cdef_in.v, a.f.rec.v, nc, hipMemcpyDeviceToDevice, s);
    const int nb8 = (a.geo.mi_cols >> 1) * (a.geo.mi_rows >> 1);
    hipLaunchKernelGGL(k_av1_cdef, dim3((nb8 + 3) / 4), dim3(256), 0, s, a);
    hipLaunchKernelGGL(k_av1_finish, dim3((a.f.stride_y + 255) / 256), dim3(256), 0, s, a);
}

}  // namespace gpu
}  // namespace av1
}  // namespace sk

// Test entry: k_av1_cdf + the k_av1_ec_* coder over caller token streams (tile t:
// tok[offs[t], offs[t] + ns[t])) with the default CDFs of qidx; out receives tile t's
// bytes at the prefix of sizes, words (optional) the interval words of k_av1_cdf.
// Returns 0, or -1 on a HIP error.
extern "C" int sk_av1_ec_tokens_hip(const uint32_t* tok, const int32_t* offs, const int32_t* ns, int tiles, int qidx,
                                    uint8_t* out, int out_cap, int32_t* sizes, uint32_t* words) {
    using namespace sk::av1::gpu;
    int maxn = 1;
    for (int t = 0; t < tiles; t++) maxn = ns[t] > maxn ? ns[t] : maxn;
    Av1Args a;
    memset(&a, 0, sizeof(a));
    a.geo.tile_cols = tiles;
    a.geo.tile_rows = 1;
    a.tile_tok_cap = maxn;
    a.tile_cap = 8 * maxn + 64;
    a.out_cap = out_cap;
    ec_buffers(tiles, a.tile_cap, &a.ec_max_blocks, &a.ec_vcap);
    std::vector<uint32_t> tc((size_t)tiles * maxn, 0u);
    for (int t = 0; t < tiles; t++) memcpy(&tc[(size_t)t * maxn], tok + offs[t], sizeof(uint32_t) * ns[t]);
    int frame[2] = {0, qidx};
    bool ok = tiles <= 64;
    auto chk = [&](hipError_t e) { ok = ok && e == hipSuccess; };
    chk(hipMalloc(&a.tokc, tc.size() * 4));
    chk(hipMalloc(&a.pw, (tc.size() + (size_t)tiles * kEcParts * 64) * 4));
    chk(hipMalloc(&a.tile_ntok, tiles * 4));
    chk(hipMalloc(&a.frame, 8));
    chk(hipMalloc(&a.ecmap, (size_t)a.ec_max_blocks * 128 * sizeof(uint2)));
    chk(hipMalloc(&a.ecblk, (size_t)a.ec_max_blocks * sizeof(int4)));
    chk(hipMalloc(&a.ecv, (size_t)tiles * a.ec_vcap * 8));
    chk(hipMalloc(&a.ecf, (size_t)tiles * a.ec_vcap * 4));
    chk(hipMalloc(&a.tile_bits, tiles * 4));
    chk(hipMalloc(&a.tile_size, tiles * 4));
    chk(hipMalloc(&a.out_host, out_cap));
    chk(hipMalloc(&a.out_size_host, tiles * 4));
    if (ok) {
        chk(hipMemcpy(a.tokc, tc.data(), tc.size() * 4, hipMemcpyHostToDevice));
        chk(hipMemcpy(a.tile_ntok, ns, tiles * 4, hipMemcpyHostToDevice));
        chk(hipMemcpy(a.frame, frame, 8, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_av1_cdf, dim3(tiles * kEcParts), dim3(64), 0, 0, a);
        launch_ec(a, tiles, 0);
        chk(hipGetLastError());
        chk(hipDeviceSynchronize());
        chk(hipMemcpy(sizes, a.out_size_host, tiles * 4, hipMemcpyDeviceToHost));
        chk(hipMemcpy(out, a.out_host, out_cap, hipMemcpyDeviceToHost));
        if (words) {   // k_av1_cdf's interval words, tile t at offs[t]
            std::vector<uint32_t> w(tc.size());
            chk(hipMemcpy(w.data(), a.pw, w.size() * 4, hipMemcpyDeviceToHost));
            for (int t = 0; t < tiles; t++) memcpy(words + offs[t], &w[(size_t)t * maxn], sizeof(uint32_t) * ns[t]);
        }
    }
    for (void* p : {(void*)a.tokc, (void*)a.pw, (void*)a.tile_ntok, (void*)a.frame, (void*)a.ecmap, (void*)a.ecblk,
                    (void*)a.ecv, (void*)a.ecf, (void*)a.tile_bits, (void*)a.tile_size, (void*)a.out_host,
                    (void*)a.out_size_host})
        (void)hipFree(p);
    return ok ? 0 : -1;
}

