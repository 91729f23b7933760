// CPU reference backend of the HEVC encoder: the golden model for the HIP back end
// (kernels/hevc_kernels.hip produces the same CU decisions, levels, reconstruction,
// bins and bytes) and the `use_cpu` path.
#include "hevc_encoder.h"
#include "hevc_pcabac.h"
#include <stdlib.h>
#include <string.h>
#include <algorithm>
#include <stdexcept>

namespace sk {
namespace hevc {

using h264::ACT_I;
using h264::ACT_P;
using h264::ACT_SKIPALL;
using h264::SliceTask;

void build_intra_ref_av(const uint8_t* plane, int stride, int x0, int y0, int n, int avail, uint8_t* ref) {
    uint8_t av[4 * 32 + 1];
    const int len = 4 * n + 1;
    memset(av, 0, (size_t)len);
    memset(ref, 0, (size_t)len);
    // left column p[-1][y], y = 0..2n-1 at ref[2n-1-y] (y >= n: below-left)
    for (int y = 0; y < 2 * n; y++)
        if (avail & (y < n ? AV_L : AV_BL)) {
            ref[2 * n - 1 - y] = plane[(size_t)(y0 + y) * stride + x0 - 1];
            av[2 * n - 1 - y] = 1;
        }
    if (avail & AV_TL) {
        ref[2 * n] = plane[(size_t)(y0 - 1) * stride + x0 - 1];
        av[2 * n] = 1;
    }
    for (int x = 0; x < 2 * n; x++)
        if (avail & (x < n ? AV_T : AV_TR)) {
            ref[2 * n + 1 + x] = plane[(size_t)(y0 - 1) * stride + x0 + x];
            av[2 * n + 1 + x] = 1;
        }
    intra_substitute(ref, av, n);
}

void intra_predict(const uint8_t* ref_raw, int log2n, int mode, int cidx, uint8_t* pred) {
    const int n = 1 << log2n;
    uint8_t filt[4 * 32 + 1];
    const uint8_t* ref = ref_raw;
    if (intra_filter_flag(mode, log2n, cidx)) {
        intra_filter(ref_raw, n, filt);
        ref = filt;
    }
    for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++) pred[y * n + x] = (uint8_t)intra_pred_sample(ref, n, log2n, mode, cidx, x, y);
}

// Host model of the chunk-parallel substream coder (hevc_pcabac.h), chunk = CTB: the
// same four phases the HIP back end runs, sequentially. `cu` lists each CTB's bin
// entries (the row's terminating end_of_subset bin included in the last).
std::vector<uint8_t> pc_code_row_host(const std::vector<std::vector<uint16_t>>& cu, const uint8_t* init_ctx,
                                      std::vector<uint32_t>* dbg_t = nullptr, std::vector<uint32_t>* dbg_r = nullptr,
                                      std::vector<uint32_t>* dbg_tail = nullptr) {
    const int nc = (int)cu.size();
    // 1. context modelling (the GPU runs one chain per context; the states are the same)
    std::vector<std::vector<uint16_t>> mod(cu);
    uint8_t ctx[CTX_COUNT];
    memcpy(ctx, init_ctx, CTX_COUNT);
    for (auto& v : mod)
        for (auto& e : v)
            if ((e & 0x80ffu) < (uint32_t)CTX_TERM) e = pc_model(ctx[e & 0xffu], (e >> 8) & 1);
    // 2. range maps: end range | shifts << 9 for every start range 256..511
    std::vector<uint32_t> map((size_t)nc * 256);
    for (int j = 0; j < nc; j++)
        for (uint32_t r0 = 256; r0 < 512; r0++) {
            uint32_t r = r0, k = 0;
            for (uint16_t e : mod[j]) k += (uint32_t)pc_range_step(e, r);
            map[(size_t)j * 256 + r0 - 256] = r | (k << 9);
        }
    // 3. composition: start range and stream bit offset of every chunk
    std::vector<uint32_t> r0(nc), t0(nc + 1);
    uint32_t r = 510, t = 0;
    for (int j = 0; j < nc; j++) {
        r0[j] = r;
        t0[j] = t;
        const uint32_t m = map[(size_t)j * 256 + r - 256];
        r = m & 511;
        t += m >> 9;
    }
    t0[nc] = t;   // T_f
    // 4. chunk coding: exclusive bytes in place, the 2 overlapping bytes as a tail
    std::vector<uint8_t> out((t >> 3) + 2, 0);
    std::vector<uint32_t> tail(nc, 0);
    for (int j = 0; j < nc; j++) {
        const int g0 = (int)(t0[j] >> 3), gn = (int)(t0[j + 1] >> 3);
        int pos = 0;
        uint32_t tl = 0;
        auto emit = [&](uint32_t b) {
            const int g = g0 + pos++;
            if (g < gn) out[g] = (uint8_t)b;
            else if (g - gn < 2) tl |= b << (8 * (g - gn));
            else throw std::logic_error("pcabac: chunk overran its tail");
        };
        PcCoder c;
        PcLpsTable lps;
        c.start(r0[j], (int)(t0[j] & 7));
        for (uint16_t e : mod[j]) c.code(e, emit, lps);
        c.flush(emit);
        if (g0 + pos != gn + 2) throw std::logic_error("pcabac: chunk byte count");
        tail[j] = tl;
    }
    if (dbg_t) {   // per chunk: stream bit offset, start range, tail (the GPU's cu_t / cu_r / tail)
        dbg_t->assign(t0.begin(), t0.end() - 1);
        dbg_r->assign(r0.begin(), r0.end());
        dbg_tail->assign(tail.begin(), tail.end());
    }
    // merge: add every tail (big-endian 16 bits at its byte) with carries toward the start
    for (int j = 0; j < nc; j++) {
        const int p = (int)(t0[j + 1] >> 3);
        uint32_t v = ((uint32_t)out[p] << 8 | out[p + 1]) + ((tail[j] & 0xff) << 8 | (tail[j] >> 8));
        out[p + 1] = (uint8_t)v;
        out[p] = (uint8_t)(v >> 8);
        for (int q = p - 1; (v >> 16) && q >= 0; q--) {
            v = (uint32_t)out[q] + 1;
            out[q] = (uint8_t)v;
            v <<= 8;
        }
    }
    // stream bits 0..T_f, the rbsp stop bit, zero alignment
    const uint32_t sb = t + 1;
    out[sb >> 3] = (uint8_t)((out[sb >> 3] & (0xff00u >> (sb & 7))) | (0x80u >> (sb & 7)));
    out.resize((sb >> 3) + 1);
    return out;
}

CpuHevcEncoder::CpuHevcEncoder(const h264::EncoderConfig& cfg) : fe(front_config(cfg)) {
    geo.init(fe.g);
    const int n = geo.units(), nc = geo.ctbs();
    cus.assign(n, CuInfo());
    coefs.assign((size_t)n * kCoefPerCu, 0);
    bins.assign((size_t)n * kCuBinCap, 0);
    bin_n.assign(n, 0);
    sao_stats.assign((size_t)3 * nc, SaoStats{});
    sao_own.assign(nc, SaoParams{});
    sao.assign(nc, SaoParams{});
    sao_cost.assign(nc, 0);
    sao_md.assign((size_t)nc * kSaoMd, 0);
    build_parameter_sets(fe.g.W, fe.g.H, cfg.full_range, cfg.fps, param_sets);
    seg_k = intra_seg_k(geo.ctb_w, geo.ctb_h);
}

void CpuHevcEncoder::load_cu_src(int cx, int cy, uint8_t* y, uint8_t* u, uint8_t* v) const {
    const h264::Geometry& g = fe.g;
    for (int r = 0; r < 16; r++) memcpy(y + r * 16, &fe.src[0][(size_t)(cy * 16 + r) * g.stride_y + cx * 16], 16);
    for (int r = 0; r < 8; r++) {
        memcpy(u + r * 8, &fe.src[1][(size_t)(cy * 8 + r) * g.stride_c + cx * 8], 8);
        memcpy(v + r * 8, &fe.src[2][(size_t)(cy * 8 + r) * g.stride_c + cx * 8], 8);
    }
}

// Transform + quantisation of one TU from source and prediction (n x n rasters); the
// TU is zeroed when that costs less (hevc_core.h RD model). Returns cbf, writes the
// levels and the reconstruction and adds the TU's RD cost to *J.
static int code_tu_1(const uint8_t* src, const uint8_t* pred, int log2n, int qp, bool intra, int lam, int16_t* lev,
                     uint8_t* rec, long long* J, bool dst, bool ts) {
    const int n = 1 << log2n, nn = n * n;
    int res[1024], c[1024], d[1024], r[1024];
    for (int i = 0; i < nn; i++) res[i] = (int)src[i] - (int)pred[i];
    if (ts) ts_forward(res, c);
    else fwd_transform(res, log2n, c, dst);
    int nz = 0, rate = kTuRateHalf;
    long long sse0 = 0, sse1 = 0;
    for (int i = 0; i < nn; i++) {
        const int l = quant_level(c[i], qp, log2n, intra);
        lev[i] = (int16_t)l;
        nz |= l;
        rate += level_rate_half(l);
        d[i] = dequant_level(l, qp, log2n);
        sse0 += (long long)res[i] * res[i];
    }
    if (nz) {
        if (ts) ts_inverse(d, r);
        else inv_transform(d, log2n, r, dst);
        for (int i = 0; i < nn; i++) {
            rec[i] = (uint8_t)sk_clip255(pred[i] + r[i]);
            const int e = (int)src[i] - (int)rec[i];
            sse1 += (long long)e * e;
        }
        if (512 * sse0 <= 512 * sse1 + (long long)lam * rate) nz = 0;   // zeroing is cheaper
    }
    if (!nz) {
        for (int i = 0; i < nn; i++) lev[i] = 0;
        memcpy(rec, pred, (size_t)nn);
        *J += 512 * sse0;
    } else {
        *J += 512 * sse1 + (long long)lam * rate;
    }
    return nz != 0;
}
// code_tu_1 with the transform (DST for intra luma 4x4); 4x4 TUs also try transform
// skip and keep the cheaper (*ts = 1 when skipping wins; ties keep the transform).
static int code_tu(const uint8_t* src, const uint8_t* pred, int log2n, int qp, bool intra, int lam, int16_t* lev,
                   uint8_t* rec, long long* J, bool dst = false, int* ts = nullptr) {
    if (ts) *ts = 0;
    if (log2n != 2 || !ts) return code_tu_1(src, pred, log2n, qp, intra, lam, lev, rec, J, dst, false);
    long long j0 = 0, j1 = 0;
    int16_t l1[16];
    uint8_t r1[16];
    const int f0 = code_tu_1(src, pred, 2, qp, intra, lam, lev, rec, &j0, dst, false);
    const int f1 = code_tu_1(src, pred, 2, qp, intra, lam, l1, r1, &j1, dst, true);
    if (f1 && j1 < j0) {
        memcpy(lev, l1, sizeof(l1));
        memcpy(rec, r1, sizeof(r1));
        *ts = 1;
        *J += j1;
        return f1;
    }
    *J += j0;
    return f0;
}

// n x n block at (x, y) of a raster with row pitch `pitch` <-> contiguous n x n.
static void blk_get(const uint8_t* a, int pitch, int x, int y, int n, uint8_t* out) {
    for (int r = 0; r < n; r++) memcpy(out + r * n, a + (y + r) * pitch + x, (size_t)n);
}
static void blk_put(uint8_t* a, int pitch, int x, int y, int n, const uint8_t* in) {
    for (int r = 0; r < n; r++) memcpy(a + (y + r) * pitch + x, in + r * n, (size_t)n);
}
// One TU of a CU-sized raster (pitch 2^log2p): source / prediction block at (x, y),
// reconstruction back into rec.
static int code_tu_at(const uint8_t* src, const uint8_t* pred, int pitch, int x, int y, int log2n, int qp, bool intra,
                      int lam, int16_t* lev, uint8_t* rec, long long* J, bool dst = false, int* ts = nullptr) {
    const int n = 1 << log2n;
    uint8_t s[256], p[256], r[256];
    blk_get(src, pitch, x, y, n, s);
    blk_get(pred, pitch, x, y, n, p);
    const int f = code_tu(s, p, log2n, qp, intra, lam, lev, r, J, dst, ts);
    blk_put(rec, pitch, x, y, n, r);
    return f;
}
// The 4x4 units (z-order bits) that are 4x4 TUs for the node split mask split8.
static uint16_t tu_units4(int split8) {
    uint16_t m = 0;
    for (int q = 0; q < 4; q++)
        if ((split8 >> q) & 1) m |= (uint16_t)(15 << (4 * q));
    return m;
}
// Fills ycbf (cbf_luma per 4x4 unit in z order) from the TU structure and luma cbfs:
// c16 for an unsplit CU, c8 (bit q) for 8x8 TUs, c4 (bit 4q + j) for 4x4 ones.
static uint16_t make_ycbf(const CuInfo& cu, int c16, int c8, int c4) {
    if (!(cu.tu & 16)) return c16 ? 0xffff : 0;
    uint16_t m = 0;
    for (int q = 0; q < 4; q++)
        m |= (uint16_t)((((cu.tu >> q) & 1) ? (c4 >> (4 * q)) & 15 : (((c8 >> q) & 1) ? 15 : 0)) << (4 * q));
    return m;
}

// Residual of an inter CU (prediction in pry / pru / prv, 16x16 / 8x8 rasters): one
// 16x16 TU or four 8x8 nodes, each one 8x8 TU or four 4x4 ones, whichever costs less;
// levels into lev (kCoefPerCu), the reconstruction into ry / ru / rv, the TU fields into cu.
// Returns the tree's RD cost (hevc_core.h model).
static long long code_inter_residual(const uint8_t* sy, const uint8_t* su, const uint8_t* sv, const uint8_t* pry,
                                     const uint8_t* pru, const uint8_t* prv, int qp, int16_t* lev, uint8_t* ry,
                                     uint8_t* ru, uint8_t* rv, CuInfo& cu, int lam_boost) {
    const int qpc = chroma_qp(qp), lam = rd_lambda_q8(qp + lam_boost);
    int16_t la[kCoefPerCu], lb[kCoefPerCu], lc[256];
    uint8_t ay[256], au[64], av[64], by[256], cy4[256], bu[64], bv[64];
    long long ja = 0, jc = (long long)lam * kSplitRateHalf;   // jc: the split CU's chroma + flags
    int cbfa = code_tu(sy, pry, 4, qp, false, lam, la, ay, &ja);
    cbfa |= code_tu(su, pru, 3, qpc, false, lam, la + kCoefCb, au, &ja) << 1;
    cbfa |= code_tu(sv, prv, 3, qpc, false, lam, la + kCoefCr, av, &ja) << 2;
    int c8 = 0, c4 = 0, tuc = 0, split8 = 0, tsy = 0, tsc = 0, f = 0;
    long long jsplit = 0;
    for (int q = 0; q < 4; q++) {
        const int x = 8 * (q & 1), y = 8 * (q >> 1);
        long long j8 = 0, j4 = (long long)lam * kSplit8RateHalf;
        c8 |= code_tu_at(sy, pry, 16, x, y, 3, qp, false, lam, lb + 64 * q, by, &j8) << q;
        for (int j = 0; j < 4; j++) {
            c4 |= code_tu_at(sy, pry, 16, x + 4 * (j & 1), y + 4 * (j >> 1), 2, qp, false, lam, lc + 64 * q + 16 * j, cy4,
                             &j4, false, &f) << (4 * q + j);
            tsy |= f << (4 * q + j);
        }
        if (j4 < j8) split8 |= 1 << q;
        jsplit += j4 < j8 ? j4 : j8;
        tuc |= code_tu_at(su, pru, 8, x / 2, y / 2, 2, qpc, false, lam, lb + kCoefCb + 16 * q, bu, &jc, false, &f) << q;
        tsc |= f << q;
        tuc |= code_tu_at(sv, prv, 8, x / 2, y / 2, 2, qpc, false, lam, lb + kCoefCr + 16 * q, bv, &jc, false, &f) << (q + 4);
        tsc |= f << (q + 4);
    }
    jsplit += jc;
    int ly = 0;   // luma cbf of the chosen split structure
    for (int q = 0; q < 4; q++) ly |= ((split8 >> q) & 1) ? (c4 >> (4 * q)) & 15 : ((c8 >> q) & 1);
    if (jsplit < ja && (ly | tuc)) {
        for (int q = 0; q < 4; q++)
            if ((split8 >> q) & 1) {
                memcpy(lb + 64 * q, lc + 64 * q, 64 * sizeof(int16_t));
                for (int r = 0; r < 8; r++) memcpy(by + (8 * (q >> 1) + r) * 16 + 8 * (q & 1), cy4 + (8 * (q >> 1) + r) * 16 + 8 * (q & 1), 8);
            }
        memcpy(lev, lb, sizeof(lb));
        memcpy(ry, by, 256);
        memcpy(ru, bu, 64);
        memcpy(rv, bv, 64);
        cu.tu = (uint8_t)(16 | split8);
        cu.tuc = (uint8_t)tuc;
        cu.ycbf = make_ycbf(cu, 0, c8, c4);
        cu.tsy = (uint16_t)(tsy & cu.ycbf & tu_units4(split8));
        cu.tsc = (uint8_t)(tsc & tuc);
        cu.cbf = (uint8_t)((cu.ycbf ? 1 : 0) | ((tuc & 15) ? 2 : 0) | ((tuc >> 4) ? 4 : 0));
        return jsplit;
    }
    memcpy(lev, la, sizeof(la));
    memcpy(ry, ay, 256);
    memcpy(ru, au, 64);
    memcpy(rv, av, 64);
    cu.cbf = (uint8_t)cbfa;
    cu.tu = cu.tuc = 0;
    cu.ycbf = make_ycbf(cu, cbfa & 1, 0, 0);
    cu.tsy = 0;
    cu.tsc = 0;
    return ja;
}

void CpuHevcEncoder::put_unit_rec(int ux, int uy, const uint8_t* rec) {
    const h264::Geometry& g = fe.g;
    for (int y = 0; y < 16; y++) memcpy(&fe.rec[0][(size_t)(uy * 16 + y) * g.stride_y + ux * 16], rec + y * 16, 16);
    for (int y = 0; y < 8; y++) {
        memcpy(&fe.rec[1][(size_t)(uy * 8 + y) * g.stride_c + ux * 8], rec + 256 + y * 8, 8);
        memcpy(&fe.rec[2][(size_t)(uy * 8 + y) * g.stride_c + ux * 8], rec + 320 + y * 8, 8);
    }
}

// CU32 choice of a complete CTB whose units were coded as CU16s: the PU split the unit
// vectors allow, each PU's merge / AMVP syntax from its own neighbours, and the residual as
// the units' trees under a split root or as one 32x32 TU (+ 16x16 chroma TUs), whichever
// costs less; the CU32 replaces the four CU16s when its RD cost (header estimate + residual)
// is lower. k_hevc_inter's second phase runs the same rule.
template <class MV>
void CpuHevcEncoder::cu32_decide(int c, int r, const Cu32Work& wk, int qp, int lam_boost, MV mv) {
    const UnitGrid ug = geo.grid();
    const SliceMap m = smap();
    const int W = geo.W16;
    int mx[4], my[4], idx[4];
    for (int z = 0; z < 4; z++) {
        idx[z] = (2 * r + (z >> 1)) * W + 2 * c + (z & 1);
        mx[z] = cus[idx[z]].mvx;
        my[z] = cus[idx[z]].mvy;
    }
    const int part = cu32_part(mx, my);
    if (part < 0) return;
    CuInfo pu[2];
    memset(pu, 0, sizeof(pu));
    for (int pi = 0; pi < (part == PART_2Nx2N ? 1 : 2); pi++) {
        int xp, yp, pw, ph;
        pu_rect(part, pi, 32 * c, 32 * r, 32, &xp, &yp, &pw, &ph);
        const PuNb nb = pu_neighbours(ug, m, mv, 32 * c, 32 * r, 32, xp, yp, pw, ph, pi);
        int mlx[kMaxMergeCand], mly[kMaxMergeCand], px[2], py[2];
        pu_merge_list(nb, part, pi, mlx, mly);
        pu_amvp_list(nb, px, py);
        const int z = pi == 0 ? 0 : 3;
        pu_choose(pu[pi], mx[z], my[z], mlx, mly, px, py);
    }
    if (part == PART_2Nx2N) pu[1] = pu[0];
    const int lam = rd_lambda_q8(qp + lam_boost);
    long long jsum = 0;
    int hsplit = 0, cbf_units = 0;
    for (int z = 0; z < 4; z++) {
        jsum += wk.j[z];
        hsplit += cu16_hdr_half(cus[idx[z]]);
        cbf_units |= cus[idx[z]].cbf;
    }
    // one 32x32 TU: luma 32x32 and the 16x16 chroma TUs from the units' rasters
    uint8_t s32[kT32Coefs], p32[kT32Coefs], r32[kT32Coefs];
    for (int z = 0; z < 4; z++) {
        const int ox = 16 * (z & 1), oy = 16 * (z >> 1);
        for (int y = 0; y < 16; y++)
            for (int x = 0; x < 16; x++) {
                s32[(oy + y) * 32 + ox + x] = wk.src[z][y * 16 + x];
                p32[(oy + y) * 32 + ox + x] = wk.pred[z][y * 16 + x];
            }
        for (int k = 0; k < 2; k++)
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    const int o = (k ? kT32Cr : kT32Cb) + (oy / 2 + y) * 16 + ox / 2 + x;
                    s32[o] = wk.src[z][256 + 64 * k + y * 8 + x];
                    p32[o] = wk.pred[z][256 + 64 * k + y * 8 + x];
                }
    }
    int16_t l32[kT32Coefs];
    long long j32 = 0;
    int cbf32 = 0;
    bool tu32 = false;
    if (cbf_units) {   // the 32x32 TU is tried when some unit codes a residual (k_hevc_inter: same rule)
        const int qpc = chroma_qp(qp);
        cbf32 = code_tu_1(s32, p32, 5, qp, false, lam, l32, r32, &j32, false, false);
        cbf32 |= code_tu_1(s32 + kT32Cb, p32 + kT32Cb, 4, qpc, false, lam, l32 + kT32Cb, r32 + kT32Cb, &j32, false, false) << 1;
        cbf32 |= code_tu_1(s32 + kT32Cr, p32 + kT32Cr, 4, qpc, false, lam, l32 + kT32Cr, r32 + kT32Cr, &j32, false, false) << 2;
        tu32 = j32 < jsum;
    }
    const int root = tu32 ? cbf32 : cbf_units;
    const bool skip = part == PART_2Nx2N && pu[0].mode == CU_MERGE && !root;
    const long long jc = (long long)lam * cu32_hdr_half(part, pu[0], pu[1], skip) + (tu32 ? j32 : jsum);
    const long long js = (long long)lam * hsplit + jsum;
    if (jc >= js) return;
    for (int z = 0; z < 4; z++) {
        CuInfo& cu = cus[idx[z]];
        const CuInfo& p = pu[cu32_pu_of(part, z)];
        cu.mode = skip ? CU_SKIP : p.mode;
        cu.merge_idx = p.merge_idx;
        cu.mvp_idx = p.mvp_idx;
        cu.mvdx = p.mvdx;
        cu.mvdy = p.mvdy;
        cu.c32 = (uint8_t)(kC32 | (part << 1) | (tu32 ? kC32Tu : 0));
        if (!tu32) continue;
        cu.cbf = (uint8_t)cbf32;
        cu.tu = cu.tuc = 0;
        cu.ycbf = (cbf32 & 1) ? 0xffff : 0;
        cu.tsy = 0;
        cu.tsc = 0;
        memcpy(&coefs[(size_t)idx[z] * kCoefPerCu], l32 + z * kCoefPerCu, kCoefPerCu * sizeof(int16_t));
        uint8_t rec[kCoefPerCu];
        const int ox = 16 * (z & 1), oy = 16 * (z >> 1);
        for (int y = 0; y < 16; y++) memcpy(rec + y * 16, r32 + (oy + y) * 32 + ox, 16);
        for (int k = 0; k < 2; k++)
            for (int y = 0; y < 8; y++)
                memcpy(rec + 256 + 64 * k + y * 8, r32 + (k ? kT32Cr : kT32Cb) + (oy / 2 + y) * 16 + ox / 2, 8);
        put_unit_rec(2 * c + (z & 1), 2 * r + (z >> 1), rec);
    }
}

void CpuHevcEncoder::code_slice_inter(int s) {
    const SliceTask& t = fe.tasks[s];
    const h264::Geometry& g = fe.g;
    const UnitGrid ug = geo.grid();
    const SliceMap m = smap();
    const int qp = t.qp, W = geo.W16;
    const int lam_boost = fe.ctl_.rc().lam_boost;
    auto mv = [&](int ux, int uy, int* x, int* y) {
        *x = h264::me_qx(fe.me[uy * W + ux]);
        *y = h264::me_qy(fe.me[uy * W + ux]);
    };
    const int r0 = t.first_row >> 1, r1 = (t.first_row + t.num_rows + 1) >> 1;
    for (int r = r0; r < r1; r++)
        for (int c = 0; c < geo.ctb_w; c++) {
            // (1) every unit of the CTB as a 16x16 CU (kept: prediction, source, RD cost)
            Cu32Work wk;
            for (int z = 0; z < 4; z++) {
                const int ux = 2 * c + (z & 1), uy = 2 * r + (z >> 1);
                wk.in[z] = ug.inside(ux, uy);
                if (!wk.in[z]) continue;
                const int idx = uy * W + ux;
                CuInfo& cu = cus[idx];
                memset(&cu, 0, sizeof(cu));
                int mvx, mvy;
                mv(ux, uy, &mvx, &mvy);
                const PuNb nb = pu_neighbours(ug, m, mv, 16 * ux, 16 * uy, 16, 16 * ux, 16 * uy, 16, 16, 0);
                int mlx[kMaxMergeCand], mly[kMaxMergeCand], px[2], py[2];
                pu_merge_list(nb, PART_2Nx2N, 0, mlx, mly);
                pu_amvp_list(nb, px, py);
                uint8_t* sy = wk.src[z];
                uint8_t* pry = wk.pred[z];
                load_cu_src(ux, uy, sy, sy + 256, sy + 320);
                for (int y = 0; y < 16; y++)
                    for (int x = 0; x < 16; x++)
                        pry[y * 16 + x] = (uint8_t)luma_mc_sample(fe.ref[0].data(), g.stride_y, geo.pic_w, geo.pic_h,
                                                                  ux * 16 + x, uy * 16 + y, mvx, mvy);
                for (int y = 0; y < 8; y++)
                    for (int x = 0; x < 8; x++) {
                        pry[256 + y * 8 + x] = (uint8_t)chroma_mc_sample(fe.ref[1].data(), g.stride_c, g.stride_c,
                                                                         g.plane_h_c, ux * 8 + x, uy * 8 + y, mvx, mvy);
                        pry[320 + y * 8 + x] = (uint8_t)chroma_mc_sample(fe.ref[2].data(), g.stride_c, g.stride_c,
                                                                         g.plane_h_c, ux * 8 + x, uy * 8 + y, mvx, mvy);
                    }
                int16_t* lev = &coefs[(size_t)idx * kCoefPerCu];
                uint8_t rec[kCoefPerCu];
                wk.j[z] = code_inter_residual(sy, sy + 256, sy + 320, pry, pry + 256, pry + 320, qp, lev, rec, rec + 256,
                                              rec + 320, cu, lam_boost);
                cu.qp = (uint8_t)qp;
                pu_choose(cu, mvx, mvy, mlx, mly, px, py);
                if (cu.mode == CU_MERGE && !cu.cbf) cu.mode = CU_SKIP;
                for (int i = 0; i < 16; i++) cu.ipm[i] = 1;
                put_unit_rec(ux, uy, rec);
            }
            // (2) one 32x32 CU instead, when the motion allows a PU split and it costs less
            if (ug.complete(c, r)) cu32_decide(c, r, wk, qp, lam_boost, mv);
        }
}
// Open-loop intra decision of one unit of an I slice (all units in parallel on the GPU,
// k_hevc_intra_prep): the SAD of every mode on each 4x4 block, predicted from its source
// neighbours, gives the best mode of the 16x16 CU, of each 8x8 CU and of each 4x4 PU
// (SAD + intra_mode_bias); four CU8s (each PART_2Nx2N or PART_NxN, the cheaper) replace the
// CU16 when their total plus a split penalty is lower.
void intra_decide(const uint32_t sad[16][35], int qp, CuInfo& cu) {
    const int lam = intra_lam_sad(qp);
    int best16 = 1, c16 = 0x7fffffff;
    for (int k = 0; k < 35; k++) {   // HEVC_INTRA_ORDER, first minimum wins
        const int m = HEVC_INTRA_ORDER[k];
        int s = intra_mode_bias(m, qp);
        for (int u = 0; u < 16; u++) s += (int)sad[u][m];
        if (s < c16) { c16 = s; best16 = m; }
    }
    int csplit = kPenSplit * lam, nxn = 0, b8[4], b4[16];
    for (int q = 0; q < 4; q++) {
        int c8 = 0x7fffffff;
        b8[q] = 1;
        for (int k = 0; k < 35; k++) {
            const int m = HEVC_INTRA_ORDER[k];
            int s = intra_mode_bias(m, qp);
            for (int j = 0; j < 4; j++) s += (int)sad[4 * q + j][m];
            if (s < c8) { c8 = s; b8[q] = m; }
        }
        int cn = kPenNxN * lam;
        for (int j = 0; j < 4; j++) {
            int c4 = 0x7fffffff;
            b4[4 * q + j] = 1;
            for (int k = 0; k < 35; k++) {
                const int m = HEVC_INTRA_ORDER[k];
                const int s = (int)sad[4 * q + j][m] + intra_mode_bias(m, qp);
                if (s < c4) { c4 = s; b4[4 * q + j] = m; }
            }
            cn += c4;
        }
        if (cn < c8) nxn |= 1 << q;
        csplit += cn < c8 ? cn : c8;
    }
    memset(&cu, 0, sizeof(cu));
    cu.mode = CU_INTRA;
    if (csplit < c16) {
        cu.cu8 = (uint8_t)(16 | nxn);
        for (int u = 0; u < 16; u++) cu.ipm[u] = (uint8_t)(((nxn >> (u >> 2)) & 1) ? b4[u] : b8[u >> 2]);
    } else {
        for (int u = 0; u < 16; u++) cu.ipm[u] = (uint8_t)best16;
    }
    cu.intra_mode = cu.ipm[0];
}

// Closed-loop intra coding of one unit (its decisions from intra_decide): a CU16 chooses
// between the 16x16 TU and the split tree (each 8x8 node's TU against its four 4x4 TUs);
// a CU8-split unit codes each CU8 with its own mode(s) - PART_2Nx2N: 8x8 TU or four 4x4,
// PART_NxN: four 4x4 TUs, one per PU - every TU predicted from the reconstruction before it.
void CpuHevcEncoder::code_unit_intra(int ux, int uy, int qp) {
    const h264::Geometry& g = fe.g;
    const int qpc = chroma_qp(qp), lam = rd_lambda_q8(qp);
    const int idx = uy * geo.W16 + ux;
    CuInfo& cu = cus[idx];
    const int nbm = unit_nbm(geo.grid(), smap(), ux, uy);
    const bool cu8 = (cu.cu8 & 16) != 0;
    uint8_t sy[256], su[64], sv[64];
    load_cu_src(ux, uy, sy, su, sv);
    int16_t* lev = &coefs[(size_t)idx * kCoefPerCu];
    uint8_t* P[3] = {fe.rec[0].data(), fe.rec[1].data(), fe.rec[2].data()};
    const int st[3] = {g.stride_y, g.stride_c, g.stride_c};
    const uint8_t* S[3] = {sy, su, sv};
    auto region = [&](int c, bool save, uint8_t* buf, int ox, int oy, int n) {
        uint8_t* base = P[c] + (size_t)(uy * (c ? 8 : 16) + oy) * st[c] + ux * (c ? 8 : 16) + ox;
        if (save) blk_get(base, st[c], 0, 0, n, buf);
        else blk_put(base, st[c], 0, 0, n, buf);
    };
    int tsf = 0;
    auto tu = [&](int c, int log2n, int ox, int oy, int av, int mode, int16_t* l, long long* J) {
        const int n = 1 << log2n, x0 = ux * (c ? 8 : 16) + ox, y0 = uy * (c ? 8 : 16) + oy;
        uint8_t ref[65], pr[256], src[256], rec[256];
        build_intra_ref_av(P[c], st[c], x0, y0, n, av, ref);
        intra_predict(ref, log2n, mode, c, pr);
        blk_get(S[c], c ? 8 : 16, ox, oy, n, src);
        const int f = code_tu(src, pr, log2n, c ? qpc : qp, true, lam, l, rec, J, c == 0 && log2n == 2, &tsf);
        blk_put(P[c] + (size_t)y0 * st[c] + x0, st[c], 0, 0, n, rec);
        return f;
    };
    // (a) one 16x16 TU (CU16 only)
    int16_t la[kCoefPerCu], lb[kCoefPerCu], l4[64];
    uint8_t ay[256], au[64], av8[64];
    long long ja = 0x7fffffffffffffffll, jb = (long long)lam * kSplitRateHalf;
    int cbfa = 0;
    if (!cu8) {
        const int m = cu.ipm[0];
        ja = 0;
        cbfa = tu(0, 4, 0, 0, cu_avail(nbm), m, la, &ja);
        cbfa |= tu(1, 3, 0, 0, cu_avail(nbm), m, la + kCoefCb, &ja) << 1;
        cbfa |= tu(2, 3, 0, 0, cu_avail(nbm), m, la + kCoefCr, &ja) << 2;
        region(0, true, ay, 0, 0, 16);
        region(1, true, au, 0, 0, 8);
        region(2, true, av8, 0, 0, 8);
    }
    // (b) four nodes / CU8s
    int c8 = 0, c4 = 0, tuc = 0, tsy = 0, tsc = 0, split8 = 0;
    for (int q = 0; q < 4; q++) {
        const int av = tu_avail(q, nbm), ox = 8 * (q & 1), oy = 8 * (q >> 1);
        const int mq = cu.ipm[4 * q], nxn = cu8 && ((cu.cu8 >> q) & 1);
        long long j8 = 0x7fffffffffffffffll, j4 = (long long)lam * kSplit8RateHalf;
        uint8_t r8[64];
        int f8 = 0;
        if (!nxn) {
            j8 = 0;
            f8 = tu(0, 3, ox, oy, av, mq, lb + 64 * q, &j8);
            region(0, true, r8, ox, oy, 8);
        }
        int f4 = 0, t4 = 0;
        for (int j = 0; j < 4; j++) {
            const int bx = 2 * (q & 1) + (j & 1), by = 2 * (q >> 1) + (j >> 1);
            f4 |= tu(0, 2, 4 * bx, 4 * by, tu_avail_at(bx, by, 1, nbm), cu.ipm[4 * q + j], l4 + 16 * j, &j4) << j;
            t4 |= tsf << j;
        }
        if (j4 < j8) {
            split8 |= 1 << q;
            memcpy(lb + 64 * q, l4, sizeof(l4));
            c4 |= f4 << (4 * q);
            tsy |= t4 << (4 * q);
            jb += j4;
        } else {
            region(0, false, r8, ox, oy, 8);
            c8 |= f8 << q;
            jb += j8;
        }
        tuc |= tu(1, 2, ox / 2, oy / 2, av, mq, lb + kCoefCb + 16 * q, &jb) << q;
        tsc |= tsf << q;
        tuc |= tu(2, 2, ox / 2, oy / 2, av, mq, lb + kCoefCr + 16 * q, &jb) << (q + 4);
        tsc |= tsf << (q + 4);
    }
    if (jb < ja) {
        memcpy(lev, lb, sizeof(lb));
        cu.tu = (uint8_t)(16 | split8);
        cu.tuc = (uint8_t)tuc;
        cu.ycbf = make_ycbf(cu, 0, c8, c4);
        cu.cbf = (uint8_t)((cu.ycbf ? 1 : 0) | ((tuc & 15) ? 2 : 0) | ((tuc >> 4) ? 4 : 0));
        cu.tsy = (uint16_t)tsy;
        cu.tsc = (uint8_t)tsc;
    } else {
        memcpy(lev, la, sizeof(la));
        region(0, false, ay, 0, 0, 16);
        region(1, false, au, 0, 0, 8);
        region(2, false, av8, 0, 0, 8);
        cu.tu = cu.tuc = 0;
        cu.cbf = (uint8_t)cbfa;
        cu.ycbf = make_ycbf(cu, cbfa & 1, 0, 0);
        cu.tsy = 0;
        cu.tsc = 0;
    }
    cu.qp = (uint8_t)qp;
    fe.me[idx].mvx = fe.me[idx].mvy = 0;
    fe.me[idx].ref = 0;
    fe.me[idx].fx = fe.me[idx].fy = 0;
}

// I slices in two passes, like the H.264 intra path: (1) every unit independently
// chooses its CU structure and modes against the SOURCE neighbours (parallel on the GPU),
// (2) the units are coded in coding order (CTB raster, z order) from the reconstruction,
// choosing the transform trees by RD.
void CpuHevcEncoder::code_slice_intra(int s) {
    const SliceTask& t = fe.tasks[s];
    const h264::Geometry& g = fe.g;
    const UnitGrid ug = geo.grid();
    const SliceMap m = smap();
    const int r0 = t.first_row >> 1, r1 = (t.first_row + t.num_rows + 1) >> 1;
    for (int uy = t.first_row; uy < t.first_row + t.num_rows; uy++)
        for (int ux = 0; ux < geo.W16; ux++) {
            const int nbm = unit_nbm(ug, m, ux, uy);
            uint8_t sy[256], su[64], sv[64];
            load_cu_src(ux, uy, sy, su, sv);
            uint8_t ref4[16][17];
            for (int u = 0; u < 16; u++) {   // 4x4 block u in z order
                const int bx = (u & 1) | ((u >> 1) & 2), by = ((u >> 1) & 1) | ((u >> 2) & 2);
                build_intra_ref_av(fe.src[0].data(), g.stride_y, ux * 16 + 4 * bx, uy * 16 + 4 * by, 4,
                                   tu_avail_at(bx, by, 1, nbm), ref4[u]);
            }
            uint32_t sad[16][35];
            for (int mo = 0; mo < 35; mo++)
                for (int u = 0; u < 16; u++) {
                    const int bx = (u & 1) | ((u >> 1) & 2), by = ((u >> 1) & 1) | ((u >> 2) & 2);
                    uint8_t pr[16];
                    intra_predict(ref4[u], 2, mo, 0, pr);
                    uint32_t a = 0;
                    for (int i = 0; i < 16; i++) a += (uint32_t)sk_abs((int)sy[(4 * by + (i >> 2)) * 16 + 4 * bx + (i & 3)] - (int)pr[i]);
                    sad[u][mo] = a;
                }
            intra_decide(sad, t.qp, cus[uy * geo.W16 + ux]);
        }
    for (int r = r0; r < r1; r++)
        for (int c = 0; c < geo.ctb_w; c++)
            for (int z = 0; z < 4; z++) {
                const int ux = 2 * c + (z & 1), uy = 2 * r + (z >> 1);
                if (ug.inside(ux, uy)) code_unit_intra(ux, uy, t.qp);
            }
}

// Skip-all slices: the reference as it is, every complete CTB one skipped CU32 (merge
// candidate 0 is the zero vector there), the units of partial CTBs skipped CU16s.
void CpuHevcEncoder::code_slice_skip(int s) {
    const SliceTask& t = fe.tasks[s];
    const UnitGrid ug = geo.grid();
    fe.code_slice_skipall(s);   // motion field zero, reconstruction = reference
    for (int uy = t.first_row; uy < t.first_row + t.num_rows; uy++)
        for (int ux = 0; ux < geo.W16; ux++) {
            CuInfo& cu = cus[uy * geo.W16 + ux];
            memset(&cu, 0, sizeof(cu));
            cu.mode = CU_SKIP;
            cu.qp = (uint8_t)t.qp;
            for (int i = 0; i < 16; i++) cu.ipm[i] = 1;
            if (ug.complete(ux >> 1, uy >> 1)) cu.c32 = kC32;   // PART_2Nx2N, merge_idx 0
        }
}

// Plane geometry for SAO: plane 0 luma (CTB 32), 1 / 2 chroma (CTB 16).
static SaoPlane sao_plane(const Geo& geo, int c, const SliceMap& m) {
    const int n = c ? 16 : 32, u = c ? 8 : 16;
    return SaoPlane{geo.W16 * u, geo.H16 * u, n, m};
}

void CpuHevcEncoder::sao_analyse() {
    const h264::Geometry& g = fe.g;
    const SliceMap m = smap();
    const int rps = fe.g.rows_per_slice;   // unit rows per slice
    for (int cy = 0; cy < geo.ctb_h; cy++)
        for (int cx = 0; cx < geo.ctb_w; cx++) {
            const int idx = cy * geo.ctb_w + cx;
            // skip-all slices keep the reference as it is (finish_frame does not copy them
            // back): their stats stay empty, so every CTB there decides "off"
            const SliceTask& t = fe.tasks[(2 * cy) / rps];
            const bool coded = t.final_action == ACT_P || t.final_action == ACT_I;
            for (int c = 0; c < 3; c++) {
                SaoStats& st = sao_stats[(size_t)3 * idx + c];
                st = SaoStats{};
                if (!coded) continue;
                const SaoPlane pl = sao_plane(geo, c, m);
                const int stride = c ? g.stride_c : g.stride_y;
                for (int y = cy * pl.n; y < (cy + 1) * pl.n && y < pl.h; y++)
                    for (int x = cx * pl.n; x < (cx + 1) * pl.n && x < pl.w; x++)
                        sao_collect(st, pl, fe.rec[c].data(), stride, x, y, fe.src[c][(size_t)y * stride + x]);
            }
            const int lam = sao_lambda(t.qp);
            SaoTables tb;
            for (int i = 0; i < kSaoTableEntries; i++) sao_table_entry(&sao_stats[(size_t)3 * idx], lam, i, tb);
            for (int i = 0; i < 96; i++) sao_window(lam, i, tb);
            sao_cost[idx] = sao_pick(tb, lam, sao_own[idx]);
        }
    for (int cy = 0; cy < geo.ctb_h; cy++)
        for (int cx = 0; cx < geo.ctb_w; cx++) {
            const size_t idx = (size_t)cy * geo.ctb_w + cx;
            sao_merge_dists(&sao_stats[3 * idx], &sao_own[(size_t)cy * geo.ctb_w], cx, &sao_md[idx * kSaoMd]);
        }
    for (int cy = 0; cy < geo.ctb_h; cy++) {
        const SliceTask& t = fe.tasks[(2 * cy) / rps];
        const size_t o = (size_t)cy * geo.ctb_w;
        std::vector<uint16_t> sel(geo.ctb_w);
        std::vector<uint8_t> fl(geo.ctb_w);
        sao_row_merge(&sao_md[o * kSaoMd], &sao_own[o], &sao_cost[o], geo.ctb_w, t.qp, m, cy, &sao[o], sel.data(),
                      fl.data());
    }
}

void CpuHevcEncoder::sao_apply() {
    const h264::Geometry& g = fe.g;
    for (int c = 0; c < 3; c++) {
        const SaoPlane pl = sao_plane(geo, c, smap());
        const int stride = c ? g.stride_c : g.stride_y;
        const std::vector<uint8_t> dbk = fe.rec[c];   // the filter reads deblocked samples only
        for (int y = 0; y < pl.h; y++)
            for (int x = 0; x < pl.w; x++) {
                const SaoParams& p = sao[(size_t)(y / pl.n) * geo.ctb_w + x / pl.n];
                fe.rec[c][(size_t)y * stride + x] = (uint8_t)sao_apply_sample(p, c, pl, dbk.data(), stride, x, y);
            }
    }
}

// The binariser's view of unit (ux, uy) (hevc_core.h UnitCtx); k_hevc_bins builds the same.
static UnitCtx unit_ctx(const UnitGrid& ug, const SliceMap& m, int ux, int uy, bool p_slice) {
    UnitCtx u;
    u.z = (ux & 1) | ((uy & 1) << 1);
    u.first = u.z == 0;
    u.complete = ug.complete(ux >> 1, uy >> 1);
    u.left = ug.avail(m, ux, uy, ux - 1, uy);
    u.top = ug.avail(m, ux, uy, ux, uy - 1);
    u.row0 = (uy & 1) == 0;
    u.p_slice = p_slice;
    return u;
}
// Whether unit (ux, uy) is the last of its CTB in coding order.
static bool ctb_last_unit(const UnitGrid& ug, int ux, int uy) {
    const int z = (ux & 1) | ((uy & 1) << 1), c = ux >> 1, r = uy >> 1;
    for (int k = z + 1; k < 4; k++)
        if (ug.inside(2 * c + (k & 1), 2 * r + (k >> 1))) return false;
    return true;
}

void CpuHevcEncoder::binarize_slice(int s) {
    const SliceTask& t = fe.tasks[s];
    const bool p_slice = t.final_action != ACT_I;
    const UnitGrid ug = geo.grid();
    const SliceMap m = smap();
    const int r0 = t.first_row >> 1, r1 = (t.first_row + t.num_rows + 1) >> 1;
    const int W = geo.W16;
    for (int uy = t.first_row; uy < t.first_row + t.num_rows; uy++)
        for (int ux = 0; ux < W; ux++) {
            const int idx = uy * W + ux, c = ux >> 1, r = uy >> 1;
            const UnitCtx u = unit_ctx(ug, m, ux, uy, p_slice);
            BinBuf w{&bins[(size_t)idx * kCuBinCap], 0};
            if (u.first) sao_bins(w, sao[r * geo.ctb_w + c], m.left(c, r), m.top(c, r));   // CTB-level SAO syntax
            const size_t i0 = (size_t)2 * r * W + 2 * c;   // the CTB's unit z0
            code_unit(w, u, cus[idx], u.left ? &cus[idx - 1] : nullptr, u.top ? &cus[idx - W] : nullptr,
                      &coefs[(size_t)idx * kCoefPerCu], Ctb4{&cus[i0], &coefs[i0 * kCoefPerCu], W});
            if (ctb_last_unit(ug, ux, uy)) {
                // end_of_slice_segment_flag: the last CTB of the slice (a split row: of its segment)
                const bool end = m.split(r) ? c + 1 == m.x1(r, m.seg(c, r)) : r == r1 - 1 && c == geo.ctb_w - 1;
                w.term(end);
            }
            bin_n[idx] = w.n;
        }
    (void)r0;
}

// One slice segment NAL: CTB rows cy0 .. cy0 + rows - 1, CTB columns [x0, x1) of each (a
// split row: one row, one segment), one CABAC substream per row - its units' bin chunks in
// coding order - with WPP storage after the second CTB, entry points for the rows after
// the first.
std::vector<uint8_t> CpuHevcEncoder::write_segment(const SliceTask& t, int cy0, int rows, int x0, int x1, bool idr) {
    const bool p_slice = t.final_action != ACT_I;
    const UnitGrid ug = geo.grid();
    std::vector<std::vector<uint8_t>> sub(rows);
    uint8_t sync[CTX_COUNT];
    for (int r = 0; r < rows; r++) {
        const int cy = cy0 + r;
        uint8_t ctx[CTX_COUNT];
        if (r == 0 || geo.ctb_w < 2) ctx_init_all(ctx, p_slice ? 1 : 0, t.qp);
        else memcpy(ctx, sync, CTX_COUNT);
        const int j0 = ug.ctb_chunk0(cy, x0), j1 = ug.ctb_chunk0(cy, x1 < geo.ctb_w ? x1 : geo.ctb_w);
        const int jn = x1 < geo.ctb_w ? j1 : ug.row_chunks(cy);
        const int jsync = ug.ctb_chunk0(cy, x0 + 2 < geo.ctb_w ? x0 + 2 : geo.ctb_w);   // after CTB x0 + 1
        const int jsync_end = x0 + 2 < geo.ctb_w ? jsync : ug.row_chunks(cy);
        if (pc_host_) {   // chunk-parallel model (hevc_pcabac.h), must give the same bytes
            std::vector<std::vector<uint16_t>> cu(jn - j0);
            for (int j = j0; j < jn; j++) {
                const int u = ug.chunk_unit(cy, j);
                const uint16_t* b = &bins[(size_t)u * kCuBinCap];
                cu[j - j0].assign(b, b + bin_n[u]);
            }
            if (r + 1 < rows) cu.back().push_back((uint16_t)((1u << 8) | CTX_TERM));   // end_of_subset_one_bit
            std::vector<uint32_t> dt, dr, dtl;
            sub[r] = pc_code_row_host(cu, ctx, &dt, &dr, &dtl);
            if (pc_dbg_.size() != (size_t)3 * geo.units()) pc_dbg_.assign((size_t)3 * geo.units(), 0);
            for (int j = j0; j < jn; j++) {
                const int u = ug.chunk_unit(cy, j);
                pc_dbg_[3 * (size_t)u] = dt[j - j0];
                pc_dbg_[3 * (size_t)u + 1] = dr[j - j0];
                pc_dbg_[3 * (size_t)u + 2] = dtl[j - j0];
            }
            for (int j = j0; j < jsync_end; j++) {
                const int u = ug.chunk_unit(cy, j);
                for (int i = 0; i < bin_n[u]; i++) {
                    const uint16_t e = bins[(size_t)u * kCuBinCap + i];
                    if ((e & 0x80ffu) < (uint32_t)CTX_TERM) ctx_update(ctx[e & 0xffu], (e >> 8) & 1);
                }
            }
            memcpy(sync, ctx, CTX_COUNT);
            payload_bytes_ += (long long)sub[r].size();
            continue;
        }
        size_t cap = 64;
        for (int j = j0; j < jn; j++) cap += (size_t)bin_n[ug.chunk_unit(cy, j)] * 2 + 8;
        sub[r].assign(cap, 0);
        CabacEncoder e;
        e.start(sub[r].data());
        for (int j = j0; j < jn; j++) {
            const int u = ug.chunk_unit(cy, j);
            const uint16_t* b = &bins[(size_t)u * kCuBinCap];
            for (int i = 0; i < bin_n[u]; i++) e.code_entry(b[i], ctx);
            if (j + 1 == jsync_end) memcpy(sync, ctx, CTX_COUNT);   // WPP storage after the second CTB
        }
        if (r + 1 < rows) e.terminate(1);   // end_of_subset_one_bit
        e.finish();
        sub[r].resize(e.pos);
        payload_bytes_ += (long long)e.pos;
    }
    // entry points count emulation-prevention bytes (7.4.7.1)
    std::vector<int> esc(rows);
    for (int r = 0; r < rows; r++) esc[r] = ep_escape(sub[r].data(), (int)sub[r].size(), nullptr);
    uint8_t hdr[1024];
    memset(hdr, 0, sizeof(hdr));
    SliceHeader h;
    h.address = cy0 * geo.ctb_w + x0;
    h.first_slice = h.address == 0;
    h.idr = idr;
    h.address_bits = geo.addr_bits;
    h.slice_type = p_slice ? 1 : 2;
    h.poc_lsb = poc & ((1 << kLog2MaxPocLsb) - 1);
    h.qp_delta = t.qp - 26;
    h.num_entry = rows - 1;
    h.entry = esc.data();
    const int hn = write_slice_header(hdr, h);
    std::vector<uint8_t> rbsp(hdr, hdr + hn);
    for (int r = 0; r < rows; r++) rbsp.insert(rbsp.end(), sub[r].begin(), sub[r].end());
    // append_nal escapes the concatenation; pieces end in non-zero bytes, so this equals
    // escaping each piece on its own (what the entry points were computed from)
    std::vector<uint8_t> nal;
    append_nal(nal, idr ? kNalIdrWRadl : kNalTrailR, rbsp.data(), rbsp.size());
    return nal;
}

std::vector<uint8_t> CpuHevcEncoder::write_slice(int s, bool idr) {
    const SliceTask& t = fe.tasks[s];
    const SliceMap m = smap();
    const int r0 = t.first_row >> 1, nr = ((t.first_row + t.num_rows + 1) >> 1) - r0;
    if (!m.split(r0)) return write_segment(t, r0, nr, 0, geo.ctb_w, idr);
    std::vector<uint8_t> out;   // a split intra slice: one slice NAL per row segment
    for (int cy = r0; cy < r0 + nr; cy++)
        for (int k = 0; k < m.nseg(cy); k++) {
            const std::vector<uint8_t> nal = write_segment(t, cy, 1, m.x0(cy, k), m.x1(cy, k), idr);
            out.insert(out.end(), nal.begin(), nal.end());
        }
    return out;
}

void CpuHevcEncoder::encode(const uint8_t* bgrx, int stride, uint16_t frame_id,
                            std::vector<h264::EncodedPacket>& out) {
    fe.load_frame(bgrx, stride);
    fe.ctl_.plan(fe.stripe_dirty.data(), fe.tasks.data());
    for (auto& st : fe.ctl_.stripes()) {   // K4c gate, rotated by k_plan on the GPU
        st.subpel_prev = st.subpel_hits;
        st.subpel_hits = 0;
    }
    const int ns = geo.num_slices;
    for (int s = 0; s < ns; s++)
        if (fe.tasks[s].action == ACT_P) {
            fe.motion_search(s);
            fe.decide_scenecut(s);
        } else if (fe.tasks[s].action == ACT_I) {
            fe.intra_activity(s);
        }
    fe.ctl_.rate_control(fe.tasks.data(), fe.me.data());   // K10
    // CU coding at the slice QPs, in-loop deblocking, then the SAO decisions on the
    // deblocked picture (they are syntax of every CTB, so the binarisation follows them).
    // Every coded sample of the picture is rewritten, so a second pass starts clean.
    auto code_picture = [&] {
        for (int s = 0; s < ns; s++) {
            switch (fe.tasks[s].final_action) {
                case ACT_P: code_slice_inter(s); break;
                case ACT_I: code_slice_intra(s); break;
                default: code_slice_skip(s); break;
            }
        }
        deblock_picture(fe.rec[0].data(), fe.rec[1].data(), fe.rec[2].data(), fe.g.stride_y, fe.g.stride_c,
                        cus.data(), geo.W16, geo.H16, smap());
        sao_analyse();
        for (int s = 0; s < ns; s++) binarize_slice(s);
    };
    for (int s = 0; s < ns; s++)   // K4c quarter-pel refinement once, before the first pass
        if (fe.tasks[s].final_action == ACT_P && fe.cfg.subpel) fe.subpel_refine(s);   // k_subpel
    code_picture();
    const bool idr = fe.ctl_.picture_is_idr(fe.tasks.data());
    if (idr) poc = 0;
    std::vector<std::vector<uint8_t>> nals(ns);
    auto write_picture = [&] {
        payload_bytes_ = 0;
        for (int s = 0; s < ns; s++) nals[s] = write_slice(s, idr);
    };
    write_picture();
    // K10 per-frame cap (ratecontrol.h rc_frame_cap): a frame over it is coded again,
    // coarser, up to twice (k_rc_guard_sizes gates the GPU back end's passes the same way)
    for (int r = 0; r < h264::kMaxRecodes && fe.ctl_.rate_redo(fe.tasks.data(), 8 * payload_bytes_); r++) {
        code_picture();
        write_picture();
    }
    h264::EncodedPacket pk;
    pk.y = 0;
    pk.w = fe.g.W;
    pk.h = fe.g.H;
    pk.key = idr;
    pk.data.resize(10);
    h264::write_stripe_header(pk.data.data(), idr, frame_id, 0, fe.g.W, fe.g.H);
    if (idr) pk.data.insert(pk.data.end(), param_sets.begin(), param_sets.end());
    for (int s = 0; s < ns; s++) pk.data.insert(pk.data.end(), nals[s].begin(), nals[s].end());
    fe.ctl_.rate_account(8 * payload_bytes_);   // K10: substream payload (k_rc_account: sub_size)
    out.push_back(std::move(pk));
    sao_apply();   // the SAO output becomes the reference
    fe.finish_frame();
    poc++;
}

}  // namespace hevc
}  // namespace sk
