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

void build_intra_ref(const uint8_t* plane, int stride, int x0, int y0, int n, bool left, bool top, bool tr,
                     uint8_t* ref) {
    uint8_t av[4 * 32 + 1];
    const int len = 4 * n + 1;
    memset(av, 0, (size_t)len);
    memset(ref, 0, (size_t)len);
    // left column p[-1][y], y = 0..n-1 at ref[2n-1-y]; below-left (y >= n) never available
    if (left)
        for (int y = 0; y < n; y++) {
            ref[2 * n - 1 - y] = plane[(size_t)(y0 + y) * stride + x0 - 1];
            av[2 * n - 1 - y] = 1;
        }
    if (left && top) {
        ref[2 * n] = plane[(size_t)(y0 - 1) * stride + x0 - 1];
        av[2 * n] = 1;
    }
    if (top)
        for (int x = 0; x < n; x++) {
            ref[2 * n + 1 + x] = plane[(size_t)(y0 - 1) * stride + x0 + x];
            av[2 * n + 1 + x] = 1;
        }
    if (tr)
        for (int x = n; x < 2 * n; x++) {
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
std::vector<uint8_t> pc_code_row_host(const std::vector<std::vector<uint16_t>>& cu, const uint8_t* init_ctx) {
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
    const int n = geo.ctbs();
    cus.assign(n, CuInfo());
    coefs.assign((size_t)n * kCoefPerCu, 0);
    bins.assign((size_t)n * kCuBinCap, 0);
    bin_n.assign(n, 0);
    sao_stats.assign((size_t)3 * n, SaoStats{});
    sao_own.assign(n, SaoParams{});
    sao.assign(n, SaoParams{});
    sao_cost.assign(n, 0);
    sao_md.assign((size_t)n * kSaoMd, 0);
    build_parameter_sets(fe.g.W, fe.g.H, cfg.full_range, cfg.fps, param_sets);
}

void CpuHevcEncoder::load_cu_src(int cx, int cy, uint8_t* y, uint8_t* u, uint8_t* v) const {
    const h264::Geometry& g = fe.g;
    for (int r = 0; r < 16; r++) memcpy(y + r * 16, &fe.src[0][(size_t)(cy * 16 + r) * g.stride_y + cx * 16], 16);
    for (int r = 0; r < 8; r++) {
        memcpy(u + r * 8, &fe.src[1][(size_t)(cy * 8 + r) * g.stride_c + cx * 8], 8);
        memcpy(v + r * 8, &fe.src[2][(size_t)(cy * 8 + r) * g.stride_c + cx * 8], 8);
    }
}

// Transform + quantisation of one TU from source and prediction; returns cbf and
// writes the reconstruction.
static int code_tu(const uint8_t* src, const uint8_t* pred, int log2n, int qp, bool intra, int16_t* lev,
                   uint8_t* rec) {
    const int n = 1 << log2n, nn = n * n;
    int res[256], c[256], d[256], r[256];
    for (int i = 0; i < nn; i++) res[i] = (int)src[i] - (int)pred[i];
    fwd_transform(res, log2n, c);
    int nz = 0;
    for (int i = 0; i < nn; i++) {
        const int l = quant_level(c[i], qp, log2n, intra);
        lev[i] = (int16_t)l;
        nz |= l;
        d[i] = dequant_level(l, qp, log2n);
    }
    if (nz) {
        inv_transform(d, log2n, r);
        for (int i = 0; i < nn; i++) rec[i] = (uint8_t)sk_clip255(pred[i] + r[i]);
    } else {
        memcpy(rec, pred, (size_t)nn);
    }
    return nz != 0;
}

void CpuHevcEncoder::code_slice_inter(int s) {
    const SliceTask& t = fe.tasks[s];
    const h264::Geometry& g = fe.g;
    const int qp = t.qp, qpc = chroma_qp(qp);
    for (int cy = t.first_row; cy < t.first_row + t.num_rows; cy++)
        for (int cx = 0; cx < geo.ctb_w; cx++) {
            const int idx = cy * geo.ctb_w + cx;
            CuInfo& cu = cus[idx];
            memset(&cu, 0, sizeof(cu));
            const int mvx = h264::me_qx(fe.me[idx]), mvy = h264::me_qy(fe.me[idx]);   // quarter-pel (K4c)
            auto nb = [&](int ox, int oy, bool ok) {
                NbMv m;
                m.av = ok;
                m.mvx = ok ? h264::me_qx(fe.me[oy * geo.ctb_w + ox]) : 0;
                m.mvy = ok ? h264::me_qy(fe.me[oy * geo.ctb_w + ox]) : 0;
                return m;
            };
            const bool top = cy > t.first_row;
            const NbMv A1 = nb(cx - 1, cy, cx > 0), B1 = nb(cx, cy - 1, top);
            const NbMv B0 = nb(cx + 1, cy - 1, top && cx + 1 < geo.ctb_w), B2 = nb(cx - 1, cy - 1, top && cx > 0);
            int mlx[kMaxMergeCand], mly[kMaxMergeCand], px[2], py[2];
            merge_list(A1, B1, B0, B2, mlx, mly);
            amvp_list(A1, B1, B0, B2, px, py);
            uint8_t sy[256], su[64], sv[64], pry[256], pru[64], prv[64];
            load_cu_src(cx, cy, sy, su, sv);
            for (int y = 0; y < 16; y++)
                for (int x = 0; x < 16; x++)
                    pry[y * 16 + x] = (uint8_t)luma_mc_sample(fe.ref[0].data(), g.stride_y, geo.pic_w, geo.pic_h,
                                                              cx * 16 + x, cy * 16 + y, mvx, mvy);
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    pru[y * 8 + x] = (uint8_t)chroma_mc_sample(fe.ref[1].data(), g.stride_c, g.stride_c, g.plane_h_c,
                                                               cx * 8 + x, cy * 8 + y, mvx, mvy);
                    prv[y * 8 + x] = (uint8_t)chroma_mc_sample(fe.ref[2].data(), g.stride_c, g.stride_c, g.plane_h_c,
                                                               cx * 8 + x, cy * 8 + y, mvx, mvy);
                }
            int16_t* lev = &coefs[(size_t)idx * kCoefPerCu];
            uint8_t ry[256], ru[64], rv[64];
            int cbf = code_tu(sy, pry, 4, qp, false, lev, ry);
            cbf |= code_tu(su, pru, 3, qpc, false, lev + kCoefCb, ru) << 1;
            cbf |= code_tu(sv, prv, 3, qpc, false, lev + kCoefCr, rv) << 2;
            int midx = -1;
            for (int i = 0; i < kMaxMergeCand && midx < 0; i++)
                if (mlx[i] == mvx && mly[i] == mvy) midx = i;
            cu.cbf = (uint8_t)cbf;
            cu.qp = (uint8_t)qp;
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
            for (int y = 0; y < 16; y++)
                memcpy(&fe.rec[0][(size_t)(cy * 16 + y) * g.stride_y + cx * 16], ry + y * 16, 16);
            for (int y = 0; y < 8; y++) {
                memcpy(&fe.rec[1][(size_t)(cy * 8 + y) * g.stride_c + cx * 8], ru + y * 8, 8);
                memcpy(&fe.rec[2][(size_t)(cy * 8 + y) * g.stride_c + cx * 8], rv + y * 8, 8);
            }
        }
}

// I slices in two passes, like the H.264 intra path: (1) every CU independently
// chooses its mode against the SOURCE neighbours (parallel on the GPU), (2) the
// CTB wavefront predicts from the reconstruction with that mode.
void CpuHevcEncoder::code_slice_intra(int s) {
    const SliceTask& t = fe.tasks[s];
    const h264::Geometry& g = fe.g;
    const int qp = t.qp, qpc = chroma_qp(qp);
    for (int pass = 0; pass < 2; pass++)
        for (int cy = t.first_row; cy < t.first_row + t.num_rows; cy++)
            for (int cx = 0; cx < geo.ctb_w; cx++) {
                const int idx = cy * geo.ctb_w + cx;
                CuInfo& cu = cus[idx];
                const bool left = cx > 0, top = cy > t.first_row, tr = top && cx + 1 < geo.ctb_w;
                const std::vector<uint8_t>* P = pass == 0 ? fe.src : fe.rec;
                uint8_t sy[256], su[64], sv[64];
                load_cu_src(cx, cy, sy, su, sv);
                uint8_t refy[65], refu[33], refv[33];
                build_intra_ref(P[0].data(), g.stride_y, cx * 16, cy * 16, 16, left, top, tr, refy);
                if (pass == 0) {
                    int best = 1, best_sad = 0x7fffffff;
                    for (int k = 0; k < 35; k++) {   // HEVC_INTRA_ORDER, SAD + intra_mode_bias
                        const int m = HEVC_INTRA_ORDER[k];
                        uint8_t pr[256];
                        intra_predict(refy, 4, m, 0, pr);
                        int sad = intra_mode_bias(m, qp);
                        for (int i = 0; i < 256; i++) sad += sk_abs((int)sy[i] - (int)pr[i]);
                        if (sad < best_sad) { best_sad = sad; best = m; }
                    }
                    memset(&cu, 0, sizeof(cu));
                    cu.mode = CU_INTRA;
                    cu.intra_mode = (uint8_t)best;
                    continue;
                }
                build_intra_ref(P[1].data(), g.stride_c, cx * 8, cy * 8, 8, left, top, tr, refu);
                build_intra_ref(P[2].data(), g.stride_c, cx * 8, cy * 8, 8, left, top, tr, refv);
                const int mode = cu.intra_mode;
                uint8_t pry[256], pru[64], prv[64];
                intra_predict(refy, 4, mode, 0, pry);
                intra_predict(refu, 3, mode, 1, pru);
                intra_predict(refv, 3, mode, 2, prv);
                int16_t* lev = &coefs[(size_t)idx * kCoefPerCu];
                uint8_t ry[256], ru[64], rv[64];
                int cbf = code_tu(sy, pry, 4, qp, true, lev, ry);
                cbf |= code_tu(su, pru, 3, qpc, true, lev + kCoefCb, ru) << 1;
                cbf |= code_tu(sv, prv, 3, qpc, true, lev + kCoefCr, rv) << 2;
                cu.cbf = (uint8_t)cbf;
                cu.qp = (uint8_t)qp;
                fe.me[idx].mvx = fe.me[idx].mvy = 0;
                fe.me[idx].ref = 0;
                fe.me[idx].fx = fe.me[idx].fy = 0;
                for (int y = 0; y < 16; y++)
                    memcpy(&fe.rec[0][(size_t)(cy * 16 + y) * g.stride_y + cx * 16], ry + y * 16, 16);
                for (int y = 0; y < 8; y++) {
                    memcpy(&fe.rec[1][(size_t)(cy * 8 + y) * g.stride_c + cx * 8], ru + y * 8, 8);
                    memcpy(&fe.rec[2][(size_t)(cy * 8 + y) * g.stride_c + cx * 8], rv + y * 8, 8);
                }
            }
}

void CpuHevcEncoder::code_slice_skip(int s) {
    const SliceTask& t = fe.tasks[s];
    fe.code_slice_skipall(s);   // motion field zero, reconstruction = reference
    for (int cy = t.first_row; cy < t.first_row + t.num_rows; cy++)
        for (int cx = 0; cx < geo.ctb_w; cx++) {
            CuInfo& cu = cus[cy * geo.ctb_w + cx];
            memset(&cu, 0, sizeof(cu));
            cu.mode = CU_SKIP;
            cu.qp = (uint8_t)t.qp;
        }
}

// Plane geometry for SAO: plane 0 luma (CTB 16), 1 / 2 chroma (CTB 8).
static SaoPlane sao_plane(const Geo& geo, int c) {
    const int n = c ? 8 : 16;
    return SaoPlane{geo.ctb_w * n, geo.ctb_h * n, n, geo.rows_per_slice};
}

void CpuHevcEncoder::sao_analyse() {
    const h264::Geometry& g = fe.g;
    for (int cy = 0; cy < geo.ctb_h; cy++)
        for (int cx = 0; cx < geo.ctb_w; cx++) {
            const int idx = cy * geo.ctb_w + cx;
            // skip-all slices keep the reference as it is (finish_frame does not copy them
            // back): their stats stay empty, so every CTB there decides "off"
            const int act = fe.tasks[cy / geo.rows_per_slice].final_action;
            const bool coded = act == ACT_P || act == ACT_I;
            for (int c = 0; c < 3; c++) {
                SaoStats& st = sao_stats[(size_t)3 * idx + c];
                st = SaoStats{};
                if (!coded) continue;
                const SaoPlane pl = sao_plane(geo, c);
                const int stride = c ? g.stride_c : g.stride_y;
                for (int y = cy * pl.n; y < (cy + 1) * pl.n; y++)
                    for (int x = cx * pl.n; x < (cx + 1) * pl.n; x++)
                        sao_collect(st, pl, fe.rec[c].data(), stride, x, y, fe.src[c][(size_t)y * stride + x]);
            }
            const int lam = sao_lambda(fe.tasks[cy / geo.rows_per_slice].qp);
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
        const SliceTask& t = fe.tasks[cy / geo.rows_per_slice];
        const size_t o = (size_t)cy * geo.ctb_w;
        sao_row_merge(&sao_md[o * kSaoMd], &sao_own[o], &sao_cost[o], geo.ctb_w, t.qp, cy > t.first_row, &sao[o]);
    }
}

void CpuHevcEncoder::sao_apply() {
    const h264::Geometry& g = fe.g;
    for (int c = 0; c < 3; c++) {
        const SaoPlane pl = sao_plane(geo, c);
        const int stride = c ? g.stride_c : g.stride_y;
        const std::vector<uint8_t> dbk = fe.rec[c];   // the filter reads deblocked samples only
        for (int y = 0; y < pl.h; y++)
            for (int x = 0; x < pl.w; x++) {
                const SaoParams& p = sao[(size_t)(y / pl.n) * geo.ctb_w + x / pl.n];
                fe.rec[c][(size_t)y * stride + x] = (uint8_t)sao_apply_sample(p, c, pl, dbk.data(), stride, x, y);
            }
    }
}

void CpuHevcEncoder::binarize_slice(int s) {
    const SliceTask& t = fe.tasks[s];
    const bool p_slice = t.final_action != ACT_I;
    const int last_row = t.first_row + t.num_rows - 1;
    for (int cy = t.first_row; cy <= last_row; cy++)
        for (int cx = 0; cx < geo.ctb_w; cx++) {
            const int idx = cy * geo.ctb_w + cx;
            const bool left = cx > 0, top = cy > t.first_row;
            const int skip_ctx = (left && cus[idx - 1].mode == CU_SKIP) + (top && cus[idx - geo.ctb_w].mode == CU_SKIP);
            const int cand_a = (left && cus[idx - 1].mode == CU_INTRA) ? cus[idx - 1].intra_mode : 1;
            BinBuf w{&bins[(size_t)idx * kCuBinCap], 0};
            sao_bins(w, sao[idx], left, top);   // CTB-level SAO syntax before the coding quadtree
            code_cu(w, cus[idx], &coefs[(size_t)idx * kCoefPerCu], p_slice, skip_ctx, cand_a);
            w.term(cy == last_row && cx == geo.ctb_w - 1);   // end_of_slice_segment_flag
            bin_n[idx] = w.n;
        }
}

std::vector<uint8_t> CpuHevcEncoder::write_slice(int s, bool idr) {
    const SliceTask& t = fe.tasks[s];
    const bool p_slice = t.final_action != ACT_I;
    const int rows = t.num_rows;
    std::vector<std::vector<uint8_t>> sub(rows);
    uint8_t sync[CTX_COUNT];
    for (int r = 0; r < rows; r++) {
        const int cy = t.first_row + r;
        uint8_t ctx[CTX_COUNT];
        if (r == 0 || geo.ctb_w < 2) ctx_init_all(ctx, p_slice ? 1 : 0, t.qp);
        else memcpy(ctx, sync, CTX_COUNT);
        if (pc_host_) {   // chunk-parallel model (hevc_pcabac.h), must give the same bytes
            std::vector<std::vector<uint16_t>> cu(geo.ctb_w);
            for (int cx = 0; cx < geo.ctb_w; cx++) {
                const uint16_t* b = &bins[(size_t)(cy * geo.ctb_w + cx) * kCuBinCap];
                cu[cx].assign(b, b + bin_n[cy * geo.ctb_w + cx]);
            }
            if (r + 1 < rows) cu.back().push_back((uint16_t)((1u << 8) | CTX_TERM));   // end_of_subset_one_bit
            sub[r] = pc_code_row_host(cu, ctx);
            for (int cx = 0; cx < 2 && cx < geo.ctb_w; cx++)
                for (int i = 0; i < bin_n[cy * geo.ctb_w + cx]; i++) {
                    const uint16_t e = bins[(size_t)(cy * geo.ctb_w + cx) * kCuBinCap + i];
                    if ((e & 0x80ffu) < (uint32_t)CTX_TERM) ctx_update(ctx[e & 0xffu], (e >> 8) & 1);
                }
            memcpy(sync, ctx, CTX_COUNT);
            payload_bytes_ += (long long)sub[r].size();
            continue;
        }
        size_t cap = 64;
        for (int cx = 0; cx < geo.ctb_w; cx++) cap += (size_t)bin_n[cy * geo.ctb_w + cx] * 2 + 8;
        sub[r].assign(cap, 0);
        CabacEncoder e;
        e.start(sub[r].data());
        for (int cx = 0; cx < geo.ctb_w; cx++) {
            const int idx = cy * geo.ctb_w + cx;
            const uint16_t* b = &bins[(size_t)idx * kCuBinCap];
            for (int i = 0; i < bin_n[idx]; i++) e.code_entry(b[i], ctx);
            if (cx == 1) memcpy(sync, ctx, CTX_COUNT);   // WPP storage after the second CTB
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
    h.first_slice = s == 0;
    h.idr = idr;
    h.address = t.first_row * geo.ctb_w;
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
    for (int s = 0; s < ns; s++) {
        switch (fe.tasks[s].final_action) {
            case ACT_P:
                if (fe.cfg.subpel) fe.subpel_refine(s);   // k_subpel
                code_slice_inter(s);
                break;
            case ACT_I: code_slice_intra(s); break;
            default: code_slice_skip(s); break;
        }
    }
    // in-loop deblocking, then SAO decisions on the deblocked picture (they are syntax of
    // every CTB, so the binarisation follows them)
    deblock_picture(fe.rec[0].data(), fe.rec[1].data(), fe.rec[2].data(), fe.g.stride_y, fe.g.stride_c, cus.data(),
                    geo.ctb_w, geo.ctb_h, geo.rows_per_slice);
    sao_analyse();
    for (int s = 0; s < ns; s++) binarize_slice(s);
    const bool idr = fe.ctl_.picture_is_idr(fe.tasks.data());
    if (idr) poc = 0;
    h264::EncodedPacket pk;
    pk.y = 0;
    pk.w = fe.g.W;
    pk.h = fe.g.H;
    pk.key = idr;
    pk.data.resize(10);
    h264::write_stripe_header(pk.data.data(), idr, frame_id, 0, fe.g.W, fe.g.H);
    if (idr) pk.data.insert(pk.data.end(), param_sets.begin(), param_sets.end());
    payload_bytes_ = 0;
    for (int s = 0; s < ns; s++) {
        std::vector<uint8_t> nal = write_slice(s, idr);
        pk.data.insert(pk.data.end(), nal.begin(), nal.end());
    }
    fe.ctl_.rate_account(8 * payload_bytes_);   // K10: substream payload (k_rc_account: sub_size)
    out.push_back(std::move(pk));
    sao_apply();   // the SAO output becomes the reference
    fe.finish_frame();
    poc++;
}

}  // namespace hevc
}  // namespace sk
