// H.265 sample adaptive offset (SAO, 7.3.8.3 / 8.7.3) shared by the CPU reference
// (hevc_cpu.cpp) and the gfx950 kernels (k_hevc_sao_stats / k_hevc_sao_row /
// k_hevc_sao_apply): per-CTB statistics of the deblocked picture against the source,
// the encoder's parameter decision, the CTB syntax binarisation and the normative
// filter itself. Slices are stripes of whole CTB rows and
// pps_loop_filter_across_slices_enabled_flag is 0, so an edge-offset neighbour in another
// slice (or outside the picture) leaves the sample unchanged.
#pragma once
#include <cstddef>
#include "hevc_core.h"

namespace sk {
namespace hevc {

enum SaoType : uint8_t { SAO_OFF = 0, SAO_BAND = 1, SAO_EDGE = 2 };

// Statistics of one component of one CTB over the samples SAO may change:
// sum of (source - deblocked) and the count, per edge class and category 1..4, per band.
struct SaoStats {
    int32_t eo_s[4][4], eo_n[4][4];
    int32_t bo_s[32], bo_n[32];
};
constexpr int kSaoStatsInts = 96;
static_assert(sizeof(SaoStats) == kSaoStatsInts * 4, "SaoStats layout");

// Parameters of one CTB (Cr shares type and class with Cb). off[c][k] = SaoOffsetVal[k + 1].
struct SaoParams {
    uint8_t type[3];
    uint8_t eo_class[3];
    uint8_t band_pos[3];
    uint8_t merge_left;
    int8_t off[3][4];
    int32_t pad;
};
static_assert(sizeof(SaoParams) == 28, "SaoParams layout");

// Edge class neighbour offsets (Table 8-? hPos / vPos): 0 horizontal, 1 vertical, 2 135 deg, 3 45 deg.
SK_HD int sao_dx(int cls, int i) { return cls == 1 ? 0 : (cls == 3 ? (i ? -1 : 1) : (i ? 1 : -1)); }
SK_HD int sao_dy(int cls, int i) { return cls == 0 ? 0 : (i ? 1 : -1); }
SK_HD int sk_sign(int v) { return (v > 0) - (v < 0); }
// edgeIdx (8.7.3.2): 2 + sign(c - a) + sign(c - b), {0,1,2} -> {1,2,0}; 0 = unchanged.
SK_HD int sao_edge_idx(int c, int a, int b) {
    const int e = 2 + sk_sign(c - a) + sk_sign(c - b);
    return e <= 2 ? (e == 2 ? 0 : e + 1) : e;
}

// Geometry of one plane for SAO: w x h samples, CTB side n (16 luma / 8 chroma), and
// the picture's slice layout (SliceMap, hevc_core.h).
struct SaoPlane {
    int w, h, n;
    SliceMap m;
    // Whether an edge-offset class may change sample (x, y): both neighbours inside the
    // picture and in the sample's slice.
    SK_HD bool eo_ok(int cls, int x, int y) const {
        const int s = m.id(x / n, y / n);
        for (int i = 0; i < 2; i++) {
            const int xx = x + sao_dx(cls, i), yy = y + sao_dy(cls, i);
            if (xx < 0 || yy < 0 || xx >= w || yy >= h || m.id(xx / n, yy / n) != s) return false;
        }
        return true;
    }
};

// Adds sample (x, y) of the deblocked plane `rec` with source value `src` to the stats.
SK_HD void sao_collect(SaoStats& st, const SaoPlane& g, const uint8_t* rec, int stride, int x, int y, int src) {
    const int c = rec[(size_t)y * stride + x], d = src - c;
    st.bo_s[c >> 3] += d;
    st.bo_n[c >> 3] += 1;
    for (int cls = 0; cls < 4; cls++) {
        if (!g.eo_ok(cls, x, y)) continue;
        const int a = rec[(size_t)(y + sao_dy(cls, 0)) * stride + x + sao_dx(cls, 0)];
        const int b = rec[(size_t)(y + sao_dy(cls, 1)) * stride + x + sao_dx(cls, 1)];
        const int e = sao_edge_idx(c, a, b);
        if (e) {
            st.eo_s[cls][e - 1] += d;
            st.eo_n[cls][e - 1] += 1;
        }
    }
}

// SAO lambda in Q4 per QP: 16 * 0.57 * 2^((QP - 12) / 3) (the HM rate-distortion lambda
// for SSE distortion); costs below are 16 * SSE change + lambda * bits.
SK_TABLE int32_t SAO_LAMBDA_Q4[52] = {1,    1,    1,    1,    1,    2,    2,    3,    4,     5,     6,     7,    9,
                                      11,   14,   18,   23,   29,   36,   46,   58,   73,    92,    116,   146,  184,
                                      232,  292,  368,  463,  584,  735,  927,  1167, 1471,  1853,  2335,  2942, 3706,
                                      4669, 5883, 7412, 9339, 11766, 14825, 18678, 23533, 29649, 37356, 47065, 59298, 74711};
// sao_offset_abs bins: TR, cMax 7.
SK_HD int sao_abs_bins(int a) { return a < 7 ? a + 1 : 7; }
// 16 * SSE change of offset o on a category with sum s and count n.
SK_HD long long sao_dist(int o, int s, int n) { return 16ll * ((long long)n * o * o - 2ll * o * s); }

// Best offset of one category: o in [lo, hi], minimising distortion + lambda * bins
// (+ one sign bin for a non-zero band offset). First minimum from o = 0 outward wins.
SK_HD long long sao_best_offset(int s, int n, int lo, int hi, bool sign_bin, int lam, int* best_o) {
    long long best = 0;
    int bo = 0;
    best = (long long)lam * sao_abs_bins(0);
    for (int m = 1; m <= 7; m++)
        for (int sg = 0; sg < 2; sg++) {
            const int o = sg ? -m : m;
            if (o < lo || o > hi) continue;
            const long long c = sao_dist(o, s, n) + (long long)lam * (sao_abs_bins(m) + (sign_bin ? 1 : 0));
            if (c < best) { best = c; bo = o; }
        }
    *best_o = bo;
    return best;
}

// Own parameters of one CTB, in two steps so the GPU can run the first one lane-parallel:
// (1) sao_tables: the best offset and its cost for every edge category (component, class,
// category) and every band, and the cost of every 4-band window; (2) sao_pick: per
// component group (luma; Cb + Cr, which share type and class) the cheapest of off / each
// edge class / the best band windows, first minimum in that order. Costs are
// 16 * SSE change + lambda * bins.
struct SaoTables {
    long long eo_c[3][4][4];
    long long bo_c[3][32];
    long long win[3][32];
    int8_t eo_o[3][4][4];
    int8_t bo_o[3][32];
};
// Entry `i` of the best-offset tables: i < 48 edge (c, cls, k), else band (c, b).
SK_HD void sao_table_entry(const SaoStats* st, int lam, int i, SaoTables& t) {
    int o;
    if (i < 48) {
        const int c = i >> 4, cls = (i >> 2) & 3, k = i & 3;
        t.eo_c[c][cls][k] = sao_best_offset(st[c].eo_s[cls][k], st[c].eo_n[cls][k], k < 2 ? 0 : -7, k < 2 ? 7 : 0,
                                            false, lam, &o);
        t.eo_o[c][cls][k] = (int8_t)o;
    } else {
        const int c = (i - 48) >> 5, b = (i - 48) & 31;
        t.bo_c[c][b] = sao_best_offset(st[c].bo_s[b], st[c].bo_n[b], -7, 7, true, lam, &o);
        t.bo_o[c][b] = (int8_t)o;
    }
}
constexpr int kSaoTableEntries = 48 + 96;
// Window `i` (c = i >> 5, position i & 31): band_position (5 bits) + its four bands.
SK_HD void sao_window(int lam, int i, SaoTables& t) {
    const int c = i >> 5, ps = i & 31;
    long long w = (long long)lam * 5;
    for (int k = 0; k < 4; k++) w += t.bo_c[c][(ps + k) & 31];
    t.win[c][ps] = w;
}
SK_HD long long sao_pick(const SaoTables& t, int lam, SaoParams& p) {
    p.merge_left = 0;
    p.pad = 0;
    long long total = 0;
    for (int grp = 0; grp < 2; grp++) {   // 0: luma, 1: Cb + Cr
        const int c0 = grp ? 1 : 0, c1 = grp ? 2 : 0;
        long long best = (long long)lam * 1;   // sao_type_idx = 0: one bin
        int btype = SAO_OFF, bcls = 0;
        for (int cls = 0; cls < 4; cls++) {
            long long cost = (long long)lam * 4;   // type (2 bins) + class (2 bits, once per group)
            for (int c = c0; c <= c1; c++)
                for (int k = 0; k < 4; k++) cost += t.eo_c[c][cls][k];
            if (cost < best) { best = cost; btype = SAO_EDGE; bcls = cls; }
        }
        long long bcost = (long long)lam * 2;
        int bpos[3] = {0, 0, 0};
        for (int c = c0; c <= c1; c++) {
            long long wbest = t.win[c][0];
            for (int ps = 1; ps < 32; ps++)
                if (t.win[c][ps] < wbest) { wbest = t.win[c][ps]; bpos[c] = ps; }
            bcost += wbest;
        }
        if (bcost < best) { best = bcost; btype = SAO_BAND; }
        bool any = false;
        for (int c = c0; c <= c1; c++) {
            p.type[c] = (uint8_t)btype;
            p.eo_class[c] = (uint8_t)(btype == SAO_EDGE ? bcls : 0);
            p.band_pos[c] = (uint8_t)(btype == SAO_BAND ? bpos[c] : 0);
            for (int k = 0; k < 4; k++) {
                const int o = btype == SAO_EDGE ? t.eo_o[c][bcls][k]
                                                : (btype == SAO_BAND ? t.bo_o[c][(bpos[c] + k) & 31] : 0);
                p.off[c][k] = (int8_t)o;
                any |= o != 0;
            }
        }
        if (!any) {   // an "on" set whose offsets are all zero is worse than off
            best = (long long)lam * 1;
            for (int c = c0; c <= c1; c++) p.type[c] = p.eo_class[c] = p.band_pos[c] = 0;
        }
        total += best;
    }
    return total;
}
// x 45 / 64: the SAO decisions' rate term at 0.7 of the table (tools/rd_codecs.py content,
// CTB-32 quadtree: -0.8 % / -1.0 % BD-rate with the intra mode bias at 2 lambda)
SK_HD int sao_lambda(int qp) { return sk_max((SAO_LAMBDA_Q4[sk_clip(qp, 0, 51)] * 45) >> 6, 1); }

// Distortion change (16 * SSE) of parameter set p on a CTB's stats (merge evaluation).
SK_HD long long sao_params_dist(const SaoStats* st, const SaoParams& p) {
    long long d = 0;
    for (int c = 0; c < 3; c++) {
        if (p.type[c] == SAO_EDGE)
            for (int k = 0; k < 4; k++) d += sao_dist(p.off[c][k], st[c].eo_s[p.eo_class[c]][k], st[c].eo_n[p.eo_class[c]][k]);
        else if (p.type[c] == SAO_BAND)
            for (int k = 0; k < 4; k++) {
                const int b = (p.band_pos[c] + k) & 31;
                d += sao_dist(p.off[c][k], st[c].bo_s[b], st[c].bo_n[b]);
            }
    }
    return d;
}
// Equal types, classes, band positions and offsets (merge_left and the padding aside):
// six masked words instead of 21 byte compares (the sequential SAO merge chain runs it).
SK_HD bool sao_same(const SaoParams& a, const SaoParams& b) {
    static_assert(offsetof(SaoParams, merge_left) == 9 && offsetof(SaoParams, off) == 10, "SaoParams layout");
    const uint32_t* x = reinterpret_cast<const uint32_t*>(&a);
    const uint32_t* y = reinterpret_cast<const uint32_t*>(&b);
    return x[0] == y[0] && x[1] == y[1] && ((x[2] ^ y[2]) & 0xffff00ffu) == 0 && x[3] == y[3] && x[4] == y[4] &&
           ((x[5] ^ y[5]) & 0x0000ffffu) == 0;
}

// Merge decision along one CTB row (sequential: a merged CTB copies its left neighbour's
// final parameters, i.e. the own parameters of the CTB the run started at). The
// distortion of those parameters on CTB x comes precomputed (all CTBs in parallel):
// md[x][j] = sao_params_dist(stats of x, own[x - 1 - j]) for j < kSaoMergeWin, and
// md[x][kSaoMergeWin] = the own parameters' distortion. A run that started further back
// is continued only with identical parameters (then merging is never worse).
// Merge-up is never chosen (rows stay independent); its flag is still coded as 0.
constexpr int kSaoMergeWin = 8;
constexpr int kSaoMd = kSaoMergeWin + 1;
SK_HD void sao_merge_dists(const SaoStats* st_x, const SaoParams* own_row, int x, long long* md) {
    for (int j = 0; j < kSaoMergeWin; j++) md[j] = x - 1 - j >= 0 ? sao_params_dist(st_x, own_row[x - 1 - j]) : 0;
    md[kSaoMergeWin] = sao_params_dist(st_x, own_row[x]);
}
// m / cy: the row's slices (a CTB merges left only inside its slice, and codes the
// merge-up flag only under a CTB of its slice).
// The decisions alone: sel[x] = the CTB whose own parameters CTB x takes, bit 15 set when
// x merges left (the GPU runs this on one lane and copies the parameters with all 64).
// fl[x]: bit 0 = CTB x has a left neighbour in its slice, bit 1 = an upper one (the slice
// map's tests, precomputed so the sequential chain does not evaluate them).
SK_HD uint8_t sao_row_flags(const SliceMap& m, int cy, int x) {
    return (uint8_t)((m.left(x, cy) ? 1 : 0) | (m.top(x, cy) ? 2 : 0));
}
SK_HD void sao_row_decide(const long long* md_row, const SaoParams* own, const long long* own_cost, int ctb_w, int qp,
                          const uint8_t* fl, uint16_t* sel) {
    const int lam = sao_lambda(qp);
    int src = 0;   // CTB whose own parameters the previous CTB's final parameters are
    for (int x = 0; x < ctb_w; x++) {
        int sx = x;
        uint16_t merge = 0;
        if (fl[x] & 1) {
            const int j = x - 1 - src;
            const long long* md = md_row + (size_t)x * kSaoMd;
            bool ok = true;
            long long dm = 0;
            if (j < kSaoMergeWin) dm = md[j];
            else if (sao_same(own[x], own[src])) dm = md[kSaoMergeWin];
            else ok = false;
            const long long cown = own_cost[x] + (long long)lam * ((fl[x] & 2) ? 2 : 1);   // merge_left = 0 (+ merge_up = 0)
            if (ok && dm + (long long)lam * 1 < cown) {
                sx = src;
                merge = 0x8000;
            }
        }
        sel[x] = (uint16_t)(sx | merge);
        src = sx;
    }
}
SK_HD void sao_row_apply_sel(const SaoParams* own, uint16_t sel, SaoParams* out) {
    SaoParams p = own[sel & 0x7fff];
    p.merge_left = (sel >> 15) & 1;
    *out = p;
}
SK_HD void sao_row_merge(const long long* md_row, const SaoParams* own, const long long* own_cost, int ctb_w, int qp,
                         const SliceMap& m, int cy, SaoParams* out, uint16_t* sel, uint8_t* fl) {
    for (int x = 0; x < ctb_w; x++) fl[x] = sao_row_flags(m, cy, x);
    sao_row_decide(md_row, own, own_cost, ctb_w, qp, fl, sel);
    for (int x = 0; x < ctb_w; x++) sao_row_apply_sel(own, sel[x], out + x);
}

// CTB syntax sao(rx, ry) (7.3.8.3) as bin entries. left/up: the neighbour CTB exists in
// this slice.
template <class W>
SK_HD void sao_bins(W& w, const SaoParams& p, bool left, bool up) {
    if (left) w.ctx(CTX_SAO_MERGE, p.merge_left);
    if (p.merge_left) return;
    if (up) w.ctx(CTX_SAO_MERGE, 0);
    for (int c = 0; c < 3; c++) {
        const int t = p.type[c];
        if (c < 2) {   // sao_type_idx: TR cMax 2, first bin context, second bypass
            w.ctx(CTX_SAO_TYPE, t != SAO_OFF);
            if (t != SAO_OFF) w.bypass(t == SAO_EDGE ? 1u : 0u, 1);
        }
        if (t == SAO_OFF) continue;
        for (int k = 0; k < 4; k++) {   // sao_offset_abs: TR cMax 7, bypass
            const int a = sk_abs(p.off[c][k]);
            w.bypass(a < 7 ? ((1u << (a + 1)) - 2u) : 0x7fu, a < 7 ? a + 1 : 7);
        }
        if (t == SAO_BAND) {
            for (int k = 0; k < 4; k++)
                if (p.off[c][k]) w.bypass(p.off[c][k] < 0 ? 1u : 0u, 1);
            w.bypass(p.band_pos[c], 5);
        } else if (c < 2) {
            w.bypass(p.eo_class[c], 2);
        }
    }
}

// Normative filter (8.7.3) for sample (x, y) of a plane: the deblocked value and its
// neighbours come from `rec`; returns the SAO output.
// off[c][k] through a packed word and a shift: a run-time index into the array keeps the
// parameters in GPU scratch memory
SK_HD int sao_off(const SaoParams& p, int c, int k) {
    const uint32_t w = (uint32_t)(uint8_t)p.off[c][0] | (uint32_t)(uint8_t)p.off[c][1] << 8 |
                       (uint32_t)(uint8_t)p.off[c][2] << 16 | (uint32_t)(uint8_t)p.off[c][3] << 24;
    return (int)(int8_t)(uint8_t)(w >> (8 * k));
}
SK_HD int sao_apply_sample(const SaoParams& p, int c, const SaoPlane& g, const uint8_t* rec, int stride, int x, int y) {
    const int v = rec[(size_t)y * stride + x];
    if (p.type[c] == SAO_BAND) {
        const int k = ((v >> 3) - p.band_pos[c]) & 31;
        return k < 4 ? sk_clip255(v + sao_off(p, c, k)) : v;
    }
    if (p.type[c] == SAO_EDGE) {
        const int cls = p.eo_class[c];
        if (!g.eo_ok(cls, x, y)) return v;
        const int a = rec[(size_t)(y + sao_dy(cls, 0)) * stride + x + sao_dx(cls, 0)];
        const int b = rec[(size_t)(y + sao_dy(cls, 1)) * stride + x + sao_dx(cls, 1)];
        const int e = sao_edge_idx(v, a, b);
        return e ? sk_clip255(v + sao_off(p, c, e - 1)) : v;
    }
    return v;
}

}  // namespace hevc
}  // namespace sk
