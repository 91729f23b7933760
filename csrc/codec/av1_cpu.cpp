// CPU reference backend of the AV1 encoder: headers and OBUs, block decisions,
// reconstruction and tile entropy coding. It is the golden model of the HIP back
// end (kernels/av1_kernels.hip produces the same decisions, levels, reconstruction
// and tile bytes) and the `use_cpu` path; dav1d decodes its output to exactly the
// reconstruction kept here (tests/test_av1_encoder.py).
#include "av1_encoder.h"
#include "av1_lf.h"
#include "av1_cdef.h"
#include <string.h>
#include <algorithm>

namespace sk {
namespace av1 {

using h264::ACT_I;
using h264::ACT_NONE;
using h264::ACT_P;
using h264::ACT_SKIPALL;

// ------------------------------------------------------------------------------ headers
void put_leb128(std::vector<uint8_t>& out, uint64_t v) {
    do {
        uint8_t b = v & 0x7f;
        v >>= 7;
        if (v) b |= 0x80;
        out.push_back(b);
    } while (v);
}

void append_obu(std::vector<uint8_t>& out, int type, const uint8_t* payload, size_t n) {
    out.push_back((uint8_t)((type << 3) | 2));   // obu_has_size_field
    put_leb128(out, n);
    out.insert(out.end(), payload, payload + n);
}

int choose_level_idx(int W, int H, float fps) {
    const double ps = (double)W * H, sr = ps * (fps > 0 ? fps : 60.0);
    struct L { int idx; double ps, sr; };
    static const L levels[] = {{0, 147456, 4423680},       {1, 278784, 8363520},       {4, 665856, 19975680},
                               {5, 1065024, 31950720},     {8, 2359296, 70778880},     {9, 2359296, 141557760},
                               {12, 8912896, 267386880},   {13, 8912896, 534773760},   {14, 8912896, 1069547520},
                               {16, 35651584, 1069547520}, {17, 35651584, 2139095040}, {18, 35651584, 4278190080.0}};
    for (const L& l : levels)
        if (ps <= l.ps && sr <= l.sr) return l.idx;
    return 31;   // unconstrained
}

// H.264 QP -> AV1 qindex with the same quantiser step (orthonormal units:
// H.264 0.625 * 2^(QP/6); AV1 Ac_Qlookup / 8).
int qidx_for_qp(int qp) {
    double step = 0.625;
    for (int i = 0; i < qp; i++) step *= 1.122462048309373;   // 2^(1/6)
    int best = 1;
    double bd = 1e30;
    for (int q = 1; q < 256; q++) {
        const double d = AV1_AC_QLOOKUP[q] / 8.0 - step;
        if ((d < 0 ? -d : d) < bd) {
            bd = d < 0 ? -d : d;
            best = q;
        }
    }
    return best;
}

void write_sequence_header(BitWriter& w, int W, int H, int level_idx, int full_range) {
    w.put(0, 3);   // seq_profile: Main
    w.put(0, 1);   // still_picture
    w.put(0, 1);   // reduced_still_picture_header
    w.put(0, 1);   // timing_info_present_flag
    w.put(0, 1);   // initial_display_delay_present_flag
    w.put(0, 5);   // operating_points_cnt_minus_1
    w.put(0, 12);  // operating_point_idc[0]
    w.put((uint32_t)level_idx, 5);
    if (level_idx > 7) w.put(0, 1);   // seq_tier: Main
    int wb = 1, hb = 1;
    while ((1 << wb) < W) wb++;
    while ((1 << hb) < H) hb++;
    w.put((uint32_t)(wb - 1), 4);
    w.put((uint32_t)(hb - 1), 4);
    w.put((uint32_t)(W - 1), wb);
    w.put((uint32_t)(H - 1), hb);
    w.put(0, 1);   // frame_id_numbers_present_flag
    w.put(0, 1);   // use_128x128_superblock
    w.put(0, 1);   // enable_filter_intra
    w.put(0, 1);   // enable_intra_edge_filter
    w.put(0, 1);   // enable_interintra_compound
    w.put(0, 1);   // enable_masked_compound
    w.put(0, 1);   // enable_warped_motion
    w.put(0, 1);   // enable_dual_filter
    w.put(0, 1);   // enable_order_hint
    w.put(1, 1);   // seq_choose_screen_content_tools: allow_screen_content_tools per frame
    w.put(0, 1);   // seq_choose_integer_mv
    w.put(0, 1);   // seq_force_integer_mv = 0 (fractional vectors)
    w.put(0, 1);   // enable_superres
    w.put(1, 1);   // enable_cdef (av1_cdef.h)
    w.put(0, 1);   // enable_restoration
    // color_config
    w.put(0, 1);   // high_bitdepth
    w.put(0, 1);   // mono_chrome
    w.put(1, 1);   // color_description_present_flag
    w.put(1, 8);   // color_primaries BT.709
    w.put(1, 8);   // transfer_characteristics BT.709
    w.put(1, 8);   // matrix_coefficients BT.709
    w.put(full_range ? 1 : 0, 1);   // color_range (h264_fullcolor)
    w.put(0, 2);   // chroma_sample_position: unknown
    w.put(0, 1);   // separate_uv_delta_q
    w.put(0, 1);   // film_grain_params_present
    w.trailing();
}

void write_frame_header(BitWriter& w, const Av1Geo& g, const FrameParams& fp) {
    w.put(0, 1);                        // show_existing_frame
    w.put(fp.key ? 0 : 1, 2);           // frame_type KEY / INTER
    w.put(1, 1);                        // show_frame
    if (!fp.key) w.put(0, 1);           // error_resilient_mode
    w.put(0, 1);                        // disable_cdf_update
    w.put(fp.screen ? 1 : 0, 1);        // allow_screen_content_tools (palette, key frames)
    w.put(0, 1);                        // frame_size_override_flag
    if (!fp.key) {
        w.put(7, 3);                    // primary_ref_frame = PRIMARY_REF_NONE
        w.put(0x01, 8);                 // refresh_frame_flags: slot 0 holds LAST
        for (int i = 0; i < 7; i++) w.put(0, 3);   // ref_frame_idx[i] = 0
        w.put(0, 1);                    // render_and_frame_size_different
        w.put(0, 1);                    // allow_high_precision_mv
        w.put(0, 1);                    // is_filter_switchable
        w.put(0, 2);                    // interpolation_filter = EIGHTTAP
        w.put(0, 1);                    // is_motion_mode_switchable
    } else {
        w.put(0, 1);                    // render_and_frame_size_different
        if (fp.screen) w.put(0, 1);     // allow_intrabc
    }
    w.put(1, 1);                        // disable_frame_end_update_cdf
    // tile_info: uniform spacing
    w.put(1, 1);
    for (int k = g.min_log2_tile_cols; k < g.max_log2_tile_cols; k++) {
        const int inc = k < g.tile_cols_log2;
        w.put((uint32_t)inc, 1);
        if (!inc) break;
    }
    const int min_log2_rows = sk_max(g.min_log2_tiles - g.tile_cols_log2, 0);
    for (int k = min_log2_rows; k < g.max_log2_tile_rows; k++) {
        const int inc = k < g.tile_rows_log2;
        w.put((uint32_t)inc, 1);
        if (!inc) break;
    }
    if (g.tile_cols_log2 > 0 || g.tile_rows_log2 > 0) {
        w.put(0, g.tile_rows_log2 + g.tile_cols_log2);   // context_update_tile_id
        w.put((uint32_t)(fp.tile_size_bytes - 1), 2);
    }
    // quantization_params
    w.put((uint32_t)fp.qidx, 8);
    w.put(0, 1);   // DeltaQYDc
    w.put(0, 1);   // DeltaQUDc
    w.put(0, 1);   // DeltaQUAc
    w.put(0, 1);   // using_qmatrix
    w.put(0, 1);   // segmentation_enabled
    if (fp.qidx > 0) w.put(0, 1);   // delta_q_present
    // loop_filter_params (av1_lf.h): one level for luma V / H and both chroma planes,
    // sharpness 0, no deltas
    w.put((uint32_t)fp.lf_level, 6);
    w.put((uint32_t)fp.lf_level, 6);
    if (fp.lf_level) {
        w.put((uint32_t)fp.lf_level, 6);
        w.put((uint32_t)fp.lf_level, 6);
    }
    w.put(0, 3);   // loop_filter_sharpness
    w.put(1, 1);   // loop_filter_delta_enabled
    w.put(1, 1);   // loop_filter_delta_update
    for (int i = 0; i < 8; i++) {   // ref deltas: INTRA_FRAME 1 -> 0, the rest keep their defaults
        w.put(i == 0 ? 1 : 0, 1);
        if (i == 0) w.put(0, 7);    // su(1+6) = 0
    }
    w.put(1, 1);                    // mode delta 0 (GLOBALMV / zero-motion class) = -63: level 0
    w.put(128 - 63, 7);             // su(1+6) two's complement of -63
    w.put(0, 1);                    // mode delta 1 keeps 0
    // cdef_params (av1_cdef.h): one strength set, cdef_bits = 0
    const CdefParams cp = cdef_choose(fp.qidx, ac_q(fp.qidx));
    w.put((uint32_t)(cp.damping - 3), 2);
    w.put(0, 2);
    w.put((uint32_t)cp.y_pri, 4);
    w.put((uint32_t)(cp.y_sec == 4 ? 3 : cp.y_sec), 2);
    w.put((uint32_t)cp.uv_pri, 4);
    w.put((uint32_t)(cp.uv_sec == 4 ? 3 : cp.uv_sec), 2);
    w.put(0, 1);   // tx_mode_select = 0 -> TX_MODE_LARGEST
    if (!fp.key) w.put(0, 1);   // reference_select
    w.put(1, 1);   // reduced_tx_set
    if (!fp.key)
        for (int i = 0; i < 7; i++) w.put(0, 1);   // is_global[LAST..ALTREF]
    w.align();     // byte_alignment() before the tile group (OBU_FRAME)
}

// ------------------------------------------------------------------------------ encoder
CpuAv1Encoder::CpuAv1Encoder(const h264::EncoderConfig& cfg, int tcl, int trl) : fe(front_config(cfg)) {
    const int W = fe.g.W, H = fe.g.H;
    // tiles: as many as the level allows (the entropy coder's parallel axis), 16x16 SB max per tile side
    const int sbc = (W + 63) / 64, sbr = (H + 63) / 64;
    int want_c = tcl, want_r = trl;
    int auto_c, auto_r;
    auto_tiles(sbc, sbr, &auto_c, &auto_r);
    if (want_c < 0) want_c = auto_c;
    if (want_r < 0) want_r = auto_r;
    geo_init(geo, W, H, want_c, want_r);
    blk.assign((size_t)geo.c8 * geo.r8, BlkInfo{});
    lev.assign((size_t)fe.g.mb_w * fe.g.mb_h * kLevPerUnit, 0);
    lctx_w[0] = geo.mi_cols;
    lctx_h[0] = geo.mi_rows;
    lctx_w[1] = lctx_w[2] = geo.mi_cols >> 1;
    pal.assign((size_t)geo.c8 * geo.r8 * 8, 0);
    lctx_h[1] = lctx_h[2] = geo.mi_rows >> 1;
    for (int p = 0; p < 3; p++) lctx[p].assign((size_t)lctx_w[p] * lctx_h[p], 0);
    level_idx = choose_level_idx(W, H, cfg.fps);
}

void CpuAv1Encoder::set_cells(int r, int c, int bsl, const BlkInfo& b) {
    const int n8 = (1 << bsl) >> 1;
    for (int y = 0; y < n8; y++)
        for (int x = 0; x < n8; x++) {
            const int ry = (r >> 1) + y, cx = (c >> 1) + x;
            if (ry < geo.r8 && cx < geo.c8) blk[(size_t)ry * geo.c8 + cx] = b;
        }
}

void CpuAv1Encoder::set_lctx(int plane, int x4, int y4, int n4, uint8_t v) {
    for (int y = 0; y < n4; y++)
        for (int x = 0; x < n4; x++)
            if (y4 + y < lctx_h[plane] && x4 + x < lctx_w[plane])
                lctx[plane][(size_t)(y4 + y) * lctx_w[plane] + x4 + x] = v;
}

int16_t* CpuAv1Encoder::unit_lev(int r, int c, int bsl, int plane) const {
    const int ux = c >> 2, uy = r >> 2;
    int16_t* u = const_cast<int16_t*>(&lev[((size_t)uy * fe.g.mb_w + ux) * kLevPerUnit]);
    if (bsl >= 2) return u + (plane == 0 ? 0 : (plane == 1 ? 256 : 320));
    const int k = ((r >> 1) & 1) * 2 + ((c >> 1) & 1);
    return u + (plane == 0 ? 64 * k : (plane == 1 ? 256 + 16 * k : 320 + 16 * k));
}

static uint8_t level_summary(const int16_t* lv, int nn) {
    int cul = 0;
    for (int i = 0; i < nn; i++) cul += lv[i] < 0 ? -lv[i] : lv[i];
    const int dc = lv[0] < 0 ? 1 : (lv[0] > 0 ? 2 : 0);
    return (uint8_t)(sk_min(cul, 63) | (dc << 6));
}

// Levels of one n x n block against `pred` for transform type tt (TX_DCT_DCT / TX_IDTX)
// and their RD cost (av1_core.h tx_rd_cost; k_av1_inter / k_av1_intra_rec compute the same).
static long long quant_block(const uint8_t* src, int sstride, const uint8_t* pred, int log2n, int qidx, bool intra,
                             int tt, int16_t* lv, long long* jzero = nullptr) {
    const int n = 1 << log2n, nn = n * n;
    int32_t res[256], co[256];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) res[i * n + j] = (int)src[(size_t)i * sstride + j] - (int)pred[i * n + j];
    if (tt == TX_IDTX)
        for (int k = 0; k < nn; k++) co[k] = 8 * res[k];
    else
        fwd_transform(res, log2n, co);
    const int qd = dc_q(qidx), qa = ac_q(qidx);
    long long d = 0, z = 0;
    for (int k = 0; k < nn; k++) {
        const int q = k == 0 ? qd : qa;
        lv[k] = (int16_t)quantize(co[k], q, intra);
        const long long e = (long long)co[k] - dequant(lv[k], q);
        d += e * e;
        z += (long long)res[k] * res[k];
    }
    // J of coding nothing (the skip alternative, no rate): 256 x the residual's SSE, the
    // coefficient-domain scale of tx_rd_cost's distortion (8 x orthonormal, x4)
    if (jzero) *jzero += 256 * z;
    int eob = 0;
    for (int c = nn - 1; c >= 0 && !eob; c--)
        if (lv[default_scan(log2n, c)]) eob = c + 1;
    int r2 = tx_eob_bits2(eob);
    for (int c = 0; c < eob; c++) r2 += tx_bits2(lv[default_scan(log2n, c)]);
    return tx_rd_cost(4 * d, r2, qa);
}

// Inter tail trimming, dequantisation and reconstruction of a block's levels into rec
// (pred where all levels are zero); returns whether any level is nonzero.
static bool recon_block(int16_t* lv, int log2n, int qidx, bool intra, int tt, const uint8_t* pred, uint8_t* rec,
                        int rstride) {
    const int n = 1 << log2n, nn = n * n;
    int32_t dq[256], rr[256];
    if (!intra) trim_tail(lv, log2n);
    const int qd = dc_q(qidx), qa = ac_q(qidx);
    bool nz = false;
    for (int k = 0; k < nn; k++) {
        nz |= lv[k] != 0;
        dq[k] = dequant(lv[k], k == 0 ? qd : qa);
    }
    if (nz) {
        inv_transform(dq, log2n, rr, tt == TX_IDTX);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) rec[(size_t)i * rstride + j] = (uint8_t)sk_clip255(pred[i * n + j] + rr[i * n + j]);
    } else {
        for (int i = 0; i < n; i++) memcpy(rec + (size_t)i * rstride, pred + i * n, (size_t)n);
    }
    return nz;
}

static bool any_nonzero(const int16_t* lv, int nn) {
    for (int k = 0; k < nn; k++)
        if (lv[k]) return true;
    return false;
}
// A transform type is only coded with nonzero luma levels; an inter block without them
// has DCT_DCT chroma (TxTypes of an all-zero luma block, spec transform_block).
static bool any_after_trim(const int16_t* lv, int log2n) {
    int16_t t[256];
    memcpy(t, lv, sizeof(int16_t) << (2 * log2n));
    trim_tail(t, log2n);
    return any_nonzero(t, 1 << (2 * log2n));
}

// DCT_DCT with the reconstruction (chroma of intra blocks: UV_DC_PRED implies DCT_DCT).
static bool code_residual(const uint8_t* src, int sstride, const uint8_t* pred, int log2n, int qidx, bool intra,
                          int16_t* lv, uint8_t* rec, int rstride) {
    quant_block(src, sstride, pred, log2n, qidx, intra, TX_DCT_DCT, lv);
    return recon_block(lv, log2n, qidx, intra, TX_DCT_DCT, pred, rec, rstride);
}

// Key frames: DC / V / H / SMOOTH / SMOOTH_V / SMOOTH_H / PAETH by SAD. The mode is
// chosen open-loop, predicting from the *source* edges with the decoder's
// availability rules, so every block is decided independently (in parallel on the
// GPU); the reconstruction then predicts from the reconstructed edges in coding
// order (the per-tile wavefront).
static const uint8_t kIntraCands[7] = {DC_PRED, V_PRED, H_PRED, SMOOTH_PRED, SMOOTH_V_PRED, SMOOTH_H_PRED, PAETH_PRED};

int intra_mode_decision(const uint8_t* src, int stride, int x, int y, int log2n, bool au, bool al, int max_x, int max_y) {
    const int n = 1 << log2n;
    IntraEdge e;
    intra_edges(src, stride, x, y, n, au, al, max_x, max_y, e);
    uint8_t pred[256];
    int best = DC_PRED, best_cost = 1 << 30;
    for (int m : kIntraCands) {
        intra_predict(e, m, log2n, pred);
        int sad = 0;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) sad += sk_abs((int)src[(size_t)(y + i) * stride + x + j] - pred[i * n + j]);
        const int cost = sad + (m == DC_PRED ? 0 : n * 2);   // mode-bits bias
        if (cost < best_cost) {
            best_cost = cost;
            best = m;
        }
    }
    return best;
}

void CpuAv1Encoder::intra_block(int r, int c, int bsl, const TileRect& t) {
    const h264::Geometry& g = fe.g;
    const bool au = inside(t, r - 1, c), al = inside(t, r, c - 1);
    const int log2n = bsl + 2, n = 1 << log2n;
    const int x = c * 4, y = r * 4;
    BlkInfo b = blk[(size_t)(r >> 1) * geo.c8 + (c >> 1)];   // mode from the decision pass
    IntraEdge ey;
    intra_edges(fe.rec[0].data(), g.stride_y, x, y, n, au, al, geo.mi_cols * 4 - 1, geo.mi_rows * 4 - 1, ey);
    uint8_t py[256];
    intra_predict(ey, b.mode, log2n, py);
    int16_t* ly = unit_lev(r, c, bsl, 0);
    // luma transform type: DCT_DCT or IDTX (screen content: sharp text codes as samples), by RD cost
    int16_t lid[256];
    const uint8_t* sy = &fe.src[0][(size_t)y * g.stride_y + x];
    const long long jd = quant_block(sy, g.stride_y, py, log2n, fp.qidx, true, TX_DCT_DCT, ly);
    const long long ji = quant_block(sy, g.stride_y, py, log2n, fp.qidx, true, TX_IDTX, lid);
    b.tx_type = (int16_t)(ji < jd && any_nonzero(lid, n * n) ? TX_IDTX : TX_DCT_DCT);
    if (b.tx_type == TX_IDTX) memcpy(ly, lid, sizeof(int16_t) * n * n);
    b.pal_n = 0;
    uint8_t col[kPalMax] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int k = fp.screen && r + (1 << bsl) <= geo.mi_rows && c + (1 << bsl) <= geo.mi_cols
                      ? palette_colors(sy, g.stride_y, n, col) : 0;
    if (k) {   // exact palette vs the transform path (J of the levels just chosen)
        uint8_t map[256];
        int rate2 = palette_rate2_head(k);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) map[i * n + j] = (uint8_t)palette_index(col, k, sy[(size_t)i * g.stride_y + j]);
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) rate2 += palette_rate2_px(map, n, i, j, k);
        if (tx_rd_cost(0, rate2, ac_q(fp.qidx)) < (jd < ji ? jd : ji)) {
            b.pal_n = (uint8_t)k;
            b.mode = DC_PRED;
            b.tx_type = TX_DCT_DCT;
            memset(ly, 0, sizeof(int16_t) * n * n);
            for (int i = 0; i < n; i++) memcpy(&py[i * n], sy + (size_t)i * g.stride_y, (size_t)n);
            set_palette(r, c, bsl, col);
        }
    }
    bool nz = recon_block(ly, log2n, fp.qidx, true, b.tx_type, py, &fe.rec[0][(size_t)y * g.stride_y + x], g.stride_y);
    // chroma: UV_DC_PRED. Every other UV mode implies an ADST-family chroma transform
    // (Mode_To_Txfm, §7.13.3 compute_tx_type); this encoder's transforms are DCT_DCT.
    const int cl2 = log2n - 1, cn = n >> 1, cx = x >> 1, cy = y >> 1;
    IntraEdge eu, ev;
    intra_edges(fe.rec[1].data(), g.stride_c, cx, cy, cn, au, al, geo.mi_cols * 2 - 1, geo.mi_rows * 2 - 1, eu);
    intra_edges(fe.rec[2].data(), g.stride_c, cx, cy, cn, au, al, geo.mi_cols * 2 - 1, geo.mi_rows * 2 - 1, ev);
    uint8_t bu[64], bv[64];
    intra_predict(eu, DC_PRED, cl2, bu);
    intra_predict(ev, DC_PRED, cl2, bv);
    int16_t* lu = unit_lev(r, c, bsl, 1);
    int16_t* lvv = unit_lev(r, c, bsl, 2);
    nz |= code_residual(&fe.src[1][(size_t)cy * g.stride_c + cx], g.stride_c, bu, cl2, fp.qidx, true, lu,
                        &fe.rec[1][(size_t)cy * g.stride_c + cx], g.stride_c);
    nz |= code_residual(&fe.src[2][(size_t)cy * g.stride_c + cx], g.stride_c, bv, cl2, fp.qidx, true, lvv,
                        &fe.rec[2][(size_t)cy * g.stride_c + cx], g.stride_c);
    b.flags = nz ? 0 : 2;
    set_cells(r, c, bsl, b);
    const int n4 = 1 << bsl;
    set_lctx(0, c, r, n4, nz ? level_summary(ly, n * n) : 0);
    set_lctx(1, c >> 1, r >> 1, n4 >> 1, nz ? level_summary(lu, cn * cn) : 0);
    set_lctx(2, c >> 1, r >> 1, n4 >> 1, nz ? level_summary(lvv, cn * cn) : 0);
}

void CpuAv1Encoder::set_palette(int r, int c, int bsl, const uint8_t* col) {
    const int n8 = (1 << bsl) >> 1;
    for (int y = 0; y < n8; y++)
        for (int x = 0; x < n8; x++) {
            const int ry = (r >> 1) + y, cx = (c >> 1) + x;
            if (ry < geo.r8 && cx < geo.c8) memcpy(&pal[((size_t)ry * geo.c8 + cx) * 8], col, kPalMax);
        }
}

void CpuAv1Encoder::key_partition(int r, int c, int bsl, const TileRect& t, bool decide) {
    if (r >= geo.mi_rows || c >= geo.mi_cols) return;
    const int half = (1 << bsl) >> 1;
    const bool has_rows = r + half < geo.mi_rows, has_cols = c + half < geo.mi_cols;
    if (bsl == 1 || (bsl == 2 && has_rows && has_cols)) {
        if (decide) {
            BlkInfo b{};
            b.bsl = (uint8_t)bsl;
            b.uv_mode = DC_PRED;
            b.mode = (uint8_t)intra_mode_decision(fe.src[0].data(), fe.g.stride_y, c * 4, r * 4, bsl + 2,
                                                  inside(t, r - 1, c), inside(t, r, c - 1), geo.mi_cols * 4 - 1,
                                                  geo.mi_rows * 4 - 1);
            set_cells(r, c, bsl, b);
        } else {
            intra_block(r, c, bsl, t);
        }
        return;
    }
    for (int q = 0; q < 4; q++) key_partition(r + (q >> 1) * half, c + (q & 1) * half, bsl - 1, t, decide);
}

void CpuAv1Encoder::decide_key() {
    for (int pass = 0; pass < 2; pass++)
        for (int t = 0; t < geo.tile_cols * geo.tile_rows; t++) {
            const TileRect tr = tile_rect(geo, t);
            for (int r = tr.mi_row0; r < tr.mi_row1; r += 16)
                for (int c = tr.mi_col0; c < tr.mi_col1; c += 16) key_partition(r, c, 4, tr, pass == 0);
        }
}

// One motion-compensated block: prediction from fe.ref, residual, reconstruction.
void CpuAv1Encoder::inter_block(int r, int c, int bsl, int mv_row, int mv_col) {
    const h264::Geometry& g = fe.g;
    const int log2n = bsl + 2, n = 1 << log2n, x = c * 4, y = r * 4;
    uint8_t py[256], pu[64], pv[64];
    mc_block(fe.ref[0].data(), g.stride_y, geo.W - 1, geo.H - 1, x, y, n, n, 0, mv_row, mv_col, py, n);
    const int cn = n >> 1, cx = x >> 1, cy = y >> 1;
    const int lxc = ((geo.W + 1) >> 1) - 1, lyc = ((geo.H + 1) >> 1) - 1;
    mc_block(fe.ref[1].data(), g.stride_c, lxc, lyc, cx, cy, cn, cn, 1, mv_row, mv_col, pu, cn);
    mc_block(fe.ref[2].data(), g.stride_c, lxc, lyc, cx, cy, cn, cn, 1, mv_row, mv_col, pv, cn);
    int16_t* lp[3] = {unit_lev(r, c, bsl, 0), unit_lev(r, c, bsl, 1), unit_lev(r, c, bsl, 2)};
    int16_t* ly = lp[0];
    int16_t* lu = lp[1];
    int16_t* lvv = lp[2];
    // transform type of the block (inter chroma follows luma): DCT_DCT or IDTX by the
    // RD cost over the three planes
    const uint8_t* sp[3] = {&fe.src[0][(size_t)y * g.stride_y + x], &fe.src[1][(size_t)cy * g.stride_c + cx],
                            &fe.src[2][(size_t)cy * g.stride_c + cx]};
    const uint8_t* pp[3] = {py, pu, pv};
    const int ss[3] = {g.stride_y, g.stride_c, g.stride_c}, ln[3] = {log2n, log2n - 1, log2n - 1};
    int16_t lid[3][256];
    long long jd = 0, ji = 0, jz = 0;
    for (int p = 0; p < 3; p++) {
        jd += quant_block(sp[p], ss[p], pp[p], ln[p], fp.qidx, false, TX_DCT_DCT, lp[p], &jz);
        ji += quant_block(sp[p], ss[p], pp[p], ln[p], fp.qidx, false, TX_IDTX, lid[p]);
    }
    // IDTX only where the DCT codes something (a block the DCT quantises to nothing stays a
    // skip) and the luma keeps levels (else chroma is DCT_DCT, see any_after_trim)
    const bool dct_codes = any_after_trim(lp[0], log2n) || any_after_trim(lp[1], log2n - 1) ||
                           any_after_trim(lp[2], log2n - 1);
    int tt = dct_codes && ji < jd && any_after_trim(lid[0], log2n) ? TX_IDTX : TX_DCT_DCT;
    if (tt == TX_IDTX)
        for (int p = 0; p < 3; p++) memcpy(lp[p], lid[p], sizeof(int16_t) << (2 * ln[p]));
    // RD skip: the levels must pay for themselves against the prediction alone (static
    // screen content at fine quantisers otherwise re-codes every block's last grain of
    // error in one frame: 2x budgets at the QP where it starts)
    if (jz <= (tt == TX_IDTX ? ji : jd))
        for (int p = 0; p < 3; p++) memset(lp[p], 0, sizeof(int16_t) << (2 * ln[p]));
    bool nz = recon_block(ly, log2n, fp.qidx, false, tt, py, &fe.rec[0][(size_t)y * g.stride_y + x], g.stride_y);
    nz |= recon_block(lu, log2n - 1, fp.qidx, false, tt, pu, &fe.rec[1][(size_t)cy * g.stride_c + cx], g.stride_c);
    nz |= recon_block(lvv, log2n - 1, fp.qidx, false, tt, pv, &fe.rec[2][(size_t)cy * g.stride_c + cx], g.stride_c);
    BlkInfo b{};
    b.tx_type = (int16_t)(nz ? tt : TX_DCT_DCT);
    b.bsl = (uint8_t)bsl;
    b.flags = (uint8_t)(1 | (nz ? 0 : 2));
    b.mv_row = (int16_t)mv_row;
    b.mv_col = (int16_t)mv_col;
    b.mode = GLOBALMV;
    set_cells(r, c, bsl, b);
    const int n4 = 1 << bsl;
    set_lctx(0, c, r, n4, nz ? level_summary(ly, n * n) : 0);
    set_lctx(1, c >> 1, r >> 1, n4 >> 1, nz ? level_summary(lu, cn * cn) : 0);
    set_lctx(2, c >> 1, r >> 1, n4 >> 1, nz ? level_summary(lvv, cn * cn) : 0);
}

void CpuAv1Encoder::inter_unit(int ux, int uy, int mv_row, int mv_col) {
    const int r = uy * 4, c = ux * 4;
    if (r >= geo.mi_rows || c >= geo.mi_cols) return;
    if (r + 2 < geo.mi_rows && c + 2 < geo.mi_cols) {
        inter_block(r, c, 2, mv_row, mv_col);
        return;
    }
    for (int q = 0; q < 4; q++) {
        const int rr = r + (q >> 1) * 2, cc = c + (q & 1) * 2;
        if (rr < geo.mi_rows && cc < geo.mi_cols) inter_block(rr, cc, 1, mv_row, mv_col);
    }
}

void CpuAv1Encoder::decide_inter() {
    const h264::Geometry& g = fe.g;
    for (int s = 0; s < g.num_slices; s++) {
        const h264::SliceTask& t = fe.tasks[s];
        for (int uy = t.first_row; uy < t.first_row + t.num_rows; uy++)
            for (int ux = 0; ux < g.mb_w; ux++) {
                const h264::MeResult& m = fe.me[(size_t)uy * g.mb_w + ux];
                const bool moving = t.final_action == ACT_P;
                inter_unit(ux, uy, moving ? 8 * m.mvy : 0, moving ? 8 * m.mvx : 0);
            }
    }
    // static merging: 32x32 then 64x64 blocks whose cells are all skipped with one vector
    for (int lvl = 3; lvl <= 4; lvl++) {
        const int sz = 1 << lvl, half = sz >> 1;
        for (int r = 0; r < geo.mi_rows; r += sz)
            for (int c = 0; c < geo.mi_cols; c += sz) {
                if (r + sz > geo.mi_rows || c + sz > geo.mi_cols) continue;   // inside the picture (k_av1_merge)
                const BlkInfo& b0 = blk[(size_t)(r >> 1) * geo.c8 + (c >> 1)];
                bool ok = true;
                for (int y = r >> 1; ok && y < std::min((r + sz) >> 1, geo.r8); y++)
                    for (int x = c >> 1; ok && x < std::min((c + sz) >> 1, geo.c8); x++) {
                        const BlkInfo& b = blk[(size_t)y * geo.c8 + x];
                        ok = blk_skip(b) && b.mv_row == b0.mv_row && b.mv_col == b0.mv_col;
                    }
                if (!ok) continue;
                BlkInfo m = b0;
                m.bsl = (uint8_t)lvl;
                set_cells(r, c, lvl, m);
            }
    }
}

// Pass A: each inter block's mode from its MV stack (the stack depends on the
// neighbours' vectors only, so every block can be decided independently).
void CpuAv1Encoder::decide_modes() {
    const BlkGrid grid{blk.data(), geo.c8};
    for (int t = 0; t < geo.tile_cols * geo.tile_rows; t++) {
        const TileRect tr = tile_rect(geo, t);
        for (int y8 = tr.mi_row0 >> 1; y8 < (tr.mi_row1 + 1) >> 1; y8++)
            for (int x8 = tr.mi_col0 >> 1; x8 < (tr.mi_col1 + 1) >> 1; x8++) {
                BlkInfo& b = blk[(size_t)y8 * geo.c8 + x8];
                const int n8 = (1 << b.bsl) >> 1;
                if (!blk_inter(b) || (y8 & (n8 - 1)) || (x8 & (n8 - 1))) continue;   // block origin cells only
                const int r = y8 * 2, c = x8 * 2;
                MvStack s;
                find_mv_stack(s, grid, tr, geo.mi_rows, geo.mi_cols, r, c, b.bsl,
                              [&](int mr, int mc) { return decoded_before(mr, mc, r, c); });
                int mode, idx = 0;
                if (b.mv_row == 0 && b.mv_col == 0) mode = GLOBALMV;
                else if (b.mv_row == s.mv[0][0] && b.mv_col == s.mv[0][1]) mode = NEARESTMV;
                else if (s.n >= 2 && b.mv_row == s.mv[1][0] && b.mv_col == s.mv[1][1]) {
                    mode = NEARMV;
                    idx = 1;
                } else mode = NEWMV;
                BlkInfo m = b;
                m.mode = (uint8_t)mode;
                m.flags = (uint8_t)((m.flags & 0x0f) | (idx << 4));
                set_cells(r, c, b.bsl, m);
            }
    }
}

// ------------------------------------------------------------------------------ tile coding
FrameView CpuAv1Encoder::view() const {
    FrameView v;
    v.geo = geo;
    v.blk = blk.data();
    v.lev = lev.data();
    for (int p = 0; p < 3; p++) {
        v.lctx[p] = lctx[p].data();
        v.lctx_w[p] = lctx_w[p];
    }
    v.unit_w = fe.g.mb_w;
    v.qidx = fp.qidx;
    v.key = fp.key;
    v.screen = fp.screen;
    v.pal = pal.data();
    v.src_y = fe.src[0].data();
    v.stride_y = fe.g.stride_y;
    return v;
}

std::vector<uint8_t> CpuAv1Encoder::code_tile(int t) {
    const TileRect tr = tile_rect(geo, t);
    MvStack stk;
    FrameView v = view();
    v.stk = &stk;
    CdfContext cx = AV1_DEFAULT_CDF[coef_qctx(fp.qidx)];
    VectorSink sink;
    SymbolCoder<VectorSink> coder(sink);
    DirectSink<SymbolCoder<VectorSink>> w{coder, cx};
    int ux, uy;
    for (int i = 0; tile_unit(geo, tr, i, &ux, &uy); i++) code_unit(w, cx, v, tr, ux, uy);
    coder.finish();
    std::vector<uint8_t> out(sink.v.size());
    if (!out.empty()) carry_bytes(sink.v.data(), (int)sink.v.size(), out.data());
    return out;
}

std::vector<uint8_t> CpuAv1Encoder::assemble(const std::vector<std::vector<uint8_t>>& tiles) {
    size_t maxsz = 1;
    for (size_t i = 0; i + 1 < tiles.size(); i++) maxsz = std::max(maxsz, tiles[i].size());
    fp.tile_size_bytes = maxsz <= 0x100 ? 1 : (maxsz <= 0x10000 ? 2 : (maxsz <= 0x1000000 ? 3 : 4));
    std::vector<uint8_t> out;
    append_obu(out, 2, nullptr, 0);   // temporal delimiter
    if (fp.key) {
        BitWriter sh;
        write_sequence_header(sh, geo.W, geo.H, level_idx, fe.cfg.full_range);
        append_obu(out, 1, sh.buf.data(), sh.buf.size());
    }
    BitWriter fh;
    write_frame_header(fh, geo, fp);
    std::vector<uint8_t> payload = fh.buf;
    const int nt = (int)tiles.size();
    if (nt > 1) payload.push_back(0);   // tile_start_and_end_present_flag = 0 + byte_alignment
    for (int i = 0; i < nt; i++) {
        if (i + 1 < nt) {
            const uint32_t sz = (uint32_t)tiles[i].size() - 1;
            for (int k = 0; k < fp.tile_size_bytes; k++) payload.push_back((uint8_t)(sz >> (8 * k)));
        }
        payload.insert(payload.end(), tiles[i].begin(), tiles[i].end());
    }
    append_obu(out, 6, payload.data(), payload.size());   // OBU_FRAME
    return out;
}

void CpuAv1Encoder::encode(const uint8_t* bgrx, int stride, uint16_t frame_id, std::vector<h264::EncodedPacket>& out) {
    fe.load_frame(bgrx, stride);
    fe.ctl_.plan(fe.stripe_dirty.data(), fe.tasks.data());
    const int ns = fe.g.num_slices;
    bool key = false;
    for (int s = 0; s < ns; s++) {
        h264::SliceTask& t = fe.tasks[s];
        t.final_action = t.action;
        if (t.action == ACT_P) {
            fe.motion_search(s);
            fe.decide_scenecut(s);
        } else if (t.action == ACT_I) {
            fe.intra_activity(s);
        }
        key |= t.final_action == ACT_I;
    }
    if (key)   // AV1 has no intra slices: a key frame refreshes the whole picture
        for (int s = 0; s < ns; s++) fe.tasks[s].final_action = ACT_I;
    fe.ctl_.rate_control(fe.tasks.data(), fe.me.data());   // K10
    fp.key = key;
    fp.screen = key && palette_on;
    uint8_t tab[52];
    for (int q = 0; q < 52; q++) tab[q] = (uint8_t)qidx_for_qp(q);
    std::vector<std::vector<uint8_t>> tiles(geo.tile_cols * geo.tile_rows);
    long long payload = 0;   // K10 accounting unit: tile payload bits (k_rc_account: tile sizes)
    // block decisions, reconstruction and tile coding at the frame's qindex; every block
    // of the picture is rewritten, so a second pass starts clean
    auto code_picture = [&] {
        {   // K10: the frame's fractional QP under CRF / CBR (k_av1_setup: same rule)
            const h264::RcState& rc = fe.ctl_.rc();
            fp.qidx = rc.mode == h264::RC_CQP ? tab[sk_clip(fe.tasks[0].qp, 0, 51)] : frame_qidx(tab, rc.cur_qpf);
        }
        fp.lf_level = lf_level_for(ac_q(fp.qidx), key);
        std::fill(blk.begin(), blk.end(), BlkInfo{});
        if (key) {
            decide_key();
        } else {
            decide_inter();
            decide_modes();
        }
        payload = 0;
        for (int t = 0; t < (int)tiles.size(); t++) {
            tiles[t] = code_tile(t);
            payload += 8 * (long long)tiles[t].size();
        }
    };
    code_picture();
    // K10 per-frame cap (ratecontrol.h rc_frame_cap): a frame over it is coded again at a
    // coarser qindex, up to twice (k_rc_guard_sizes gates the GPU back end's passes)
    for (int r = 0; r < h264::kMaxRecodes && fe.ctl_.rate_redo(fe.tasks.data(), payload); r++) code_picture();
    h264::EncodedPacket pk;
    pk.y = 0;
    pk.w = fe.g.W;
    pk.h = fe.g.H;
    pk.key = key;
    pk.data.resize(10);
    h264::write_stripe_header(pk.data.data(), key, frame_id, 0, fe.g.W, fe.g.H);
    std::vector<uint8_t> tu = assemble(tiles);
    pk.data.insert(pk.data.end(), tu.begin(), tu.end());
    fe.ctl_.rate_account(payload);
    out.push_back(std::move(pk));
    // every row of the picture was coded: the reconstruction is the next reference;
    // static slices were coded as zero-motion skips (zero MV field, k_av1_finish)
    for (int s = 0; s < ns; s++)
        if (fe.tasks[s].final_action == ACT_NONE || fe.tasks[s].final_action == ACT_SKIPALL) {
            h264::SliceTask& t = fe.tasks[s];
            t.final_action = ACT_P;
            for (int j = t.first_row * fe.g.mb_w; j < (t.first_row + t.num_rows) * fe.g.mb_w; j++)
                fe.me[j].mvx = fe.me[j].mvy = 0;
        }
    // in-loop deblocking (7.14) of the reconstruction: per plane all vertical edges, then
    // all horizontal ones
    const h264::Geometry& g = fe.g;
    LfFrame lf{blk.data(), geo.c8, geo.mi_rows, geo.mi_cols, geo.W, geo.H,
               {fp.lf_level, fp.lf_level, fp.lf_level, fp.lf_level}};
    if (fp.lf_level)
        for (int p = 0; p < 3; p++)
            for (int pass = 0; pass < 2; pass++)
                for (int r = 0; r < geo.mi_rows; r += p ? 2 : 1)
                    for (int c = 0; c < geo.mi_cols; c += p ? 2 : 1)
                        lf_edge(lf, p, pass, r, c, fe.rec[p].data(), p ? g.stride_c : g.stride_y);
    // CDEF (7.15) on the deblocked picture
    const CdefParams cp = cdef_choose(fp.qidx, ac_q(fp.qidx));
    if (cdef_on(cp)) {
        std::vector<uint8_t> in[3] = {fe.rec[0], fe.rec[1], fe.rec[2]};
        const uint8_t* ip[3] = {in[0].data(), in[1].data(), in[2].data()};
        uint8_t* op[3] = {fe.rec[0].data(), fe.rec[1].data(), fe.rec[2].data()};
        const int st[3] = {g.stride_y, g.stride_c, g.stride_c};
        for (int sr = 0; sr < geo.mi_rows; sr += 16)
            for (int sc = 0; sc < geo.mi_cols; sc += 16) {
                if (!cdef_sb_on(blk.data(), geo, sr, sc)) continue;   // cdef_idx -1: every block skipped
                for (int r = sr; r < sr + 16 && r < geo.mi_rows; r += 2)
                    for (int c = sc; c < sc + 16 && c < geo.mi_cols; c += 2)
                        cdef_block(ip, st, op, st, cp, r, c, blk_skip(blk[(size_t)(r >> 1) * geo.c8 + (c >> 1)]),
                                   geo.mi_rows, geo.mi_cols);
            }
    }
    // rows past the picture bottom repeat the last row (what AV1's reference clamp reads)
    for (int y = geo.H; y < g.plane_h_y; y++)
        memcpy(&fe.rec[0][(size_t)y * g.stride_y], &fe.rec[0][(size_t)(geo.H - 1) * g.stride_y], g.stride_y);
    const int hc = (geo.H + 1) >> 1;
    for (int p = 1; p < 3; p++)
        for (int y = hc; y < g.plane_h_c; y++)
            memcpy(&fe.rec[p][(size_t)y * g.stride_c], &fe.rec[p][(size_t)(hc - 1) * g.stride_c], g.stride_c);
    fe.finish_frame();
    frames++;
}

}  // namespace av1
}  // namespace sk
