// CPU reference backend of the H.264 stripe encoder. It is (1) the `use_cpu`
// execution path of the pixelflux-compatible capture module and (2) the golden
// model for the HIP pipeline: every stage below has a kernel counterpart in
// csrc/kernels/h264_kernels.hip that must produce bit-identical buffers.
#include "h264_frame.h"
#include "color.h"
#include "h264_deblock.h"
#include <string.h>
#include <algorithm>

namespace sk {
namespace h264 {

CpuH264Encoder::CpuH264Encoder(const EncoderConfig& c) : cfg(c) {
    g.init(cfg);
    scaled_ = (cfg.src_width > 0 && cfg.src_width != cfg.width) || (cfg.src_height > 0 && cfg.src_height != cfg.height);
    if (scaled_)
        scale_ = scale_params(cfg.src_width > 0 ? cfg.src_width : cfg.width,
                              cfg.src_height > 0 ? cfg.src_height : cfg.height, cfg.width, cfg.height);
    ctl_.init(cfg, g);
    size_t ny = (size_t)g.stride_y * g.plane_h_y, nc = (size_t)g.stride_c * g.plane_h_c;
    for (int p = 0; p < 3; p++) {
        size_t n = p ? nc : ny;
        src[p].assign(n, 0);
        prev[p].assign(n, 0);
        ref[p].assign(n, 0);
        ref1[p].assign(n, 0);
        rec[p].assign(n, 0);
    }
    mb_dirty.assign(g.num_mbs(), 1);
    stripe_dirty.assign(g.num_slices, 1);
    mbs.assign(g.num_mbs(), MbInfo());
    coefs.assign((size_t)g.num_mbs() * kCoefPerMb, 0);
    me.assign(g.num_mbs(), MeResult());
    mvfield.assign((size_t)g.num_mbs() * 2, 0);
    dbinfo.assign(g.num_mbs(), DbInfo());
    fs_mv.assign((size_t)g.num_mbs() * 2, 0);
    tasks.assign(g.num_slices, SliceTask());
    if (cfg.fullframe) {
        param_sets.resize(1);
        build_parameter_sets(g.W, g.H, cfg.full_range, cfg.fps, param_sets[0], cfg.num_refs);
    } else {
        param_sets.resize(g.num_slices);
        for (int s = 0; s < g.num_slices; s++)
            build_parameter_sets(g.W, g.slice_pix_h(s), cfg.full_range, cfg.fps, param_sets[s], cfg.num_refs);
    }
}

void CpuH264Encoder::set_overlay_image(int slot, const uint8_t* bgra, int w, int h) {
    if (slot < 0 || slot >= kOverlaySlots) return;
    w = std::max(0, std::min(w, kOverlayMaxDim));
    h = std::max(0, std::min(h, kOverlayMaxDim));
    overlay_img[slot].assign(bgra, bgra + (size_t)w * h * 4);
    overlay[slot].w = w;
    overlay[slot].h = h;
    if (!w || !h) overlay[slot].on = 0;
}

void CpuH264Encoder::set_overlay_pos(int slot, int on, int x, int y, int tdx, int tdy) {
    if (slot < 0 || slot >= kOverlaySlots) return;
    OverlayParams& o = overlay[slot];
    o.on = on && o.w > 0 && o.h > 0;
    o.x = x;
    o.y = y;
    o.tdx = tdx > 0 ? tdx : 0;
    o.tdy = tdy > 0 ? tdy : 0;
}

// K3: per-MB damage against the previous source, per-stripe dirty flags.
void CpuH264Encoder::detect_damage() {
    std::fill(stripe_dirty.begin(), stripe_dirty.end(), 0);
    for (int mby = 0; mby < g.mb_h; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) {
            bool d = first_frame;
            for (int y = 0; y < 16 && !d; y++) {
                size_t o = (size_t)(mby * 16 + y) * g.stride_y + mbx * 16;
                d = memcmp(&src[0][o], &prev[0][o], 16) != 0;
            }
            for (int p = 1; p < 3 && !d; p++)
                for (int y = 0; y < 8 && !d; y++) {
                    size_t o = (size_t)(mby * 8 + y) * g.stride_c + mbx * 8;
                    d = memcmp(&src[p][o], &prev[p][o], 8) != 0;
                }
            mb_dirty[mby * g.mb_w + mbx] = d;
            if (d) stripe_dirty[mby / g.rows_per_slice] = 1;
        }
}

void CpuH264Encoder::load_frame_yuv() {
    const int W = g.W, H = g.H;
    for (int y = 0; y < g.plane_h_y; y++)
        for (int x = 0; x < g.stride_y; x++)
            src[0][(size_t)y * g.stride_y + x] = yuv_sample(yuv_in.fmt, yuv_in.p, yuv_in.stride, 0, x, y, W, H);
    for (int c = 1; c < 3; c++)
        for (int y = 0; y < g.plane_h_c; y++)
            for (int x = 0; x < g.stride_c; x++)
                src[c][(size_t)y * g.stride_c + x] = yuv_sample(yuv_in.fmt, yuv_in.p, yuv_in.stride, c, x, y, W, H);
}

void CpuH264Encoder::load_frame(const uint8_t* bgrx, int stride) {
    const int W = g.W, H = g.H;
    if (yuv_in.fmt != YUV_NONE) {   // planar input: no K1, straight to the damage pass
        load_frame_yuv();
        yuv_in.fmt = YUV_NONE;
        detect_damage();
        return;
    }
    const bool ov = overlay[0].on || overlay[1].on;
    const uint8_t* ovimg[kOverlaySlots] = {overlay_img[0].data(), overlay_img[1].data()};
    for (int qy = 0; qy < g.plane_h_c; qy++) {
        int y0 = std::min(2 * qy, H - 1), y1 = std::min(2 * qy + 1, H - 1);
        const uint8_t* r0 = bgrx + (size_t)y0 * stride;
        const uint8_t* r1 = bgrx + (size_t)y1 * stride;
        for (int qx = 0; qx < g.stride_c; qx++) {
            int x0 = std::min(2 * qx, W - 1), x1 = std::min(2 * qx + 1, W - 1);
            uint8_t y[4], cb, cr;
            if (scaled_ || ov) {   // K2: bilinear resample of the capture, same integer math as the kernel
                uint32_t q[4];
                if (scaled_) {
                    q[0] = scale_fetch(bgrx, stride, scale_, x0, y0);
                    q[1] = scale_fetch(bgrx, stride, scale_, x1, y0);
                    q[2] = scale_fetch(bgrx, stride, scale_, x0, y1);
                    q[3] = scale_fetch(bgrx, stride, scale_, x1, y1);
                } else {
                    memcpy(&q[0], r0 + 4 * x0, 4);
                    memcpy(&q[1], r0 + 4 * x1, 4);
                    memcpy(&q[2], r1 + 4 * x0, 4);
                    memcpy(&q[3], r1 + 4 * x1, 4);
                }
                if (ov) {   // K12/K13 in picture coordinates (padding repeats the edge pixel)
                    q[0] = overlay_px(q[0], x0, y0, overlay, ovimg);
                    q[1] = overlay_px(q[1], x1, y0, overlay, ovimg);
                    q[2] = overlay_px(q[2], x0, y1, overlay, ovimg);
                    q[3] = overlay_px(q[3], x1, y1, overlay, ovimg);
                }
                bgrx_quad_to_yuv((const uint8_t*)&q[0], (const uint8_t*)&q[1], (const uint8_t*)&q[2],
                                 (const uint8_t*)&q[3], cfg.full_range, y, &cb, &cr);
            } else {
                bgrx_quad_to_yuv(r0 + 4 * x0, r0 + 4 * x1, r1 + 4 * x0, r1 + 4 * x1, cfg.full_range, y,
                                 &cb, &cr);
            }
            size_t oy = (size_t)(2 * qy) * g.stride_y + 2 * qx;
            src[0][oy] = y[0];
            src[0][oy + 1] = y[1];
            src[0][oy + g.stride_y] = y[2];
            src[0][oy + g.stride_y + 1] = y[3];
            src[1][(size_t)qy * g.stride_c + qx] = cb;
            src[2][(size_t)qy * g.stride_c + qx] = cr;
        }
    }
    detect_damage();
}

int CpuH264Encoder::sad_at(int mbx, int mby, int dx, int dy, const SliceTask& t, int refi) const {
    int y_lo = t.pic_row0 * 16, y_hi = (t.pic_row0 + t.pic_rows) * 16 - 1;
    int x_hi = g.stride_y - 1;
    int sad = 0;
    for (int y = 0; y < 16; y++) {
        int sy = sk_clip(mby * 16 + y + dy, y_lo, y_hi);
        const uint8_t* s = &src[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16];
        const uint8_t* r = &refs(refi)[0][(size_t)sy * g.stride_y];
        for (int x = 0; x < 16; x++) {
            int sx = sk_clip(mbx * 16 + x + dx, 0, x_hi);
            sad += sk_abs((int)s[x] - (int)r[sx]);
        }
    }
    return sad;
}

// K4a reference: exhaustive +-16 search ranked by fs_key (k_me_mfma computes the
// same integers with int8 MFMA cross-correlations).
void CpuH264Encoder::full_search(int mbx, int mby, const SliceTask& t, int16_t* out) const {
    const int y_lo = t.pic_row0 * 16, y_hi = (t.pic_row0 + t.pic_rows) * 16 - 1, x_hi = g.stride_y - 1;
    static thread_local int win[kFsWin][kFsWin];
    int sb[16][16];
    for (int wy = 0; wy < kFsWin; wy++) {
        const uint8_t* row = &ref[0][(size_t)sk_clip(mby * 16 - kFsR + wy, y_lo, y_hi) * g.stride_y];
        for (int wx = 0; wx < kFsWin; wx++) win[wy][wx] = (int)row[sk_clip(mbx * 16 - kFsR + wx, 0, x_hi)] - 128;
    }
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) sb[y][x] = (int)src[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16 + x] - 128;
    uint64_t best = ~0ull;
    for (int dyw = 0; dyw < 2 * kFsR; dyw++)
        for (int dxw = 0; dxw < 2 * kFsR; dxw++) {
            int ssq = 0, cross = 0;
            for (int y = 0; y < 16; y++) {
                const int* w = &win[dyw + y][dxw];
                for (int x = 0; x < 16; x++) {
                    ssq += w[x] * w[x];
                    cross += sb[y][x] * w[x];
                }
            }
            best = std::min(best, fs_key(ssq - 2 * cross, dyw, dxw));
        }
    out[0] = (int16_t)fs_key_dx(best);
    out[1] = (int16_t)fs_key_dy(best);
}

// sum |Y - mean| of the source MB (k_motion_search mb_activity)
int CpuH264Encoder::mb_activity(int mbx, int mby) const {
    int sum = 0;
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) sum += src[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16 + x];
    const int mean = (sum + 128) >> 8;
    int dev = 0;
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++) dev += sk_abs((int)src[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16 + x] - mean);
    return dev;
}

// Planned intra slice: the activity of every MB (K10's key-frame complexity), no search.
void CpuH264Encoder::intra_activity(int s) {
    const SliceTask& t = tasks[s];
    for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) me[(size_t)mby * g.mb_w + mbx] = MeResult{0, 0, 0, mb_activity(mbx, mby), 0, 0, 0};
}

void CpuH264Encoder::motion_search(int s) {
    const SliceTask& t = tasks[s];
    const int lam = lambda_for_qp(rc_me_qp(ctl_.rc(), t.qp));
    const int R = cfg.me_range;
    auto cost_of = [&](int mbx, int mby, int dx, int dy, int* sad_out) {
        int sad = sad_at(mbx, mby, dx, dy, t);
        *sad_out = sad;
        return sad + lam * (sk_se_bits(4 * dx) + sk_se_bits(4 * dy));
    };
    for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) {
            int idx = mby * g.mb_w + mbx;
            int cx[7], cy[7], n = 0;
            cx[n] = 0; cy[n] = 0; n++;
            auto add = [&](int ox, int oy) {
                int j = oy * g.mb_w + ox;
                cx[n] = sk_clip(mvfield[2 * j], -R, R);
                cy[n] = sk_clip(mvfield[2 * j + 1], -R, R);
                n++;
            };
            add(mbx, mby);
            if (mbx > 0) add(mbx - 1, mby);
            if (mbx + 1 < g.mb_w) add(mbx + 1, mby);
            if (mby - 1 >= t.pic_row0) add(mbx, mby - 1);
            if (mby + 1 < t.pic_row0 + t.pic_rows) add(mbx, mby + 1);
            if (cfg.me_full && mb_dirty[idx]) {
                // the MB's previous vector already matches exactly (scrolls, moving windows):
                // nothing can beat it, skip the exhaustive search
                const int px = sk_clip(mvfield[2 * idx], -R, R), py = sk_clip(mvfield[2 * idx + 1], -R, R);
                if (sad_at(mbx, mby, px, py, t) == 0) {
                    fs_mv[2 * idx] = (int16_t)px;
                    fs_mv[2 * idx + 1] = (int16_t)py;
                } else {
                    full_search(mbx, mby, t, &fs_mv[2 * idx]);
                }
                cx[n] = sk_clip(fs_mv[2 * idx], -R, R);
                cy[n] = sk_clip(fs_mv[2 * idx + 1], -R, R);
                n++;
            }
            int bx = 0, by = 0, bsad = 0;
            int bcost = cost_of(mbx, mby, 0, 0, &bsad);
            for (int i = 1; i < n; i++) {
                int sd;
                int c = cost_of(mbx, mby, cx[i], cy[i], &sd);
                if (c < bcost) { bcost = c; bx = cx[i]; by = cy[i]; bsad = sd; }
            }
            const int ddx[4] = {0, -1, 1, 0}, ddy[4] = {-1, 0, 0, 1};
            for (int it = 0; it < cfg.me_iters; it++) {
                int nb = -1, ncost = bcost, nsad = 0;
                for (int k = 0; k < 4; k++) {
                    int x = bx + ddx[k], y = by + ddy[k];
                    if (x < -R || x > R || y < -R || y > R) continue;
                    int sd;
                    int c = cost_of(mbx, mby, x, y, &sd);
                    if (c < ncost) { ncost = c; nb = k; nsad = sd; }
                }
                if (nb < 0) break;
                bx += ddx[nb]; by += ddy[nb]; bcost = ncost; bsad = nsad;
            }
            const int dev = mb_activity(mbx, mby);
            int refi = 0;
            if (t.num_refs > 1 && mb_dirty[idx]) {
                // second reference at the zero vector (a window or caret returning to the
                // state of two pictures ago): worth it when SAD + lambda * 3 bits wins
                const int s1 = sad_at(mbx, mby, 0, 0, t, 1);
                if (s1 + 3 * lam < bcost) {
                    bx = by = 0;
                    bsad = s1;
                    refi = 1;
                }
            }
            me[idx].mvx = (int16_t)bx;
            me[idx].mvy = (int16_t)by;
            me[idx].sad = bsad;
            me[idx].intra_est = dev;
            me[idx].ref = (int16_t)refi;
            me[idx].fx = me[idx].fy = 0;
        }
}

// K4c: quarter-pel refinement of every P macroblock of slice s whose integer SAD is
// above kSubpelMinSad (after the integer search
// and the scene-cut decision): the 8 half-sample neighbours of the integer vector, then
// the 8 quarter-sample neighbours of the best, by SAD against the 6-tap interpolated
// reference (luma_qpel_sample). A candidate replaces the best only if strictly better.
void CpuH264Encoder::subpel_refine(int s) {
    const SliceTask& t = tasks[s];
    const int ylo = t.pic_row0 * 16, yhi = (t.pic_row0 + t.pic_rows) * 16 - 1;
    static const int8_t ring[8][2] = {{-1, -1}, {0, -1}, {1, -1}, {-1, 0}, {1, 0}, {-1, 1}, {0, 1}, {1, 1}};
    StripeState& sst = ctl_.stripes()[s];
    if (!subpel_gate(t.frame_num, sst.subpel_prev, t.num_rows * g.mb_w)) {
        for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
            for (int mbx = 0; mbx < g.mb_w; mbx++) me[(size_t)mby * g.mb_w + mbx].fx = me[(size_t)mby * g.mb_w + mbx].fy = 0;
        return;
    }
    for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) {
            MeResult& r = me[(size_t)mby * g.mb_w + mbx];
            r.fx = r.fy = 0;
            if (r.sad <= kSubpelMinSad) continue;
            const uint8_t* ref = refs(r.ref)[0].data();
            auto sad_q = [&](int qx, int qy) {
                int sad = 0;
                for (int y = 0; y < 16; y++) {
                    const uint8_t* srow = &src[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16];
                    for (int x = 0; x < 16; x++)
                        sad += sk_abs((int)srow[x] - luma_qpel_sample(ref, g.stride_y, g.stride_y, ylo, yhi,
                                                                      mbx * 16 + x, mby * 16 + y, qx, qy));
                }
                return sad;
            };
            int bx = 4 * r.mvx, by = 4 * r.mvy, best = sad_q(bx, by);
            const int int_sad = best;
            for (int step = 2; step >= 1; step--) {
                const int cx = bx, cy = by;
                for (int k = 0; k < 8; k++) {
                    const int qx = cx + step * ring[k][0], qy = cy + step * ring[k][1];
                    const int c = sad_q(qx, qy);
                    if (c < best) {
                        best = c;
                        bx = qx;
                        by = qy;
                    }
                }
            }
            r.fx = (int8_t)(bx - 4 * r.mvx);
            r.fy = (int8_t)(by - 4 * r.mvy);
            sst.subpel_hits += (r.fx | r.fy) != 0 && subpel_hit(best, int_sad);
        }
}

void CpuH264Encoder::decide_scenecut(int s) {
    SliceTask& t = tasks[s];
    t.final_action = t.action;
    if (t.action != ACT_P || !t.allow_scenecut) return;
    long long inter = 0, intra = 0;
    for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) {
            inter += me[mby * g.mb_w + mbx].sad;
            intra += me[mby * g.mb_w + mbx].intra_est;
        }
    if (inter > intra) t.final_action = ACT_I;
}

void CpuH264Encoder::mc_luma(int mbx, int mby, int mvx, int mvy, const SliceTask& t,
                             uint8_t* pred, int refi) const {
    int y_lo = t.pic_row0 * 16, y_hi = (t.pic_row0 + t.pic_rows) * 16 - 1;
    const uint8_t* ref = refs(refi)[0].data();
    for (int y = 0; y < 16; y++)
        for (int x = 0; x < 16; x++)
            pred[y * 16 + x] = (uint8_t)luma_qpel_sample(ref, g.stride_y, g.stride_y, y_lo, y_hi, mbx * 16 + x,
                                                         mby * 16 + y, mvx, mvy);
}

void CpuH264Encoder::mc_chroma(int mbx, int mby, int mvx, int mvy, const SliceTask& t,
                               uint8_t* pu, uint8_t* pv, int refi) const {
    int h = t.pic_rows * 8;
    int y0 = t.pic_row0 * 8;
    for (int c = 0; c < 2; c++) {
        const uint8_t* base = &refs(refi)[1 + c][(size_t)y0 * g.stride_c];
        uint8_t* o = c ? pv : pu;
        for (int y = 0; y < 8; y++)
            for (int x = 0; x < 8; x++)
                o[y * 8 + x] = (uint8_t)chroma_mc_sample(base, g.stride_c, g.stride_c, h, mbx * 8 + x,
                                                         mby * 8 - y0 + y, mvx, mvy);
    }
}

void CpuH264Encoder::code_slice_inter(int s, bool redo) {
    const SliceTask& t = tasks[s];
    if (cfg.subpel && !redo) subpel_refine(s);
    for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) {
            int idx = mby * g.mb_w + mbx;
            MbInfo& mb = mbs[idx];
            memset(&mb, 0, sizeof(mb));
            int mvx = me_qx(me[idx]), mvy = me_qy(me[idx]);
            const int refi = me[idx].ref;
            auto nbr = [&](int ox, int oy, bool ok) {
                MvNb n;
                n.avail = ok;
                n.ref = ok ? me[oy * g.mb_w + ox].ref : -1;
                n.mvx = ok ? me_qx(me[oy * g.mb_w + ox]) : 0;
                n.mvy = ok ? me_qy(me[oy * g.mb_w + ox]) : 0;
                return n;
            };
            bool top = mby > t.first_row;
            MvNb A = nbr(mbx - 1, mby, mbx > 0);
            MvNb B = nbr(mbx, mby - 1, top);
            MvNb C = nbr(mbx + 1, mby - 1, top && mbx + 1 < g.mb_w);
            if (!C.avail) C = nbr(mbx - 1, mby - 1, top && mbx > 0);
            int pmx, pmy, smx, smy;
            mv_pred16x16(A, B, C, refi, &pmx, &pmy);
            mv_pskip(A, B, C, &smx, &smy);

            uint8_t sy[256], su[64], sv[64], py[256], pu[64], pv[64];
            for (int y = 0; y < 16; y++)
                memcpy(sy + y * 16, &src[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16], 16);
            for (int y = 0; y < 8; y++) {
                memcpy(su + y * 8, &src[1][(size_t)(mby * 8 + y) * g.stride_c + mbx * 8], 8);
                memcpy(sv + y * 8, &src[2][(size_t)(mby * 8 + y) * g.stride_c + mbx * 8], 8);
            }
            mc_luma(mbx, mby, mvx, mvy, t, py, refi);
            mc_chroma(mbx, mby, mvx, mvy, t, pu, pv, refi);
            MbTransform tr;
            residual_transform(sy, py, su, pu, sv, pv, tr);
            int16_t* coef = &coefs[(size_t)idx * kCoefPerMb];
            mb.type = MB_P_16x16;
            int qp = quant_mb_with_budget(tr, t.qp, false, mb, coef, host_cavlc_tables(), mb_start_qp(t, idx));
            mb.mvx = (int16_t)mvx;
            mb.mvy = (int16_t)mvy;
            mb.ref = (uint8_t)refi;
            if (mb.cbp == 0 && refi == 0 && mvx == smx && mvy == smy) {
                mb.type = MB_P_SKIP;
            } else {
                mb.mvdx = (int16_t)(mvx - pmx);
                mb.mvdy = (int16_t)(mvy - pmy);
            }
            uint8_t ry[256], ru[64], rv[64];
            recon_luma(coef, qp, false, mb.cbp & 15, py, ry);
            recon_chroma(coef, qp, (mb.cbp >> 4) & 3, pu, pv, ru, rv);
            for (int y = 0; y < 16; y++)
                memcpy(&rec[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16], ry + y * 16, 16);
            for (int y = 0; y < 8; y++) {
                memcpy(&rec[1][(size_t)(mby * 8 + y) * g.stride_c + mbx * 8], ru + y * 8, 8);
                memcpy(&rec[2][(size_t)(mby * 8 + y) * g.stride_c + mbx * 8], rv + y * 8, 8);
            }
        }
}

// Intra 16x16 luma mode (evaluation order DC, V, H, Plane) and chroma mode (DC, H, V,
// Plane) by SAD against the given neighbour samples. Also returns the chroma prediction.
static void intra_decide(const uint8_t* sy, const uint8_t* su, const uint8_t* sv, const uint8_t* top,
                         const uint8_t* left, int tl, const uint8_t (*ctop)[8], const uint8_t (*cleft)[8],
                         const int* ctl, bool aT, bool aL, int* luma_mode, int* chroma_mode,
                         int* luma_sad = nullptr) {
    int dc = i16_dc(top, left, aT, aL);
    int pa = 0, pb = 0, pc = 0;
    if (aT && aL) i16_plane_params(top, left, tl, &pa, &pb, &pc);
    const int order[4] = {2, 0, 1, 3};
    int best_mode = 2, best_sad = 0x7fffffff;
    for (int oi = 0; oi < 4; oi++) {
        int m = order[oi];
        if ((m == 0 && !aT) || (m == 1 && !aL) || (m == 3 && !(aT && aL))) continue;
        int sad = 0;
        for (int y = 0; y < 16; y++)
            for (int x = 0; x < 16; x++)
                sad += sk_abs((int)sy[y * 16 + x] - i16_pred_pixel(m, x, y, top, left, tl, aT, aL, dc, pa, pb, pc));
        if (sad < best_sad) { best_sad = sad; best_mode = m; }
    }
    int best_cm = 0, best_csad = 0x7fffffff;
    for (int m = 0; m < 4; m++) {
        if ((m == 1 && !aL) || (m == 2 && !aT) || (m == 3 && !(aT && aL))) continue;
        int sad = 0;
        for (int c = 0; c < 2; c++) {
            uint8_t p[64];
            intra_chroma_pred(m, ctop[c], cleft[c], ctl[c], aT, aL, p);
            const uint8_t* sp = c ? sv : su;
            for (int i = 0; i < 64; i++) sad += sk_abs((int)sp[i] - (int)p[i]);
        }
        if (sad < best_csad) { best_csad = sad; best_cm = m; }
    }
    *luma_mode = best_mode;
    *chroma_mode = best_cm;
    if (luma_sad) *luma_sad = best_sad;
}

// Luma of an Intra4x4 macroblock at `qp`, block by block in decoding order: prediction
// from `outside(x, y)` (MB-relative samples of the neighbour MBs) and, inside the MB, from
// the blocks reconstructed so far (or the source itself for the open-loop pre-pass);
// chroma levels from trc.wc. Fills coef, nnz, cbp and the luma reconstruction `ry`;
// returns the conservative bit bound (h264_mb.h mb_bits_crude_i16).
template <class S>
static int code_i4_at(int qp, const uint8_t* sy, S outside, bool aT, bool aL, bool aTR, bool open_loop,
                      const MbTransform& trc, MbInfo& mb, int16_t* coef, uint8_t* ry) {
    const uint8_t* inner = open_loop ? sy : ry;
    auto sample = [&](int x, int y) -> int {
        if (x >= 0 && x < 16 && y >= 0) return inner[y * 16 + x];
        return outside(x, y);
    };
    int cbp_l = 0;
    for (int b = 0; b < 16; b++) {
        I4Ref r;
        i4_ref(sample, b, aT, aL, aTR, r);
        const int m = i4_mode(mb, b), bx = blk_x(b) * 4, by = blk_y(b) * 4;
        int pred[16], res[16], w[16], rec[16];
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) {
                pred[y * 4 + x] = i4_pred_px(m, r, x, y);
                res[y * 4 + x] = (int)sy[(by + y) * 16 + bx + x] - pred[y * 4 + x];
            }
        fdct4x4(res, w);
        int16_t* c = coef + kCoefLuma + b * 16;
        const int n = quant_block_i4(w, qp, c);
        mb.nnz[b] = (uint8_t)n;
        if (n) cbp_l |= 1 << (b >> 2);
        recon_block_i4(c, qp, pred, rec);
        for (int y = 0; y < 4; y++)
            for (int x = 0; x < 4; x++) ry[(by + y) * 16 + bx + x] = (uint8_t)rec[y * 4 + x];
    }
    for (int k = 0; k < 16; k++) coef[kCoefLumaDC + k] = 0;
    const int cbp_c = quant_chroma(trc, qp, true, coef, mb.nnz);
    mb.cbp = (uint8_t)(cbp_l | (cbp_c << 4));
    mb.qp = (uint8_t)qp;
    return mb_bits_crude_i16(mb, coef, host_cavlc_tables());
}

// Edges (row above, column left, corner) of MB (mbx, mby) in plane set P.
static void mb_edges(const std::vector<uint8_t>* P, const Geometry& g, int mbx, int mby, bool aT, bool aL,
                     uint8_t* top, uint8_t* left, int* tl, uint8_t (*ctop)[8], uint8_t (*cleft)[8], int* ctl) {
    const int sy_ = g.stride_y, sc = g.stride_c;
    memset(top, 0, 16);
    memset(left, 0, 16);
    memset(ctop, 0, 16);
    memset(cleft, 0, 16);
    *tl = 0;
    ctl[0] = ctl[1] = 0;
    if (aT)
        for (int i = 0; i < 16; i++) top[i] = P[0][(size_t)(mby * 16 - 1) * sy_ + mbx * 16 + i];
    if (aL)
        for (int i = 0; i < 16; i++) left[i] = P[0][(size_t)(mby * 16 + i) * sy_ + mbx * 16 - 1];
    if (aT && aL) *tl = P[0][(size_t)(mby * 16 - 1) * sy_ + mbx * 16 - 1];
    for (int c = 0; c < 2; c++) {
        const std::vector<uint8_t>& Q = P[1 + c];
        if (aT)
            for (int i = 0; i < 8; i++) ctop[c][i] = Q[(size_t)(mby * 8 - 1) * sc + mbx * 8 + i];
        if (aL)
            for (int i = 0; i < 8; i++) cleft[c][i] = Q[(size_t)(mby * 8 + i) * sc + mbx * 8 - 1];
        if (aT && aL) ctl[c] = Q[(size_t)(mby * 8 - 1) * sc + mbx * 8 - 1];
    }
}

// I slices in two passes (same decisions as k_intra_prep + k_code_intra):
//  1. open loop, every MB independent: modes chosen against the SOURCE neighbours and
//     the QP escalation the MB needs with that prediction (the start QP);
//  2. the MB wavefront proper: prediction from the reconstructed neighbours with those
//     modes, quantisation starting at the start QP (escalating further if still needed).
void CpuH264Encoder::code_slice_intra(int s) {
    const SliceTask& t = tasks[s];
    const int sy_ = g.stride_y, sc = g.stride_c;
    const bool split = intra_split(t, g.mb_w, cfg.deblock, cfg.intra4x4);
    const int first = t.first_row * g.mb_w;
    for (int pass = 0; pass < 2; pass++)
        for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
            for (int mbx = 0; mbx < g.mb_w; mbx++) {
                int idx = mby * g.mb_w + mbx;
                MbInfo& mb = mbs[idx];
                bool aT = mby > t.first_row, aL = mbx > 0;
                if (split) {   // K5 sub-slice: left neighbour inside it only, never the top
                    aT = false;
                    aL = aL && (idx - first) % kIntraSubMbs != 0;
                }
                uint8_t top[16], left[16], ctop[2][8], cleft[2][8];
                int tl, ctl[2];
                mb_edges(pass == 0 ? src : rec, g, mbx, mby, aT, aL, top, left, &tl, ctop, cleft, ctl);
                uint8_t sy[256], su[64], sv[64];
                for (int y = 0; y < 16; y++)
                    memcpy(sy + y * 16, &src[0][(size_t)(mby * 16 + y) * sy_ + mbx * 16], 16);
                for (int y = 0; y < 8; y++) {
                    memcpy(su + y * 8, &src[1][(size_t)(mby * 8 + y) * sc + mbx * 8], 8);
                    memcpy(sv + y * 8, &src[2][(size_t)(mby * 8 + y) * sc + mbx * 8], 8);
                }
                int best_mode, best_cm, start_qp = mb_start_qp(t, idx);
                bool i4 = false;
                const bool aTR = aT && mbx + 1 < g.mb_w;
                const std::vector<uint8_t>* P = pass == 0 ? src : rec;
                auto outside = [&](int x, int y) -> int {
                    return P[0][(size_t)(mby * 16 + y) * sy_ + mbx * 16 + x];
                };
                if (pass == 0) {
                    int sad16 = 0;
                    intra_decide(sy, su, sv, top, left, tl, ctop, cleft, ctl, aT, aL, &best_mode, &best_cm, &sad16);
                    if (cfg.intra4x4) {
                        MbInfo cand;
                        memset(&cand, 0, sizeof(cand));
                        auto src_sample = [&](int x, int y) -> int {
                            return (x >= 0 && x < 16 && y >= 0) ? (int)sy[y * 16 + x] : outside(x, y);
                        };
                        const int cost4 = i4_decide(src_sample, sy, aT, aL, aTR, t.qp, cand);
                        if (i4_wins(cost4, sad16, t.qp)) {
                            i4 = true;
                            mb.i4lo = cand.i4lo;
                            mb.i4hi = cand.i4hi;
                        }
                    }
                } else {
                    i4 = mb.type == MB_I4x4;
                    best_mode = mb.i16_mode;
                    best_cm = mb.chroma_mode;
                    start_qp = mb.qp;
                }
                if (i4) {
                    uint8_t pu[64], pv[64], ry[256], ru[64], rv[64];
                    intra_chroma_pred(best_cm, ctop[0], cleft[0], ctl[0], aT, aL, pu);
                    intra_chroma_pred(best_cm, ctop[1], cleft[1], ctl[1], aT, aL, pv);
                    MbTransform trc;
                    residual_transform(sy, sy, su, pu, sv, pv, trc);   // chroma part (luma residual is 0)
                    const uint32_t m_lo = mb.i4lo, m_hi = mb.i4hi;
                    int16_t* coef = &coefs[(size_t)idx * kCoefPerMb];
                    memset(&mb, 0, sizeof(mb));
                    mb.type = MB_I4x4;
                    mb.chroma_mode = (uint8_t)best_cm;
                    mb.i4lo = m_lo;
                    mb.i4hi = m_hi;
                    int qp = start_qp >= 0 ? start_qp : t.qp;
                    const int cap = sk_min(51, t.qp + 24);
                    for (;;) {
                        const int bound = code_i4_at(qp, sy, outside, aT, aL, aTR, pass == 0, trc, mb, coef, ry);
                        if (qp + 6 > cap || bound <= mb_bit_budget(true)) break;
                        qp += 6;
                    }
                    if (pass == 0) continue;   // mb keeps type, modes and the start QP for pass 2
                    me[idx].mvx = me[idx].mvy = 0;
                    me[idx].ref = 0;
                    me[idx].fx = me[idx].fy = 0;
                    recon_chroma(coef, qp, (mb.cbp >> 4) & 3, pu, pv, ru, rv);
                    for (int y = 0; y < 16; y++)
                        memcpy(&rec[0][(size_t)(mby * 16 + y) * sy_ + mbx * 16], ry + y * 16, 16);
                    for (int y = 0; y < 8; y++) {
                        memcpy(&rec[1][(size_t)(mby * 8 + y) * sc + mbx * 8], ru + y * 8, 8);
                        memcpy(&rec[2][(size_t)(mby * 8 + y) * sc + mbx * 8], rv + y * 8, 8);
                    }
                    continue;
                }
                int dc = i16_dc(top, left, aT, aL);
                int pa = 0, pb = 0, pc = 0;
                if (aT && aL) i16_plane_params(top, left, tl, &pa, &pb, &pc);
                uint8_t py[256], pu[64], pv[64];
                for (int y = 0; y < 16; y++)
                    for (int x = 0; x < 16; x++)
                        py[y * 16 + x] = (uint8_t)i16_pred_pixel(best_mode, x, y, top, left, tl, aT, aL, dc, pa, pb, pc);
                intra_chroma_pred(best_cm, ctop[0], cleft[0], ctl[0], aT, aL, pu);
                intra_chroma_pred(best_cm, ctop[1], cleft[1], ctl[1], aT, aL, pv);
                MbTransform tr;
                residual_transform(sy, py, su, pu, sv, pv, tr);
                int16_t* coef = &coefs[(size_t)idx * kCoefPerMb];
                memset(&mb, 0, sizeof(mb));
                mb.type = MB_I16x16;
                mb.i16_mode = (uint8_t)best_mode;
                mb.chroma_mode = (uint8_t)best_cm;
                int qp = quant_mb_with_budget(tr, t.qp, true, mb, coef, host_cavlc_tables(), start_qp);
                if (pass == 0) continue;   // mb keeps the modes and the start QP for pass 2
                me[idx].mvx = me[idx].mvy = 0;
                me[idx].ref = 0;
                me[idx].fx = me[idx].fy = 0;
                uint8_t ry[256], ru[64], rv[64];
                recon_luma(coef, qp, true, mb.cbp & 15, py, ry);
                recon_chroma(coef, qp, (mb.cbp >> 4) & 3, pu, pv, ru, rv);
                for (int y = 0; y < 16; y++)
                    memcpy(&rec[0][(size_t)(mby * 16 + y) * sy_ + mbx * 16], ry + y * 16, 16);
                for (int y = 0; y < 8; y++) {
                    memcpy(&rec[1][(size_t)(mby * 8 + y) * sc + mbx * 8], ru + y * 8, 8);
                    memcpy(&rec[2][(size_t)(mby * 8 + y) * sc + mbx * 8], rv + y * 8, 8);
                }
            }
}

void CpuH264Encoder::code_slice_skipall(int s) {
    const SliceTask& t = tasks[s];
    for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) {
            int idx = mby * g.mb_w + mbx;
            memset(&mbs[idx], 0, sizeof(MbInfo));
            me[idx].mvx = me[idx].mvy = 0;
            me[idx].ref = 0;
            me[idx].fx = me[idx].fy = 0;
        }
    int y0 = t.first_row * 16, y1 = (t.first_row + t.num_rows) * 16;
    memcpy(&rec[0][(size_t)y0 * g.stride_y], &ref[0][(size_t)y0 * g.stride_y], (size_t)(y1 - y0) * g.stride_y);
    for (int p = 1; p < 3; p++)
        memcpy(&rec[p][(size_t)(y0 / 2) * g.stride_c], &ref[p][(size_t)(y0 / 2) * g.stride_c],
               (size_t)(y1 - y0) / 2 * g.stride_c);
}

void CpuH264Encoder::mb_neighbours(int mbx, int mby, int first_row, MbNeighbours& nb, int sub0) const {
    const int idx = mby * g.mb_w + mbx;
    nb.left = mbx > 0 && idx - 1 >= sub0 ? &mbs[idx - 1] : nullptr;
    nb.top = mby > first_row && idx - g.mb_w >= sub0 ? &mbs[idx - g.mb_w] : nullptr;
}

std::vector<std::vector<uint8_t>> CpuH264Encoder::write_slice(int s) {
    const SliceTask& t = tasks[s];
    const int nmb = t.num_rows * g.mb_w, first = t.first_row * g.mb_w;
    bool intra = t.final_action == ACT_I;
    // one NAL per sub-slice of a split I slice (K5), else one for the slice
    const bool split = intra_split(t, g.mb_w, cfg.deblock, cfg.intra4x4);
    const int nsub = split ? intra_sub_count(nmb) : 1, sub_len = split ? kIntraSubMbs : nmb;
    std::vector<std::vector<uint8_t>> nals;
    for (int j = 0; j < nsub; j++) {
        const int k0 = j * sub_len, k1 = sk_min(nmb, k0 + sub_len);   // stripe-relative MB range
        std::vector<uint8_t> buf((size_t)(k1 - k0) * (kMaxMbBits / 8 + 16) + 64, 0);
        BitWriter w(buf.data());
        SliceHeaderParams h;
        h.first_mb = (cfg.fullframe ? first : 0) + k0;
        h.slice_type = intra ? 2 : 0;
        h.idr = intra && t.idr_on_intra;
        h.frame_num = h.idr ? 0 : t.frame_num;
        h.idr_pic_id = t.idr_pic_id;
        h.slice_qp = t.qp;
        h.deblock = slice_deblock(cfg.deblock, t);
        h.num_refs = intra ? 1 : t.num_refs;
        write_slice_header(w, h);
        if (t.final_action == ACT_SKIPALL) {
            put_ue(w, (uint32_t)nmb);
        } else {
            int skip_run = 0, qp_prev = t.qp;
            for (int k = k0; k < k1; k++) {
                const int idx = first + k, mbx = idx % g.mb_w, mby = idx / g.mb_w;
                const MbInfo& mb = mbs[idx];
                if (mb.type == MB_P_SKIP) { skip_run++; continue; }
                if (!intra) { put_ue(w, (uint32_t)skip_run); skip_run = 0; }
                int dq = 0;
                if (mb_has_qp_delta(mb)) { dq = mb.qp - qp_prev; qp_prev = mb.qp; }
                MbNeighbours nb;
                mb_neighbours(mbx, mby, t.first_row, nb, first + k0);
                write_mb_header(w, mb, !intra, dq, intra ? 1 : t.num_refs, nb);
                write_mb_residual(w, mb, nb, &coefs[(size_t)idx * kCoefPerMb], host_cavlc_tables());
            }
            if (skip_run > 0) put_ue(w, (uint32_t)skip_run);
        }
        w.put1(1);
        while (w.pos & 7) w.put1(0);
        buf.resize(w.pos / 8);
        nals.push_back(std::move(buf));
    }
    return nals;
}

void CpuH264Encoder::package(uint16_t frame_id, std::vector<std::vector<std::vector<uint8_t>>>& rbsp,
                             std::vector<EncodedPacket>& out) {
    if (cfg.fullframe) {
        bool idr = ctl_.picture_is_idr(tasks.data());
        EncodedPacket pk;
        pk.y = 0; pk.w = g.W; pk.h = g.H; pk.key = idr;
        pk.data.resize(10);
        write_stripe_header(pk.data.data(), idr, frame_id, 0, g.W, g.H);
        if (idr) pk.data.insert(pk.data.end(), param_sets[0].begin(), param_sets[0].end());
        for (int s = 0; s < g.num_slices; s++) {
            const SliceTask& t = tasks[s];
            int hdr = (t.final_action == ACT_I && idr) ? 0x65 : 0x41;
            for (const auto& n : rbsp[s]) append_nal(pk.data, hdr, n.data(), n.size());
        }
        out.push_back(std::move(pk));
        return;
    }
    for (int s = 0; s < g.num_slices; s++) {
        const SliceTask& t = tasks[s];
        if (t.final_action == ACT_NONE) continue;
        bool idr = t.final_action == ACT_I;
        EncodedPacket pk;
        pk.y = g.slice_pix_y(s); pk.w = g.W; pk.h = g.slice_pix_h(s); pk.key = idr;
        pk.data.resize(10);
        write_stripe_header(pk.data.data(), idr, frame_id, pk.y, pk.w, pk.h);
        if (idr) pk.data.insert(pk.data.end(), param_sets[s].begin(), param_sets[s].end());
        for (const auto& n : rbsp[s]) append_nal(pk.data, idr ? 0x65 : 0x41, n.data(), n.size());
        out.push_back(std::move(pk));
    }
}

void CpuH264Encoder::finish_frame() {
    for (int s = 0; s < g.num_slices; s++) {
        const SliceTask& t = tasks[s];
        const int y0 = t.first_row * 16, y1 = (t.first_row + t.num_rows) * 16;
        if (cfg.num_refs > 1 && t.final_action != ACT_NONE) {
            // sliding window: the picture before the one being added becomes reference 1
            // (a skip-all picture is a reference too: ref 1 = the old ref 0 = its content)
            memcpy(&ref1[0][(size_t)y0 * g.stride_y], &ref[0][(size_t)y0 * g.stride_y], (size_t)(y1 - y0) * g.stride_y);
            for (int p = 1; p < 3; p++)
                memcpy(&ref1[p][(size_t)(y0 / 2) * g.stride_c], &ref[p][(size_t)(y0 / 2) * g.stride_c],
                       (size_t)(y1 - y0) / 2 * g.stride_c);
        }
        if (t.final_action == ACT_NONE || t.final_action == ACT_SKIPALL) {
            if (t.final_action == ACT_SKIPALL)
                for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
                    for (int mbx = 0; mbx < g.mb_w; mbx++) {
                        int j = mby * g.mb_w + mbx;
                        mvfield[2 * j] = mvfield[2 * j + 1] = 0;
                    }
            continue;
        }
        memcpy(&ref[0][(size_t)y0 * g.stride_y], &rec[0][(size_t)y0 * g.stride_y], (size_t)(y1 - y0) * g.stride_y);
        for (int p = 1; p < 3; p++)
            memcpy(&ref[p][(size_t)(y0 / 2) * g.stride_c], &rec[p][(size_t)(y0 / 2) * g.stride_c],
                   (size_t)(y1 - y0) / 2 * g.stride_c);
        if (slice_deblock(cfg.deblock, t)) {  // K7: the reference picture is the deblocked reconstruction
            const int sub_len = intra_split(t, g.mb_w, cfg.deblock, cfg.intra4x4) ? kIntraSubMbs : 0;
            db_slice_info(mbs.data(), g.mb_w, t.first_row, t.num_rows, t.qp, dbinfo.data(), sub_len);
            deblock_slice_cpu(ref[0].data(), ref[1].data(), ref[2].data(), g.stride_y, g.stride_c, dbinfo.data(),
                              g.mb_w, t.first_row, t.num_rows, sub_len);
        }
        for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
            for (int mbx = 0; mbx < g.mb_w; mbx++) {
                int j = mby * g.mb_w + mbx;
                mvfield[2 * j] = me[j].mvx;
                mvfield[2 * j + 1] = me[j].mvy;
            }
    }
    for (int p = 0; p < 3; p++) prev[p].swap(src[p]);
    ctl_.commit(tasks.data());
    first_frame = false;
}

// Per-MB AQ offsets from the source luma (same integer math as k_aq).
void CpuH264Encoder::compute_aq(int s) {
    if (cfg.aq_strength <= 0) return;
    if (aq.size() != (size_t)g.num_mbs()) aq.assign(g.num_mbs(), 0);
    const SliceTask& t = tasks[s];
    for (int mby = t.first_row; mby < t.first_row + t.num_rows; mby++)
        for (int mbx = 0; mbx < g.mb_w; mbx++) {
            uint32_t sum = 0, ssq = 0;
            for (int y = 0; y < 16; y++) {
                const uint8_t* r = &src[0][(size_t)(mby * 16 + y) * g.stride_y + mbx * 16];
                for (int x = 0; x < 16; x++) {
                    sum += r[x];
                    ssq += (uint32_t)r[x] * r[x];
                }
            }
            aq[(size_t)mby * g.mb_w + mbx] = (int8_t)aq_offset(aq_energy(sum, ssq), cfg.aq_strength);
        }
}

void CpuH264Encoder::encode(const uint8_t* bgrx, int stride, uint16_t frame_id,
                            std::vector<EncodedPacket>& out) {
    load_frame(bgrx, stride);
    ctl_.plan(stripe_dirty.data(), tasks.data());
    for (auto& st : ctl_.stripes()) {   // k_plan rotates the same pair on the GPU
        st.subpel_prev = st.subpel_hits;
        st.subpel_hits = 0;
    }
    for (int s = 0; s < g.num_slices; s++)
        if (tasks[s].action == ACT_P) {
            motion_search(s);
            decide_scenecut(s);
        } else if (tasks[s].action == ACT_I) {
            intra_activity(s);
        }
    ctl_.rate_control(tasks.data(), me.data());   // K10 (ratecontrol.h)
    std::vector<std::vector<std::vector<uint8_t>>> rbsp(g.num_slices);
    // K10 accounting unit: slice RBSP payload bits (k_rc_account reads the same sizes)
    auto payload_bits = [&] {
        long long b = 0;
        for (int s = 0; s < g.num_slices; s++)
            if (tasks[s].final_action != ACT_NONE)
                for (const auto& n : rbsp[s]) b += 8 * (long long)n.size();
        return b;
    };
    for (int s = 0; s < g.num_slices; s++) {
        if (tasks[s].final_action == ACT_P || tasks[s].final_action == ACT_I) compute_aq(s);
        switch (tasks[s].final_action) {
            case ACT_P: code_slice_inter(s); break;
            case ACT_I: code_slice_intra(s); break;
            case ACT_SKIPALL: code_slice_skipall(s); break;
            default: continue;
        }
        rbsp[s] = write_slice(s);
    }
    long long bits = payload_bits();
    // CBR guard: a frame that overflows the VBV is coded again, coarser (k_rc_guard)
    if (ctl_.rate_redo(tasks.data(), bits)) {
        for (int s = 0; s < g.num_slices; s++) {
            if (tasks[s].final_action == ACT_P) code_slice_inter(s, true);
            else if (tasks[s].final_action == ACT_I) code_slice_intra(s);
            else continue;
            rbsp[s] = write_slice(s);
        }
        bits = payload_bits();
    }
    package(frame_id, rbsp, out);
    ctl_.rate_account(bits);
    finish_frame();
}

}  // namespace h264
}  // namespace sk
