// Session-level H.264 encoder interface: configuration, geometry, per-stripe
// control state (damage / paint-over / keyframe decisions) and the frame plan
// handed to an execution backend (CPU reference or the HIP pipeline).
//
// Stripe semantics mirror the pixelflux contract used by the reference server
// (selkies.py:2919-2964 CaptureSettings; client demux selkies-core.js:2925-3032):
//  * striped mode: every stripe is an independent H.264 stream (own SPS/PPS,
//    own IDR) emitted as a 0x04 packet [type|key|frame_id|y|w|h] + Annex-B;
//    undamaged stripes emit nothing.
//  * full-frame mode (encoder "x264enc"): one picture whose slices are the
//    stripes, emitted as a single 0x04 packet with y = 0.
#pragma once
#include <string.h>
#include <stdint.h>
#include <vector>
#include <string>
#include "h264_core.h"
#include "ratecontrol.h"

namespace sk {
namespace h264 {

struct EncoderConfig {
    int width = 1920;
    int height = 1080;
    int stripe_height = 64;      // pixels, multiple of 16
    int fullframe = 0;
    int full_range = 0;          // h264_fullcolor
    int qp = 25;                 // h264_crf mapped to a constant QP
    int paint_qp = 18;           // h264_paintover_crf
    int use_paint_over = 1;
    int paint_over_trigger = 15;
    int paint_over_burst = 5;
    int streaming_mode = 0;
    int damage_threshold = 10;
    int damage_duration = 20;
    int me_range = 64;           // max |mv| in integer pixels
    int me_iters = 24;           // diamond refinement iterations
    int scenecut = 1;
    float fps = 60.f;
    int deblock = 2;             // in-loop deblocking (idc 2: inside each slice): 0 off (x264 ultrafast), 1 on,
                                 // 2 automatic: the slices coded at QP >= kAutoDeblockQp (slice_deblock)
    int me_full = 1;             // +-16 exhaustive MFMA search candidate (dirty MBs of P slices)
    int shared_copy = 0;         // HIP: uploads on the device's shared copy stream (in submit order)
    int num_refs = 1;            // reference frames per stream (sliding-window DPB): 1, or 2 for the
                                 // previous-but-one picture as a second P reference (blinking/toggling UI)
    int src_width = 0;           // K2: capture size when it differs from width x height (0 = same);
    int src_height = 0;          //     the frame is resampled (bilinear) inside the K1 conversion
    int codec = 0;               // 0 = H.264, 1 = HEVC (hevc_encoder.h: same front end, full frame), 2 = AV1
    int tile_cols_log2 = -1;     // AV1 tiles (av1_encoder.h): -1 = automatic
    int tile_rows_log2 = -1;
    int rc_mode = RC_CQP;        // K10 rate control (ratecontrol.h): CQP, CRF (qp = CRF value), CBR
    int bitrate_kbps = 0;        // CBR target
    int vbv_ms = 0;              // CBR buffer (ratecontrol.h rc_init): 0 = 1.5 frame intervals
    int aq_strength = 0;         // MB-level adaptive QP strength, Q4 (16 = 1.0; 0 = off): h264_mb.h aq_offset
    int subpel = 1;              // quarter-pel refinement of P vectors (K4c, H.264 and HEVC); AV1 keeps integer vectors
    int intra4x4 = 0;            // H.264 I slices may code MBs as I_NxN (nine 4x4 modes) where cheaper; off
                                 // by default like x264's ultrafast preset (partitions none)
};

struct Geometry {
    int W = 0, H = 0, mb_w = 0, mb_h = 0, rows_per_slice = 0, num_slices = 0;
    int stride_y = 0, stride_c = 0, plane_h_y = 0, plane_h_c = 0;
    int fullframe = 0, stripe_height = 0;
    void init(const EncoderConfig& c) {
        W = c.width;
        H = c.height;
        fullframe = c.fullframe;
        stripe_height = c.stripe_height;
        mb_w = (W + 15) / 16;
        mb_h = (H + 15) / 16;
        rows_per_slice = c.stripe_height / 16;
        if (rows_per_slice < 1) rows_per_slice = 1;
        num_slices = (mb_h + rows_per_slice - 1) / rows_per_slice;
        stride_y = mb_w * 16;
        stride_c = mb_w * 8;
        plane_h_y = mb_h * 16;
        plane_h_c = mb_h * 8;
    }
    int slice_first_row(int s) const { return s * rows_per_slice; }
    int slice_rows(int s) const {
        int r = mb_h - s * rows_per_slice;
        return r < rows_per_slice ? r : rows_per_slice;
    }
    int slice_pix_y(int s) const { return s * rows_per_slice * 16; }
    int slice_pix_h(int s) const {
        int y0 = slice_pix_y(s);
        int y1 = y0 + slice_rows(s) * 16;
        if (y1 > H) y1 = H;
        return y1 - y0;
    }
    int num_mbs() const { return mb_w * mb_h; }
};

// Per-slice work item for one frame (POD, copied to device memory as is).
enum SliceAction : int32_t { ACT_NONE = 0, ACT_P = 1, ACT_I = 2, ACT_SKIPALL = 3 };
struct SliceTask {
    int32_t action;        // SliceAction requested by the controller
    int32_t qp;
    int32_t first_row;     // MB rows of the slice
    int32_t num_rows;
    int32_t pic_row0;      // first MB row of the picture this slice belongs to
    int32_t pic_rows;      // MB rows of that picture (MC clamp bounds)
    int32_t frame_num;     // frame_num if coded as P (or non-IDR I)
    int32_t idr_pic_id;    // idr_pic_id if coded as IDR
    int32_t allow_scenecut;
    int32_t idr_on_intra;  // striped mode: an I decision makes the stripe an IDR
    int32_t final_action;  // written by the backend (scene-cut may turn P into I)
    int32_t num_refs;      // P: reference pictures available to this slice (1..EncoderConfig::num_refs)
};
static_assert(sizeof(SliceTask) == 48, "SliceTask layout");

// K5 parallel key frames. An I slice of a stripe wider than kIntraSubMbs macroblocks is
// coded as sub-slices of kIntraSubMbs MBs each (consecutive in raster order, so most
// start mid-row: first_mb_in_slice at any MB). The reference's encoders split pictures
// the same way (num-slices 4, legacy/gstwebrtc_app.py:504, 538, 663). Since
// kIntraSubMbs < mb_w, no MB has its top neighbour in its own sub-slice: a sub-slice
// predicts from its left neighbours only, its reconstruction chain is at most
// kIntraSubMbs MBs long, and the sub-slices of a stripe are independent (one wave
// each on the GPU, k_code_intra_sub). With in-loop deblocking (disable_deblocking_filter_idc
// 2) the filter keeps off the sub-slice edges and restarts the QP_Y chain at each
// sub-slice (h264_deblock.h, k_deblock_prep / k_deblock_edges); Intra4x4 blocks see no
// top or top-right neighbour outside their sub-slice (k_code_intra_sub's I_NxN path).
constexpr int kIntraSubMbs = 40;
// Automatic deblocking (EncoderConfig::deblock = 2): a slice is filtered when it is coded
// at QP >= 34 - CBR under a tight budget, where the 4x4 / 16x16 block edges become
// visible - and left unfiltered at the CRF-25 default, as x264's ultrafast preset
// (legacy/gstwebrtc_app.py:637). Per slice, in its disable_deblocking_filter_idc (2 or 1):
// the stripes of one frame run at different (dithered) QPs.
constexpr int kAutoDeblockQp = 34;
SK_HD bool slice_deblock(int deblock, const SliceTask& t) {
    return deblock == 1 || (deblock == 2 && t.qp >= kAutoDeblockQp);
}
SK_HD bool intra_split(const SliceTask& t, int mb_w, int deblock, int intra4x4) {
    (void)deblock;
    (void)intra4x4;
    return t.final_action == ACT_I && mb_w > kIntraSubMbs;
}
// Sub-slices of a split I slice; nmb = its MBs.
SK_HD int intra_sub_count(int nmb) { return (nmb + kIntraSubMbs - 1) / kIntraSubMbs; }
// Upper bound of the NALs one stripe's slice can need (the GPU's per-stripe NAL slots).
SK_HD int max_nals_per_slice(int rows_per_slice, int mb_w) {
    return mb_w > kIntraSubMbs ? intra_sub_count(rows_per_slice * mb_w) : 1;
}

// K10: slices whose QP the rate controller sets: coded, and not a paint-over refresh
// (CRF; under CBR the refresh is budgeted like any other slice)
SK_HD bool rc_slice_adjustable(const SliceTask& t, int plan_qp, int mode = 1) {
    return (t.final_action == ACT_P || t.final_action == ACT_I) && (t.qp == plan_qp || mode == 2);
}

struct StripeState {
    int frame_num = 0;     // next frame_num
    int idr_pic_id = 0;
    bool need_idr = true;
    int static_frames = 0;
    int dirty_streak = 0;
    int hot_left = 0;
    int paint_left = 0;
    bool painted = true;   // nothing to paint before the first change
    int refs = 0;          // pictures in the decoder's DPB for this stream (sliding window)
    int subpel_hits = 0;   // MBs of this stripe's last frame given a fractional vector (K4c)
    int subpel_prev = 0;   // the same count one frame earlier: the adaptive refinement gate
};

// Controller knobs as a POD, so the same plan code runs on the host (CPU
// backend) and inside the HIP graph (k_plan), bit-for-bit the same decisions.
struct PlanConfig {
    int32_t fullframe, scenecut, use_paint_over, paint_over_trigger, paint_over_burst;
    int32_t damage_threshold, damage_duration, streaming_mode, qp, paint_qp, num_refs;
};
inline PlanConfig plan_config(const EncoderConfig& c) {
    return PlanConfig{c.fullframe, c.scenecut, c.use_paint_over, c.paint_over_trigger, c.paint_over_burst,
                      c.damage_threshold, c.damage_duration, c.streaming_mode, c.qp, c.paint_qp,
                      c.num_refs > 1 ? 2 : 1};
}
constexpr int kFrameNumMask = (1 << 16) - 1;  // log2_max_frame_num = 16 (h264_syntax.h)

// One stripe's decision for this frame; `pic` is the picture state (full-frame mode).
SK_HD void plan_stripe(const PlanConfig& c, StripeState& st, const StripeState& pic, bool d,
                              int first_row, int num_rows, int mb_h, SliceTask& t) {
    const bool ff = c.fullframe != 0;
    t = SliceTask{};
    t.first_row = first_row;
    t.num_rows = num_rows;
    t.pic_row0 = ff ? 0 : first_row;
    t.pic_rows = ff ? mb_h : num_rows;
    t.allow_scenecut = c.scenecut;
    t.idr_on_intra = ff ? 0 : 1;
    if (d) {
        st.static_frames = 0;
        st.dirty_streak++;
        st.painted = false;
        st.paint_left = 0;
        if (st.dirty_streak >= c.damage_threshold) st.hot_left = c.damage_duration;
    } else {
        st.static_frames++;
        st.dirty_streak = 0;
        if (st.hot_left > 0) st.hot_left--;
        if (c.use_paint_over && !st.painted && st.static_frames >= c.paint_over_trigger && st.hot_left == 0) {
            st.painted = true;
            st.paint_left = c.paint_over_burst;
        }
    }
    bool paint = false;
    if (!d && st.paint_left > 0) {
        paint = true;
        st.paint_left--;
    }
    t.qp = paint ? c.paint_qp : c.qp;
    const bool need_idr = ff ? pic.need_idr : st.need_idr;
    if (need_idr) {  // a keyframe counts as a change for paint-over purposes
        st.painted = false;
        st.static_frames = 0;
        t.action = ACT_I;
        t.allow_scenecut = 0;
    } else if (d || paint || st.hot_left > 0 || c.streaming_mode) {
        t.action = ACT_P;
    } else {
        t.action = ff ? ACT_SKIPALL : ACT_NONE;
    }
    if (ff) {
        t.frame_num = need_idr ? 0 : pic.frame_num;
        t.idr_pic_id = pic.idr_pic_id;
        if (need_idr) t.idr_on_intra = 1;
    } else {
        t.frame_num = st.frame_num;
        t.idr_pic_id = st.idr_pic_id;
    }
    const int refs = ff ? pic.refs : st.refs;
    t.num_refs = refs < 1 ? 1 : (refs < c.num_refs ? refs : c.num_refs);
    t.final_action = t.action;
}

// Striped mode: stripe state after its slice was coded with `final_action`.
SK_HD void commit_stripe(StripeState& st, int final_action, int max_refs) {
    if (final_action == ACT_I) {
        st.frame_num = 1;
        st.idr_pic_id = (st.idr_pic_id + 1) & 0xffff;
        st.need_idr = false;
        st.refs = 1;
    } else if (final_action == ACT_P) {
        st.frame_num = (st.frame_num + 1) & kFrameNumMask;
        st.refs = st.refs + 1 < max_refs ? st.refs + 1 : max_refs;
    }
}

// Full-frame mode: picture state after a picture (IDR iff every slice was an IDR slice).
SK_HD void commit_picture(StripeState& pic, bool idr, int max_refs) {
    if (idr) {
        pic.frame_num = 1;
        pic.idr_pic_id = (pic.idr_pic_id + 1) & 0xffff;
        pic.need_idr = false;
        pic.refs = 1;
    } else {
        pic.frame_num = (pic.frame_num + 1) & kFrameNumMask;
        pic.refs = pic.refs + 1 < max_refs ? pic.refs + 1 : max_refs;
    }
}

struct MeResult;

// K10 frame QP from per-slice complexity sums (sad: motion-compensated SAD of the
// slice's MBs, dev: their source activity; both only for slices planned as P, where
// the motion search ran). Same code for the CPU controller and k_rc_qp.
SK_HD void rc_apply(RcState& rc, SliceTask* tasks, const long long* sad, const long long* dev, int ns, int mb_w,
                    int plan_qp, int stride = 1) {
    if (rc.mode == RC_CQP) return;
    long long cp = 0, ci = 0;
    int np = 0, ni = 0, ni_known = 0, nidr = 0;
    for (int s = 0; s < ns; s++) {
        const SliceTask& t = tasks[s];
        if (!rc_slice_adjustable(t, plan_qp, rc.mode)) continue;
        const int mbs = t.num_rows * mb_w;
        if (t.final_action == ACT_P) {
            cp += sad[(size_t)s * stride];
            np += mbs;
        } else {
            ni += mbs;
            if (t.action == ACT_I) nidr += mbs;   // planned key frame (IDR), not a scene cut
            {   // scene cut (ME's intra estimate) or planned key frame (MB activity, no search)
                ci += dev[(size_t)s * stride];
                ni_known += mbs;
            }
        }
    }
    if (np + ni == 0) return;
    const bool intra = ni > np;
    const int qpf = intra ? rc_frame_qpf(rc, ci, ni_known, true, nidr * 2 > ni, np + ni)
                          : rc_frame_qpf(rc, cp, np, false, false, np + ni);
    for (int s = 0, i = 0; s < ns; s++)
        if (rc_slice_adjustable(tasks[s], plan_qp, rc.mode)) tasks[s].qp = rc_clamp_qp(rc, rc_dither_qp(qpf, i++));
}

// K10 CBR guard on a coded frame of `frame_bits` payload bits: when it overflows the
// VBV, every rate-controlled slice (coded at the frame QP) moves rc_redo_step coarser
// for a second coding pass. Returns the step applied (0: keep the frame).
SK_HD int rc_redo(RcState& rc, SliceTask* tasks, int ns, long long frame_bits) {
    const int step = rc_redo_step(rc, frame_bits);
    if (!step) return 0;
    const int f0 = rc.cur_qpf, f1 = sk_min(f0 + (step << 8), rc.qp_max << 8);
    rc_raise_floor(rc);
    if (f1 == f0) return 0;
    rc.redo_qpf = f0;   // the pass being replaced: a slope for a further step and the model point
    rc.redo_bits = (int32_t)(frame_bits > (1ll << 30) ? (1ll << 30) : frame_bits);
    // the frame's slices sit at the two QPs of its dither (rc_dither_qp)
    const int lo = f0 >> 8, hi = (f0 + 255) >> 8;
    for (int s = 0; s < ns; s++) {
        SliceTask& t = tasks[s];
        if ((t.final_action == ACT_P || t.final_action == ACT_I) && (t.qp == lo || t.qp == hi))
            t.qp = rc_clamp_qp(rc, t.qp + step);
    }
    rc.cur_qpf = f1;
    rc.cur_qp = (f1 + 128) >> 8;
    rc.lam_boost = rc_lam_boost(f1);
    rc.redos++;
    rc.cur_redo++;
    return (f1 - f0 + 255) >> 8;
}

// Decides, per stripe, what to encode this frame.
class Controller {
   public:
    void init(const EncoderConfig& cfg, const Geometry& g);
    void request_keyframe();
    // Rate control: QP for changed stripes / paint-over from the next frame on.
    void set_qp(int qp, int paint_qp) {
        if (qp > 0) cfg_.qp = rc_.base_qp = qp;
        if (paint_qp > 0) cfg_.paint_qp = paint_qp;
    }
    // K10: mode (RC_CQP / RC_CRF / RC_CBR) and CBR bitrate from the next frame on.
    void set_rate(int mode, int kbps) {
        const RcState old = rc_;
        rc_init(rc_, mode, cfg_.qp, kbps, cfg_.fps, cfg_.width * cfg_.height, cfg_.vbv_ms, old.codec);
        if (old.mode == mode) {   // keep the model; a new budget recentres the buffer
            for (int k = 0; k < 2; k++) {
                rc_.last_qp[k] = old.last_qp[k];
                rc_.last_qpf[k] = old.last_qpf[k];
                rc_.last_bits[k] = old.last_bits[k];
                rc_.last_cplx[k] = old.last_cplx[k];
            }
            rc_.cplx_ema = old.cplx_ema;
        }
    }
    // K10 per frame: QP of the coded, non-paint-over slices from the frame complexity
    // (after motion search / scene cut), then the coded size.
    void rate_control(SliceTask* tasks, const MeResult* me);
    void rate_account(long long frame_bits) { rc_account(rc_, frame_bits); }
    int rate_redo(SliceTask* tasks, long long frame_bits) { return rc_redo(rc_, tasks, g_.num_slices, frame_bits); }
    RcState& rc() { return rc_; }
    // dirty[s] = stripe s changed since last frame. Fills tasks[num_slices].
    void plan(const uint8_t* dirty, SliceTask* tasks);
    // After the backend ran: update frame_num / idr state from final actions.
    void commit(const SliceTask* tasks);
    bool picture_is_idr(const SliceTask* tasks) const;
    const std::vector<StripeState>& stripes() const { return st_; }
    std::vector<StripeState>& stripes() { return st_; }
    // Session-state transfer (EncoderState): committed stripe states + picture state.
    void export_states(StripeState* out) const {
        for (size_t s = 0; s < st_.size(); s++) out[s] = st_[s];
        out[st_.size()] = pic_;
    }
    void import_states(const StripeState* in) {
        for (size_t s = 0; s < st_.size(); s++) st_[s] = in[s];
        pic_ = in[st_.size()];
    }
    int qp() const { return cfg_.qp; }
    int paint_qp() const { return cfg_.paint_qp; }

   private:
    EncoderConfig cfg_;
    Geometry g_;
    std::vector<StripeState> st_;
    StripeState pic_;  // full-frame mode picture state
    RcState rc_;
};



// ---- session state transfer --------------------------------------------------
// Portable snapshot of everything that carries over from one frame to the next,
// identical for the CPU and HIP backends (so a session can move between GPUs, or
// between a GPU and the CPU reference, without an IDR):
//   StateHeader | StripeState[num_slices + 1] (committed; last = picture state) |
//   ref Y U V | ref1 Y U V (second reference) | last source Y U V (damage baseline) |
//   mvfield int16[2 * num_mbs]
// Session state (parallel/migrate.py), the same for every codec and both backends:
//   StateHeader | StripeState[num_slices + 1] (controller; the last is the picture's, whose
//   frame_num is also the next HEVC POC) | RcState (K10) | ref | ref1 | last source
//   (4:2:0 planes) | MV field. The reference planes are what the next frame predicts from
//   (HEVC: after deblocking + SAO, AV1: after loop filter + CDEF).
struct StateHeader {
    char magic[4];          // "SKH4"
    int32_t version;        // 3 (codec, RcState)
    int32_t W, H, stripe_height, fullframe, num_slices;
    int32_t started;        // a frame has been encoded (else the next one is all-dirty)
    int32_t qp, paint_qp;   // rate-control QPs in force
    int32_t codec;          // EncoderConfig::codec
    int32_t reserved[5];
};
static_assert(sizeof(StateHeader) == 64, "StateHeader layout");

inline size_t state_plane_bytes(const Geometry& g) {
    return (size_t)g.stride_y * g.plane_h_y + 2 * (size_t)g.stride_c * g.plane_h_c;
}
inline size_t state_head_bytes(const Geometry& g) {   // header + controller + rate control
    return sizeof(StateHeader) + sizeof(StripeState) * (size_t)(g.num_slices + 1) + sizeof(RcState);
}
inline size_t state_bytes(const Geometry& g) {
    return state_head_bytes(g) + 3 * state_plane_bytes(g) + sizeof(int16_t) * 2 * (size_t)g.num_mbs();
}
inline void state_header(const EncoderConfig& c, const Geometry& g, int started, int qp, int paint_qp,
                         StateHeader& h) {
    memset(&h, 0, sizeof(h));
    memcpy(h.magic, "SKH4", 4);
    h.version = 3;
    h.codec = c.codec;
    h.W = g.W;
    h.H = g.H;
    h.stripe_height = c.stripe_height;
    h.fullframe = c.fullframe;
    h.num_slices = g.num_slices;
    h.started = started;
    h.qp = qp;
    h.paint_qp = paint_qp;
}
inline bool state_header_matches(const EncoderConfig& c, const Geometry& g, const StateHeader& h) {
    return memcmp(h.magic, "SKH4", 4) == 0 && h.version == 3 && h.codec == c.codec && h.W == g.W && h.H == g.H &&
           h.stripe_height == c.stripe_height && h.fullframe == c.fullframe && h.num_slices == g.num_slices;
}

// ---- bitstream packaging (host) -------------------------------------------
int choose_level_idc(int mb_w, int mb_h, float fps);
// SPS + PPS NAL units (Annex-B, with start codes) for a picture of w x h pixels.
void build_parameter_sets(int width, int height, int full_range, float fps,
                          std::vector<uint8_t>& out, int num_refs = 1);
// Appends start code + NAL header + EP-escaped payload.
void append_nal(std::vector<uint8_t>& out, int nal_header_byte, const uint8_t* rbsp, size_t n);
size_t emulation_prevent(const uint8_t* in, size_t n, uint8_t* out);
// 10-byte 0x04 stripe header (selkies-core.js:2925-2938)
void write_stripe_header(uint8_t* p, int key, uint16_t frame_id, int y, int w, int h);

}  // namespace h264
}  // namespace sk
