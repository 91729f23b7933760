// Stripe controller (damage, paint-over, keyframes) and host-side bitstream
// packaging: SPS/PPS, NAL wrapping with emulation prevention, stripe headers.
//
// Paint-over / damage semantics follow the pixelflux knobs the reference passes
// (selkies.py:2946-2951: paint_over_trigger_frames=15, damage_block_threshold=10,
// damage_block_duration=20; settings.py:53-56). pixelflux itself is not in the
// reference tree, so the exact policy is our definition:
//  * a stripe with no damage for `paint_over_trigger` frames after a change is
//    re-encoded for `paint_over_burst` frames at the paint-over QP;
//  * a stripe damaged for `damage_threshold` consecutive frames is "hot" and is
//    encoded every frame for the next `damage_duration` frames.
#include "h264_encoder.h"
#include "h264_frame.h"
#include "h264_syntax.h"
#include <string.h>

namespace sk {
namespace h264 {

static_assert(kFrameNumMask == (1 << kLog2MaxFrameNum) - 1, "frame_num wrap");

void Controller::init(const EncoderConfig& cfg, const Geometry& g) {
    cfg_ = cfg;
    g_ = g;
    st_.assign(g.num_slices, StripeState());
    pic_ = StripeState();
    rc_init(rc_, cfg.rc_mode, cfg.qp, cfg.bitrate_kbps, cfg.fps, cfg.width * cfg.height, cfg.vbv_ms, cfg.codec);
}

void Controller::rate_control(SliceTask* tasks, const MeResult* me) {
    const int ns = g_.num_slices;
    std::vector<long long> sad(ns, 0), dev(ns, 0);
    for (int s = 0; s < ns; s++) {
        if (tasks[s].action != ACT_P && tasks[s].action != ACT_I) continue;   // planned I: activity only
        for (int j = tasks[s].first_row * g_.mb_w; j < (tasks[s].first_row + tasks[s].num_rows) * g_.mb_w; j++) {
            sad[s] += me[j].sad;
            dev[s] += me[j].intra_est;
        }
    }
    rc_apply(rc_, tasks, sad.data(), dev.data(), ns, g_.mb_w, cfg_.qp);
}

void Controller::request_keyframe() {
    for (auto& s : st_) s.need_idr = true;
    pic_.need_idr = true;
}

void Controller::plan(const uint8_t* dirty, SliceTask* tasks) {
    PlanConfig pc = plan_config(cfg_);
    if (rc_.mode == RC_CBR) pc.use_paint_over = 0;   // K10 CBR: no paint-over refresh (as k_plan)
    for (int s = 0; s < g_.num_slices; s++)
        plan_stripe(pc, st_[s], pic_, dirty[s] != 0, g_.slice_first_row(s), g_.slice_rows(s), g_.mb_h, tasks[s]);
}

bool Controller::picture_is_idr(const SliceTask* tasks) const {
    for (int s = 0; s < g_.num_slices; s++)
        if (!(tasks[s].final_action == ACT_I && tasks[s].idr_on_intra)) return false;
    return g_.num_slices > 0;
}

void Controller::commit(const SliceTask* tasks) {
    if (cfg_.fullframe) {
        commit_picture(pic_, picture_is_idr(tasks), plan_config(cfg_).num_refs);
        return;
    }
    for (int s = 0; s < g_.num_slices; s++) commit_stripe(st_[s], tasks[s].final_action, plan_config(cfg_).num_refs);
}

// ---------------------------------------------------------------------------
int choose_level_idc(int mb_w, int mb_h, float fps) {
    struct L { int idc, max_fs, max_mbps; };
    static const L levels[] = {{10, 99, 1485},       {11, 396, 3000},     {12, 396, 6000},
                               {13, 396, 11880},     {20, 396, 11880},    {21, 792, 19800},
                               {22, 1620, 20250},    {30, 1620, 40500},   {31, 3600, 108000},
                               {32, 5120, 216000},   {40, 8192, 245760},  {42, 8704, 522240},
                               {50, 22080, 589824},  {51, 36864, 983040}, {52, 36864, 2073600}};
    int fs = mb_w * mb_h;
    long mbps = (long)(fs * (fps > 0 ? fps : 60.f));
    int dim = mb_w > mb_h ? mb_w : mb_h;
    for (const L& l : levels) {
        int maxdim = 1;
        while ((maxdim + 1) * (maxdim + 1) <= 8 * l.max_fs) maxdim++;
        if (fs <= l.max_fs && mbps <= l.max_mbps && dim <= maxdim) return l.idc;
    }
    return 52;
}

size_t emulation_prevent(const uint8_t* in, size_t n, uint8_t* out) {
    size_t o = 0;
    int zeros = 0;
    for (size_t i = 0; i < n; i++) {
        uint8_t b = in[i];
        if (zeros >= 2 && b <= 3) {
            out[o++] = 3;
            zeros = 0;
        }
        out[o++] = b;
        zeros = b == 0 ? zeros + 1 : 0;
    }
    return o;
}

void append_nal(std::vector<uint8_t>& out, int hdr, const uint8_t* rbsp, size_t n) {
    size_t base = out.size();
    out.resize(base + 5 + n + n / 2 + 4);
    uint8_t* p = out.data() + base;
    p[0] = 0; p[1] = 0; p[2] = 0; p[3] = 1; p[4] = (uint8_t)hdr;
    size_t m = emulation_prevent(rbsp, n, p + 5);
    out.resize(base + 5 + m);
}

static void rbsp_trailing(BitWriter& w) {
    w.put1(1);
    while (w.pos & 7) w.put1(0);
}

void build_parameter_sets(int width, int height, int full_range, float fps,
                          std::vector<uint8_t>& out, int num_refs) {
    int mb_w = (width + 15) / 16, mb_h = (height + 15) / 16;
    uint8_t buf[128];
    memset(buf, 0, sizeof(buf));
    BitWriter w(buf);
    w.put(66, 8);          // profile_idc: Baseline
    w.put(0xC0, 8);        // constraint_set0/1 = 1 (Constrained Baseline), reserved 0
    w.put((uint32_t)choose_level_idc(mb_w, mb_h, fps), 8);
    put_ue(w, 0);          // seq_parameter_set_id
    put_ue(w, kLog2MaxFrameNum - 4);
    put_ue(w, 2);          // pic_order_cnt_type
    put_ue(w, (uint32_t)(num_refs > 1 ? 2 : 1));   // max_num_ref_frames (sliding window)
    w.put(0, 1);           // gaps_in_frame_num_value_allowed_flag
    put_ue(w, (uint32_t)(mb_w - 1));
    put_ue(w, (uint32_t)(mb_h - 1));
    w.put(1, 1);           // frame_mbs_only_flag
    w.put(1, 1);           // direct_8x8_inference_flag
    int crop_r = (mb_w * 16 - width) / 2, crop_b = (mb_h * 16 - height) / 2;
    if (crop_r || crop_b) {
        w.put(1, 1);
        put_ue(w, 0);
        put_ue(w, (uint32_t)crop_r);
        put_ue(w, 0);
        put_ue(w, (uint32_t)crop_b);
    } else {
        w.put(0, 1);
    }
    w.put(1, 1);           // vui_parameters_present_flag
    w.put(0, 1);           // aspect_ratio_info_present_flag
    w.put(0, 1);           // overscan_info_present_flag
    w.put(1, 1);           // video_signal_type_present_flag
    w.put(5, 3);           // video_format: unspecified
    w.put(full_range ? 1 : 0, 1);
    w.put(1, 1);           // colour_description_present_flag
    w.put(1, 8);           // colour_primaries BT.709
    w.put(1, 8);           // transfer_characteristics BT.709
    w.put(1, 8);           // matrix_coefficients BT.709
    w.put(0, 1);           // chroma_loc_info_present_flag
    w.put(0, 1);           // timing_info_present_flag
    w.put(0, 1);           // nal_hrd_parameters_present_flag
    w.put(0, 1);           // vcl_hrd_parameters_present_flag
    w.put(0, 1);           // pic_struct_present_flag
    w.put(1, 1);           // bitstream_restriction_flag
    w.put(1, 1);           // motion_vectors_over_pic_boundaries_flag
    put_ue(w, 0);          // max_bytes_per_pic_denom
    put_ue(w, 0);          // max_bits_per_mb_denom
    put_ue(w, 11);         // log2_max_mv_length_horizontal
    put_ue(w, 11);         // log2_max_mv_length_vertical
    put_ue(w, 0);          // max_num_reorder_frames
    put_ue(w, 1);          // max_dec_frame_buffering
    rbsp_trailing(w);
    append_nal(out, 0x67, buf, w.pos / 8);

    memset(buf, 0, sizeof(buf));
    BitWriter p(buf);
    put_ue(p, 0);          // pic_parameter_set_id
    put_ue(p, 0);          // seq_parameter_set_id
    p.put(0, 1);           // entropy_coding_mode_flag: CAVLC
    p.put(0, 1);           // bottom_field_pic_order_in_frame_present_flag
    put_ue(p, 0);          // num_slice_groups_minus1
    put_ue(p, 0);          // num_ref_idx_l0_default_active_minus1
    put_ue(p, 0);          // num_ref_idx_l1_default_active_minus1
    p.put(0, 1);           // weighted_pred_flag
    p.put(0, 2);           // weighted_bipred_idc
    put_se(p, 0);          // pic_init_qp_minus26
    put_se(p, 0);          // pic_init_qs_minus26
    put_se(p, 0);          // chroma_qp_index_offset
    p.put(1, 1);           // deblocking_filter_control_present_flag
    p.put(0, 1);           // constrained_intra_pred_flag
    p.put(0, 1);           // redundant_pic_cnt_present_flag
    rbsp_trailing(p);
    append_nal(out, 0x68, buf, p.pos / 8);
}

void write_stripe_header(uint8_t* p, int key, uint16_t frame_id, int y, int w, int h) {
    p[0] = 0x04;
    p[1] = key ? 1 : 0;
    p[2] = (uint8_t)(frame_id >> 8);
    p[3] = (uint8_t)frame_id;
    p[4] = (uint8_t)(y >> 8);
    p[5] = (uint8_t)y;
    p[6] = (uint8_t)(w >> 8);
    p[7] = (uint8_t)w;
    p[8] = (uint8_t)(h >> 8);
    p[9] = (uint8_t)h;
}

}  // namespace h264
}  // namespace sk
