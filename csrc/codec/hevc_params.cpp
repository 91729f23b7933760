// H.265 parameter sets (VPS 7.3.2.1, SPS 7.3.2.2, PPS 7.3.2.3) for the coding
// structure of hevc_core.h, NAL packaging and level selection (Annex A).
#include "hevc_encoder.h"
#include <string.h>

namespace sk {
namespace hevc {

int choose_level_idc(int w, int h, float fps) {
    const double ps = (double)w * h, sr = ps * (fps > 0 ? fps : 60.0);
    struct L { int idc; double ps, sr; };
    static const L levels[] = {{30, 36864, 552960},          {60, 122880, 3686400},
                               {63, 245760, 7372800},        {90, 552960, 16588800},
                               {93, 983040, 33177600},       {120, 2228224, 66846720},
                               {123, 2228224, 133693440},    {150, 8912896, 267386880},
                               {153, 8912896, 534773760},    {156, 8912896, 1069547520},
                               {180, 35651584, 1069547520},  {183, 35651584, 2139095040},
                               {186, 35651584, 4278190080.0}};
    for (const L& l : levels)
        if (ps <= l.ps && sr <= l.sr) return l.idc;
    return 186;
}

static void profile_tier_level(HBitWriter& w, int level_idc) {
    w.put(0, 2);              // general_profile_space
    w.put(0, 1);              // general_tier_flag (Main tier)
    w.put(1, 5);              // general_profile_idc: Main
    w.put(0x60000000u, 32);   // general_profile_compatibility_flag[1] (Main), [2] (Main 10)
    w.put1(1);                // general_progressive_source_flag
    w.put1(0);                // general_interlaced_source_flag
    w.put1(0);                // general_non_packed_constraint_flag
    w.put1(1);                // general_frame_only_constraint_flag
    w.put(0, 32);             // general_reserved_zero_43bits + general_inbld_flag (44 bits)
    w.put(0, 12);
    w.put((uint32_t)level_idc, 8);
}

void append_nal(std::vector<uint8_t>& out, int type, const uint8_t* rbsp, size_t n) {
    static const uint8_t sc[4] = {0, 0, 0, 1};
    out.insert(out.end(), sc, sc + 4);
    out.push_back((uint8_t)(type << 1));   // forbidden_zero_bit, nal_unit_type, nuh_layer_id high bit
    out.push_back(1);                      // nuh_layer_id low bits = 0, nuh_temporal_id_plus1 = 1
    const size_t o = out.size();
    out.resize(o + 2 * n + 4);
    const int m = ep_escape(rbsp, (int)n, out.data() + o);
    out.resize(o + (size_t)m);
}

void build_parameter_sets(int w, int h, int full_range, float fps, std::vector<uint8_t>& out) {
    const int pw = (w + 15) & ~15, ph = (h + 15) & ~15;
    const int level = choose_level_idc(pw, ph, fps);
    uint8_t buf[256];
    // ---- VPS ----
    memset(buf, 0, sizeof(buf));
    {
        HBitWriter v{buf, 0};
        v.put(0, 4);          // vps_video_parameter_set_id
        v.put1(1);            // vps_base_layer_internal_flag
        v.put1(1);            // vps_base_layer_available_flag
        v.put(0, 6);          // vps_max_layers_minus1
        v.put(0, 3);          // vps_max_sub_layers_minus1
        v.put1(1);            // vps_temporal_id_nesting_flag
        v.put(0xffff, 16);    // vps_reserved_0xffff_16bits
        profile_tier_level(v, level);
        v.put1(1);            // vps_sub_layer_ordering_info_present_flag
        v.ue(1);              // vps_max_dec_pic_buffering_minus1
        v.ue(0);              // vps_max_num_reorder_pics
        v.ue(0);              // vps_max_latency_increase_plus1
        v.put(0, 6);          // vps_max_layer_id
        v.ue(0);              // vps_num_layer_sets_minus1
        v.put1(0);            // vps_timing_info_present_flag
        v.put1(0);            // vps_extension_flag
        v.align_one();
        append_nal(out, kNalVps, buf, v.pos / 8);
    }
    // ---- SPS ----
    memset(buf, 0, sizeof(buf));
    {
        HBitWriter s{buf, 0};
        s.put(0, 4);          // sps_video_parameter_set_id
        s.put(0, 3);          // sps_max_sub_layers_minus1
        s.put1(1);            // sps_temporal_id_nesting_flag
        profile_tier_level(s, level);
        s.ue(0);              // sps_seq_parameter_set_id
        s.ue(1);              // chroma_format_idc 4:2:0
        s.ue((uint32_t)pw);   // pic_width_in_luma_samples
        s.ue((uint32_t)ph);   // pic_height_in_luma_samples
        const int cr = (pw - w) / 2, cb = (ph - h) / 2;   // conformance window in chroma units
        if (cr || cb) {
            s.put1(1);
            s.ue(0);
            s.ue((uint32_t)cr);
            s.ue(0);
            s.ue((uint32_t)cb);
        } else {
            s.put1(0);
        }
        s.ue(0);              // bit_depth_luma_minus8
        s.ue(0);              // bit_depth_chroma_minus8
        s.ue(kLog2MaxPocLsb - 4);
        s.put1(1);            // sps_sub_layer_ordering_info_present_flag
        s.ue(1);              // sps_max_dec_pic_buffering_minus1
        s.ue(0);              // sps_max_num_reorder_pics
        s.ue(0);              // sps_max_latency_increase_plus1
        s.ue(0);              // log2_min_luma_coding_block_size_minus3: 8x8 (intra CU8s)
        s.ue(2);              // log2_diff_max_min_luma_coding_block_size: CTB 32x32
        s.ue(0);              // log2_min_luma_transform_block_size_minus2: 4x4
        s.ue(3);              // log2_diff_max_min_luma_transform_block_size: 32x32
        s.ue(3);              // max_transform_hierarchy_depth_inter: CU32 -> 32, 16, 8, 4
        s.ue(2);              // max_transform_hierarchy_depth_intra (+1 under PART_NxN)
        s.put1(0);            // scaling_list_enabled_flag
        s.put1(0);            // amp_enabled_flag
        s.put1(1);            // sample_adaptive_offset_enabled_flag (hevc_sao.h)
        s.put1(0);            // pcm_enabled_flag
        s.ue(1);              // num_short_term_ref_pic_sets
        // st_ref_pic_set(0): one reference, the previous picture
        s.ue(1);              // num_negative_pics
        s.ue(0);              // num_positive_pics
        s.ue(0);              // delta_poc_s0_minus1
        s.put1(1);            // used_by_curr_pic_s0_flag
        s.put1(0);            // long_term_ref_pics_present_flag
        s.put1(0);            // sps_temporal_mvp_enabled_flag
        s.put1(0);            // strong_intra_smoothing_enabled_flag
        s.put1(1);            // vui_parameters_present_flag
        s.put1(0);            // aspect_ratio_info_present_flag
        s.put1(0);            // overscan_info_present_flag
        s.put1(1);            // video_signal_type_present_flag
        s.put(5, 3);          // video_format: unspecified
        s.put1(full_range ? 1 : 0);
        s.put1(1);            // colour_description_present_flag
        s.put(1, 8);          // colour_primaries BT.709
        s.put(1, 8);          // transfer_characteristics BT.709
        s.put(1, 8);          // matrix_coeffs BT.709
        s.put1(0);            // chroma_loc_info_present_flag
        s.put1(0);            // neutral_chroma_indication_flag
        s.put1(0);            // field_seq_flag
        s.put1(0);            // frame_field_info_present_flag
        s.put1(0);            // default_display_window_flag
        s.put1(0);            // vui_timing_info_present_flag
        s.put1(1);            // bitstream_restriction_flag
        s.put1(0);            // tiles_fixed_structure_flag
        s.put1(1);            // motion_vectors_over_pic_boundaries_flag
        s.put1(1);            // restricted_ref_pic_lists_flag
        s.ue(0);              // min_spatial_segmentation_idc
        s.ue(0);              // max_bytes_per_pic_denom
        s.ue(0);              // max_bits_per_min_cu_denom
        s.ue(15);             // log2_max_mv_length_horizontal
        s.ue(15);             // log2_max_mv_length_vertical
        s.put1(0);            // sps_extension_present_flag
        s.align_one();
        append_nal(out, kNalSps, buf, s.pos / 8);
    }
    // ---- PPS ----
    memset(buf, 0, sizeof(buf));
    {
        HBitWriter p{buf, 0};
        p.ue(0);              // pps_pic_parameter_set_id
        p.ue(0);              // pps_seq_parameter_set_id
        p.put1(0);            // dependent_slice_segments_enabled_flag
        p.put1(0);            // output_flag_present_flag
        p.put(0, 3);          // num_extra_slice_header_bits
        p.put1(0);            // sign_data_hiding_enabled_flag
        p.put1(0);            // cabac_init_present_flag
        p.ue(0);              // num_ref_idx_l0_default_active_minus1
        p.ue(0);              // num_ref_idx_l1_default_active_minus1
        p.se(0);              // init_qp_minus26
        p.put1(0);            // constrained_intra_pred_flag
        p.put1(1);            // transform_skip_enabled_flag (4x4 TUs, the encoder's RD choice)
        p.put1(0);            // cu_qp_delta_enabled_flag
        p.se(0);              // pps_cb_qp_offset
        p.se(0);              // pps_cr_qp_offset
        p.put1(0);            // pps_slice_chroma_qp_offsets_present_flag
        p.put1(0);            // weighted_pred_flag
        p.put1(0);            // weighted_bipred_flag
        p.put1(0);            // transquant_bypass_enabled_flag
        p.put1(0);            // tiles_enabled_flag
        p.put1(1);            // entropy_coding_sync_enabled_flag (WPP: one substream per CTB row)
        p.put1(0);            // pps_loop_filter_across_slices_enabled_flag
        p.put1(1);            // deblocking_filter_control_present_flag
        p.put1(0);            // deblocking_filter_override_enabled_flag
        p.put1(0);            // pps_deblocking_filter_disabled_flag: deblocking on (hevc_core.h)
        p.se(0);              // pps_beta_offset_div2
        p.se(0);              // pps_tc_offset_div2
        p.put1(0);            // pps_scaling_list_data_present_flag
        p.put1(0);            // lists_modification_present_flag
        p.ue(0);              // log2_parallel_merge_level_minus2
        p.put1(0);            // slice_segment_header_extension_present_flag
        p.put1(0);            // pps_extension_present_flag
        p.align_one();
        append_nal(out, kNalPps, buf, p.pos / 8);
    }
}

}  // namespace hevc
}  // namespace sk
