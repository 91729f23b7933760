// Device-side buffers and launch interface of the HIP H.264 pipeline.
#pragma once
#include <hip/hip_runtime.h>
#include "../codec/overlay.h"
#include "../codec/h264_encoder.h"
#include "../codec/h264_frame.h"
#include "../codec/h264_deblock.h"

namespace sk {
namespace h264 {
namespace gpu {

constexpr int kMbSlotBytes = 1024;     // per-MB CAVLC bit buffer (A.3.1 caps a MB at 400 B)
constexpr int kSliceHdrMax = 64;       // SPS+PPS+stripe header prefix room per slot

struct Planes {
    uint8_t* y;
    uint8_t* u;
    uint8_t* v;
};

// Everything a kernel needs, passed by value (pointers are device memory).
struct FrameArgs {
    int W, H, mb_w, mb_h, stride_y, stride_c, num_slices, rows_per_slice, fullframe;
    int full_range, me_range, me_iters;
    const uint8_t* bgrx;   // device copy of the captured frame
    int bgrx_stride;
    int scaled;            // K2: resample the capture (src_w x src_h) to W x H inside K1
    ScaleParams scale;
    Planes src, prev, ref, rec;
    Planes ref1;           // second reference (previous-but-one picture), num_refs == 2
    uint8_t* mb_dirty;     // [num_mbs]
    int* stripe_dirty;     // [num_slices] set by k_convert_damage, consumed (and cleared) by k_plan
    StripeState* plan_state;    // [num_slices + 1] controller state (last = picture state)
    int* plan_ctl;              // [0] keyframe requests seen, [1] frames planned (0 = first frame)
    const int* key_seq_host;    // host-mapped: [0] keyframe request counter, [1] qp, [2] paint qp (0 = config)
    int* key_dev;               // [6] k_plan's device copy of the snapshot (read by k_rc_qp)
    PlanConfig plan_cfg;
    SliceTask* tasks;      // [num_slices]
    MeResult* me;          // [num_mbs]
    int16_t* mvfield;      // [num_mbs][2]
    MbInfo* mbs;           // [num_mbs]
    int16_t* coefs;        // [num_mbs][kCoefPerMb]
    uint32_t* mb_bits;     // [num_mbs][kMbSlotBytes/4]
    int* mb_nbits;         // [num_mbs]
    uint32_t* rbsp;        // [num_slices][rbsp_slot_words] (self-cleaning)
    int rbsp_slot_words;
    int* mb_off;           // [num_mbs] bit offset of each MB inside its slice RBSP
    int* slice_info;       // [num_slices * nal_per_slice][4]: RBSP bytes, packet prefix bytes
    int* tile_nz;          // [num_slices * nal_per_slice][max_tiles] last non-zero RBSP byte per EP tile
    int* tile_ins;         // [num_slices * nal_per_slice][max_tiles] emulation-prevention insertions per tile
    int max_tiles;
    int out_slot_bytes;    // bytes per slice slot in host_out
    const uint8_t* param_sets;  // [num_slices or 1][kParamSetMax]
    const int* param_set_len;
    int param_set_stride;
    uint8_t* host_out;     // host-mapped packet slots [num_slices][out_slot_bytes]
    int* host_size;        // host-mapped [num_slices] bytes in each slot
    int* frame_params_dev;           // device: [0] = frame_id (loaded by k_plan)
    const int* frame_params_host;    // host-mapped source
    SliceTask* tasks_host;           // host-mapped: final slice decisions (written by k_decide)
    unsigned long long* dbg;  // optional s_memtime stamps (SK_STAMPS=1), else nullptr
    const CavlcTables* cavlc_tabs;  // precomputed CAVLC tables (device memory), copied to LDS per WG
    int num_refs;          // EncoderConfig::num_refs (1 or 2)
    int deblock;           // K7 on: ref = deblocked rec (k_deblock), else k_commit copies rec
    int me_full;           // K4a on: MFMA exhaustive-search candidate per dirty MB
    int aq_strength;       // MB-level adaptive QP strength (Q4), 0 = off
    int subpel;            // K4c quarter-pel refinement (k_subpel) before K6
    int intra4x4;          // I slices may code I_NxN macroblocks (k_intra_prep decides, k_code_intra codes)
    const uint8_t* ov_img[kOverlaySlots];   // K12/K13 overlay images (premultiplied BGRA)
    const OverlayParams* ov;                // [kOverlaySlots] placement of this frame (device copy)
    int8_t* aq;            // [num_mbs] AQ offsets (k_aq), valid for MBs of coded slices
    DbInfo* db;            // [num_mbs] deblocking side info (k_deblock_prep)
    uint4* dbe;            // [num_mbs][3] per-MB edge record: bS nibbles, packed filter params (k_deblock_edges)
    int16_t* fs_mv;        // [num_mbs][2] MFMA full-search winner (integer pel)
    RcState* rc;           // K10 rate-control state (ratecontrol.h), device
    long long* rc_slice;   // [num_slices][2] complexity sums of P-planned slices (SAD, activity)
    float rc_fps;          // session frame rate (CBR frame budget)
    int* rc_redo;          // K10 CBR guard: device flag, 1 = code the frame again (k_rc_guard)
    // K5 sub-slices (h264_encoder.h intra_split): NAL slots per slice. slice_info / tile_nz /
    // tile_ins are indexed by NAL (slice * nal_per_slice + sub-slice); sub-slice j's RBSP
    // starts at word j * sub_rbsp_words of its slice's rbsp slot.
    int nal_per_slice;
    int sub_rbsp_words;
    const int* gate;       // second-pass launches: run only when *gate != 0 (null: always)
    // planar 4:2:0 input (YuvInput, h264_frame.h) staged on the device: W x H luma (pitch
    // W), then I420 U and V ((W+1)/2 x (H+1)/2 each) or NV12 interleaved UV (pitch
    // 2 * ((W+1)/2)); yuv_fmt 0: BGRx input through k_convert_damage
    const uint8_t* yuv;
    int yuv_fmt;
};

void launch_convert_damage(const FrameArgs& a, hipStream_t s);   // K1 + K3, or k_yuv_damage for planar input
// k_plan and everything after it; guard: CBR overflow guard + gated second coding pass
void launch_encode(const FrameArgs& a, hipStream_t s, bool guard = false);
// k_plan, motion search and scene-cut decisions only (the HEVC back end follows it)
void launch_frontend(const FrameArgs& a, hipStream_t s);
void launch_commit(const FrameArgs& a, hipStream_t s);   // MV field + reference update (+ K7 deblocking)
// K10 accounting of the frame just coded: frame bytes = sum of sizes[i * stride],
// i < n (per_slice: only slices that were coded).
void launch_rc_account(const FrameArgs& a, const int* sizes, int n, int stride, int per_slice, hipStream_t s);
// K10 per-frame cap of a back end whose payload is the sum of n byte counts (HEVC / AV1);
// chained: the check after a re-code pass (runs only when *redo is up)
void launch_rc_guard_sizes(const FrameArgs& a, const int* sizes, int n, int* redo, bool chained, hipStream_t s);

}  // namespace gpu
}  // namespace h264
}  // namespace sk
