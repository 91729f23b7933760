// Frame-level state shared by the CPU reference backend and the HIP backend:
// plane geometry, per-MB buffers and the stage functions of the CPU path.
#pragma once
#include <vector>
#include <stdint.h>
#include "h264_encoder.h"
#include "h264_mb.h"
#include "h264_deblock.h"
#include "color.h"
#include "overlay.h"

namespace sk {
namespace h264 {

// Output of one encoded frame: packets already carry the 10-byte 0x04 header.
struct EncodedPacket {
    int y = 0, w = 0, h = 0, key = 0;
    std::vector<uint8_t> data;
};

// Motion-search result per macroblock (SAD only: ME cost = SAD + lambda*mvbits).
struct MeResult {
    int16_t mvx, mvy;        // integer-pel motion vector
    int32_t sad;             // SAD of the chosen vector
    int32_t intra_est;       // sum |Y - mean| of the source MB (scene-cut estimate)
    int16_t ref;             // reference picture index (0 = previous picture, 1 = the one before)
    int8_t fx, fy;           // quarter-pel refinement (-3..3) on top of 4 * (mvx, mvy): subpel_refine
};
// Integer matches this close (SAD per 16x16, i.e. <= 1 per pixel on average) keep their
// integer vector: a fractional one could not win back the extra MVD bits.
constexpr int kSubpelMinSad = 256;
// Adaptive refinement, per stripe (stripes stay independent streams): a stripe refines
// its P vectors when its previous frame's refinement moved >= 1/kSubpelGateDen of its MBs
// to a fractional vector, and on every kSubpelProbe-th P frame of the stripe
// (frame_num % 8 == 1, so the first P after an IDR probes). Integer-motion content
// (scrolling, dragging) then skips the pass. Counts live in StripeState.
// A "hit" is a fractional vector that beats the integer one by >= 1/8 of its SAD (true
// sub-pixel motion, not fitting the reference's coding noise).
constexpr int kSubpelProbe = 8;
constexpr int kSubpelGateDen = 32;
SK_HD bool subpel_gate(int frame_num, int prev_hits, int num_mbs) {
    return (frame_num & (kSubpelProbe - 1)) == 1 || prev_hits * kSubpelGateDen >= num_mbs;
}
SK_HD bool subpel_hit(int best_sad, int int_sad) { return best_sad * 8 <= int_sad * 7; }
// Quarter-pel motion vector of an ME result (H.264 MV units).
SK_HD int me_qx(const MeResult& r) { return 4 * r.mvx + r.fx; }
SK_HD int me_qy(const MeResult& r) { return 4 * r.mvy + r.fy; }

enum YuvFormat : int32_t { YUV_NONE = 0, YUV_I420 = 1, YUV_NV12 = 2 };
struct YuvInput {
    int32_t fmt;
    const uint8_t* p[3];
    int32_t stride[3];
};

// Sample of a planar 4:2:0 input at clamped coordinates (edge padding repeats the last
// row / column, as the BGRx path does): plane 0 luma, 1 Cb, 2 Cr.
SK_HD uint8_t yuv_sample(int fmt, const uint8_t* const* p, const int32_t* stride, int plane, int x, int y, int W,
                         int H) {
    if (plane == 0) return p[0][(size_t)sk_min(y, H - 1) * stride[0] + sk_min(x, W - 1)];
    const int cw = (W + 1) >> 1, ch = (H + 1) >> 1;
    x = sk_min(x, cw - 1);
    y = sk_min(y, ch - 1);
    if (fmt == YUV_NV12) return p[1][(size_t)y * stride[1] + 2 * x + (plane - 1)];
    return p[plane][(size_t)y * stride[plane] + x];
}

class CpuH264Encoder {
   public:
    explicit CpuH264Encoder(const EncoderConfig& cfg);
    void request_keyframe() { ctl_.request_keyframe(); }
    void set_qp(int qp, int paint_qp) { ctl_.set_qp(qp, paint_qp); }
    // Full pipeline for one captured frame.
    void encode(const uint8_t* bgrx, int stride_bytes, uint16_t frame_id,
                std::vector<EncodedPacket>& out);

    // ---- stages (public for tests) ----
    void load_frame(const uint8_t* bgrx, int stride_bytes);  // K1 + K3 (or yuv_in: K3 only)
    void load_frame_yuv();                                  // planar input: edge padding
    void detect_damage();                                   // K3 on src against prev
    void motion_search(int s);                              // K4 for slice s
    void intra_activity(int s);                             // planned intra slice: MB activity only
    int mb_activity(int mbx, int mby) const;
    void subpel_refine(int s);                              // K4c: half + quarter-pel refinement
    void decide_scenecut(int s);
    void compute_aq(int s);                                 // AQ offsets of slice s's MBs
    int mb_start_qp(const SliceTask& t, int idx) const {
        return cfg.aq_strength > 0 ? aq_start_qp(t.qp, aq[idx]) : -1;
    }
    void code_slice_inter(int s, bool redo = false);   // redo: CBR second pass, vectors kept
    void code_slice_intra(int s);
    void code_slice_skipall(int s);
    std::vector<std::vector<uint8_t>> write_slice(int s);    // entropy + header -> RBSP of each NAL
    void package(uint16_t frame_id, std::vector<std::vector<std::vector<uint8_t>>>& rbsp,
                 std::vector<EncodedPacket>& out);
    void finish_frame();

    EncoderConfig cfg;
    Geometry g;
    Controller ctl_;
    std::vector<uint8_t> src[3], prev[3], ref[3], rec[3];
    std::vector<uint8_t> ref1[3];  // second reference (previous-but-one picture) when num_refs == 2
    std::vector<uint8_t> mb_dirty, stripe_dirty;
    std::vector<MbInfo> mbs;
    std::vector<int16_t> coefs;
    std::vector<MeResult> me;
    std::vector<int16_t> mvfield;  // previous integer mv per MB (x, y)
    std::vector<DbInfo> dbinfo;    // deblocking side info of the current frame
    std::vector<int16_t> fs_mv;    // K4a full-search winner per MB (x, y), dirty MBs of P slices
    std::vector<SliceTask> tasks;
    std::vector<int8_t> aq;        // MB-level QP offsets (cfg.aq_strength > 0), compute_aq()
    std::vector<std::vector<uint8_t>> param_sets;  // per stripe (striped) or [0] (full frame)
    bool first_frame = true;
    bool scaled_ = false;          // K2: capture resampled to width x height
    ScaleParams scale_ = {};
    // Planar 4:2:0 input (GStreamer NV12 / I420 caps): the next load_frame() takes these
    // planes instead of BGRx (no colour conversion, no overlays, no resampling); fmt 0:
    // none. Planes of W x H luma and ((W + 1) / 2) x ((H + 1) / 2) chroma; I420 p[1] / p[2]
    // = U / V, NV12 p[1] = interleaved UV.
    YuvInput yuv_in = {};
    // K12/K13 overlays (watermark, cursor) blended inside load_frame
    OverlayParams overlay[kOverlaySlots] = {};
    std::vector<uint8_t> overlay_img[kOverlaySlots];
    void set_overlay_image(int slot, const uint8_t* bgra, int w, int h);
    void set_overlay_pos(int slot, int on, int x, int y, int tdx, int tdy);

   private:
    // neighbours inside the slice; sub0 >= 0: the MB's sub-slice starts at MB index sub0
    // (split I slice: no top neighbour, left only inside the sub-slice)
    void mb_neighbours(int mbx, int mby, int first_row, MbNeighbours& nb, int sub0 = -1) const;
    void mc_luma(int mbx, int mby, int mvx, int mvy, const SliceTask& t, uint8_t* pred, int refi = 0) const;
    void mc_chroma(int mbx, int mby, int mvx, int mvy, const SliceTask& t, uint8_t* pu,
                   uint8_t* pv, int refi = 0) const;
    int sad_at(int mbx, int mby, int dx, int dy, const SliceTask& t, int refi = 0) const;
    const std::vector<uint8_t>* refs(int refi) const { return refi ? ref1 : ref; }
    void full_search(int mbx, int mby, const SliceTask& t, int16_t* out) const;
};

}  // namespace h264
}  // namespace sk
