// H.265 / HEVC Main encoder (session level): geometry, parameter sets and the CPU
// reference backend. The front end — BGRx -> YUV 4:2:0 conversion (K1/K2), damage
// (K3), the per-stripe controller (paint-over, keyframes), integer motion search
// (K4, MFMA exhaustive candidate on the GPU) and scene-cut decisions — is the one of
// the H.264 encoder run in full-frame mode: a stripe is an HEVC slice of whole CTB
// rows (CTB 32 = 2x2 H.264 MBs: the MB grid is the quadtree's 16x16 unit grid, units in
// z order inside a CTB). The HEVC back end decides the CTB's CU split (32 / 16 / 8),
// codes the CUs, binarises them into CABAC bins, codes one WPP substream per CTB row and
// assembles slice NAL units with entry points.
//
// Reference parity: the reference's HEVC paths are GStreamer elements (nvh265enc
// legacy/gstwebrtc_app.py:369-425, x265enc :667-683, vah265enc :510-543) with the
// H.265 RTP payloader (PT 100, :848-866); this encoder is the HIP-native equivalent.
#pragma once
#include <stdlib.h>
#include <vector>
#include "h264_frame.h"
#include "hevc_core.h"
#include "hevc_sao.h"
#include "hevc_syntax.h"

namespace sk {
namespace hevc {

// Picture geometry: CTBs (32x32) and the 16x16 unit grid of the front end (its MBs).
struct Geo {
    int ctb_w = 0, ctb_h = 0, rows_per_slice = 0, num_slices = 0;   // CTB counts, slices in CTB rows
    int W16 = 0, H16 = 0;       // units
    int pic_w = 0, pic_h = 0;   // coded picture size (multiples of 16)
    int addr_bits = 0;          // slice_segment_address length
    void init(const h264::Geometry& g) {
        W16 = g.mb_w;
        H16 = g.mb_h;
        ctb_w = (W16 + 1) >> 1;
        ctb_h = (H16 + 1) >> 1;
        rows_per_slice = g.rows_per_slice >> 1;   // stripes are whole CTB rows (hevc_geometry)
        num_slices = g.num_slices;
        pic_w = g.stride_y;
        pic_h = g.plane_h_y;
        const int n = ctb_w * ctb_h;
        addr_bits = 0;
        while ((1 << addr_bits) < n) addr_bits++;
    }
    int ctbs() const { return ctb_w * ctb_h; }
    int units() const { return W16 * H16; }
    UnitGrid grid() const { return UnitGrid{W16, H16}; }
};

// Stripes (the front end's slices) of whole CTB rows: a multiple of 32 lines.
inline void hevc_geometry(h264::EncoderConfig& f) {
    f.stripe_height = f.stripe_height < 32 ? 32 : (f.stripe_height + 31) & ~31;
}

// CBR sessions code no scene-cut intra slices (as the AV1 encoder, av1_encoder.h
// cbr_config): on a bitrate budget a slice recoded as intra costs more bits at the same
// quality and its CTB wavefront is the picture's longest serial chain. Key frames on
// request and the GOP stay. Applied by both back ends (front_config, HipBackend).
inline void cbr_config(h264::EncoderConfig& f) {
    if (f.rc_mode == h264::RC_CBR) f.scenecut = 0;
}

// Front-end configuration: full-frame stripes-as-slices, one reference, no H.264 deblock.
inline h264::EncoderConfig front_config(const h264::EncoderConfig& c) {
    h264::EncoderConfig f = c;
    f.fullframe = 1;
    f.deblock = 0;
    f.num_refs = 1;
    cbr_config(f);
    hevc_geometry(f);
    return f;
}

// Slices per CTB row of intra slices (SliceMap::K): ceil(ctb_w / kIntraSegCtbs) (CTB32s);
// above 1440p (4096 CTBs) segments of kIntraSegCtbs / 2: a key frame takes about as long
// as one segment's closed-loop chain (40 units at 4K: 816 chains, one wave per SIMD;
// 5-CTB segments measured 2.2 against 2.4 ms - the chains then share SIMDs - for +1 %
// key-frame bytes). SK_HEVC_SEG_CTBS=<n> sets the segment width (tests exercise
// the split at small sizes), SK_HEVC_SEG_CTBS=0 turns the split off (RD A/B runs).
inline int intra_seg_k(int ctb_w, int ctb_h) {
    const char* e = getenv("SK_HEVC_SEG_CTBS");
    if (e && e[0] == '0') return 1;
    const int seg = e && atoi(e) > 0 ? atoi(e) : (ctb_w * ctb_h > 4096 ? kIntraSegCtbs / 2 : kIntraSegCtbs);
    return intra_seg_count(ctb_w, seg);
}

int choose_level_idc(int w, int h, float fps);
// VPS + SPS + PPS NAL units (Annex B) for a w x h picture.
void build_parameter_sets(int w, int h, int full_range, float fps, std::vector<uint8_t>& out);
// Start code + 2-byte NAL header + emulation-prevented RBSP.
void append_nal(std::vector<uint8_t>& out, int type, const uint8_t* rbsp, size_t n);

// ---- shared CU-level helpers (CPU reference; the kernels mirror them) ----------
// Linear intra reference array (see intra_substitute) of an n x n block at (x0, y0) of
// `plane` for a transform block with the neighbour availability `avail` (AV_* bits).
void build_intra_ref_av(const uint8_t* plane, int stride, int x0, int y0, int n, int avail, uint8_t* ref);
// Prediction of an n x n block for `mode` (cidx 0 luma / 1,2 chroma) from a raw reference.
void intra_predict(const uint8_t* ref_raw, int log2n, int mode, int cidx, uint8_t* pred);

// Per-CTB scratch of the inter coding: each unit's source and prediction rasters
// (Y 16x16 | Cb 8x8 | Cr 8x8) and the RD cost of its 16x16 CU's residual tree.
struct Cu32Work {
    bool in[4];
    uint8_t src[4][kCoefPerCu], pred[4][kCoefPerCu];
    long long j[4];
};

class CpuHevcEncoder {
   public:
    explicit CpuHevcEncoder(const h264::EncoderConfig& cfg);
    void request_keyframe() { fe.request_keyframe(); }
    void set_qp(int qp, int paint_qp) { fe.set_qp(qp, paint_qp); }
    void encode(const uint8_t* bgrx, int stride, uint16_t frame_id, std::vector<h264::EncodedPacket>& out);

    // ---- stages (public for tests) ----
    void code_slice_inter(int s);
    void code_slice_intra(int s);
    void code_slice_skip(int s);
    void binarize_slice(int s);
    // SAO (hevc_sao.h) on the deblocked reconstruction: stats + own decision per CTB, then
    // the merge pass per row (sao_analyse); the filter into the reference (sao_apply)
    void sao_analyse();
    void sao_apply();
    // CABAC substreams of slice s (one per CTB row) -> slice NAL (Annex B); a split intra
    // slice -> one NAL per row segment (SliceMap)
    std::vector<uint8_t> write_slice(int s, bool idr);
    std::vector<uint8_t> write_segment(const h264::SliceTask& t, int cy0, int rows, int x0, int x1, bool idr);
    long long payload_bytes_ = 0;   // substream bytes of the frame being written (K10)
    bool pc_host_ = getenv("SK_HEVC_PCABAC") != nullptr;   // write rows with pc_code_row_host
    std::vector<uint32_t> pc_dbg_;   // pc_host_: per unit chunk bit offset, start range, tail (tests)

    h264::CpuH264Encoder fe;   // front end (full-frame mode)
    Geo geo;
    std::vector<CuInfo> cus;           // per unit
    std::vector<int16_t> coefs;        // kCoefPerCu per unit
    std::vector<uint16_t> bins;        // kCuBinCap per unit
    std::vector<int> bin_n;
    std::vector<SaoStats> sao_stats;   // 3 per CTB (Y, Cb, Cr)
    std::vector<SaoParams> sao_own, sao;   // per CTB: own decision, final (after merges)
    std::vector<long long> sao_cost;
    std::vector<long long> sao_md;     // kSaoMd per CTB: merge-candidate distortions (sao_merge_dists)
    std::vector<uint8_t> param_sets;   // VPS + SPS + PPS
    int poc = 0;                       // POC of the next picture
    int seg_k = 1;                     // intra slices: slices per CTB row (SliceMap::K)
    SliceMap smap() const { return SliceMap{fe.tasks.data(), geo.ctb_w, geo.rows_per_slice, seg_k}; }

   private:
    void load_cu_src(int cx, int cy, uint8_t* y, uint8_t* u, uint8_t* v) const;
    void put_unit_rec(int ux, int uy, const uint8_t* rec);   // a unit raster into the rec planes
    template <class MV>
    void cu32_decide(int c, int r, const Cu32Work& wk, int qp, int lam_boost, MV mv);
    void code_unit_intra(int ux, int uy, int qp);            // closed-loop intra coding of one unit
};

}  // namespace hevc
}  // namespace sk
