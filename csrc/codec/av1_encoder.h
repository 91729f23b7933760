// AV1 encoder (session level): sequence / frame headers, OBU assembly and the CPU
// reference backend. The front end — BGRx -> YUV 4:2:0 conversion (K1/K2), damage
// (K3), the stripe controller and integer motion search (K4) — is the H.264
// encoder's, run in full-frame mode like the HEVC encoder's. The AV1 back end makes
// the block decisions (intra modes on key frames, motion-compensated skip /
// residual blocks on inter frames, static 32x32 / 64x64 merging), reconstructs,
// and codes one arithmetic-coded tile per tile rectangle (tiles are the parallel
// axis of entropy coding: independent CDF state and coder per tile).
//
// Reference parity: the reference's AV1 paths are GStreamer elements (nvav1enc
// legacy/gstwebrtc_app.py:426-474, vaav1enc :576-607, svtav1enc / av1enc / rav1enc
// :724-783) with the AV1 RTP payloader (PT 96, :848-938); this is the HIP-native
// equivalent (kernels/av1_kernels.hip).
#pragma once
#include <stdlib.h>
#include <vector>
#include "av1_core.h"
#include "h264_frame.h"

namespace sk {
namespace av1 {

// Units: 16x16 blocks (the front end's macroblocks), 384 levels each: luma 256,
// U 64, V 64; an edge unit split into 8x8 blocks keeps 4 x (64 + 16 + 16).
constexpr int kLevPerUnit = 384;

struct FrameParams {
    int key = 0;
    int qidx = 86;
    int tile_size_bytes = 4;
    int lf_level = 0;     // loop_filter_level[0..3] (one level, av1_lf.h lf_level_for)
    int screen = 0;       // allow_screen_content_tools: palette blocks (key frames)
};

// Palette coding of key frames (av1_core.h): on unless SK_AV1_PALETTE=0 (A/B runs).
inline bool palette_enabled() {
    const char* e = getenv("SK_AV1_PALETTE");
    return !(e && e[0] == '0');
}

// MSB-first bit writer for headers.
struct BitWriter {
    std::vector<uint8_t> buf;
    int bits = 0;
    void put(uint32_t v, int n) {
        for (int i = n - 1; i >= 0; i--) {
            if ((bits & 7) == 0) buf.push_back(0);
            if ((v >> i) & 1) buf.back() |= (uint8_t)(0x80 >> (bits & 7));
            bits++;
        }
    }
    void align() {
        while (bits & 7) put(0, 1);
    }
    void trailing() {   // trailing_bits(): a one, then zeros to the byte boundary
        put(1, 1);
        align();
    }
};
void put_leb128(std::vector<uint8_t>& out, uint64_t v);
void write_sequence_header(BitWriter& w, int W, int H, int level_idx, int full_range);
void write_frame_header(BitWriter& w, const Av1Geo& g, const FrameParams& fp);
// OBU = header byte (type, has_size_field) + leb128 size + payload
void append_obu(std::vector<uint8_t>& out, int type, const uint8_t* payload, size_t n);
int choose_level_idx(int W, int H, float fps);
int qidx_for_qp(int qp);
// Open-loop intra mode of an n x n luma block (source edges, decoder availability).
int intra_mode_decision(const uint8_t* src, int stride, int x, int y, int log2n, bool au, bool al, int max_x,
                        int max_y);

// Rate control as svtav1enc runs in the reference (legacy/gstwebrtc_app.py:733-739):
// rc=2 (CBR) with buf-optimal-sz=120 ms, intra-period -1 and no scene-change key frames
// (a cut is coded as an inter frame: a key frame costs several budgets and starves the
// frames after it). Set whatever the starting mode, since set_rate() can switch a
// session to CBR later. Applied by both back ends (front_config here, the HIP back
// end's constructor).
inline void cbr_config(h264::EncoderConfig& f) {
    if (f.vbv_ms <= 0) f.vbv_ms = 120;
    f.scenecut = 0;
}

inline h264::EncoderConfig front_config(const h264::EncoderConfig& c) {
    h264::EncoderConfig f = c;
    f.fullframe = 1;
    f.deblock = 0;
    f.num_refs = 1;
    f.subpel = 0;
    f.use_paint_over = 0;   // a paint-over would force key frames; static regions stay at the session QP
    cbr_config(f);
    return f;
}

class CpuAv1Encoder {
   public:
    explicit CpuAv1Encoder(const h264::EncoderConfig& cfg, int tile_cols_log2 = -1, int tile_rows_log2 = -1);
    void request_keyframe() { fe.request_keyframe(); }
    void set_qp(int qp, int paint_qp) { fe.set_qp(qp, paint_qp); }
    void encode(const uint8_t* bgrx, int stride, uint16_t frame_id, std::vector<h264::EncodedPacket>& out);

    // ---- stages (public for tests / the GPU back end's parity checks) ----
    void decide_key();                        // intra decisions + reconstruction, every tile
    void decide_inter();                      // motion-compensated units + static merging
    void decide_modes();                      // inter modes from the MV stacks (pass A)
    std::vector<uint8_t> code_tile(int t);    // arithmetic-coded tile payload
    std::vector<uint8_t> assemble(const std::vector<std::vector<uint8_t>>& tiles);

    h264::CpuH264Encoder fe;
    Av1Geo geo;
    FrameParams fp;
    std::vector<BlkInfo> blk;        // c8 * r8
    std::vector<int16_t> lev;        // kLevPerUnit per 16x16 unit (front-end MB grid)
    std::vector<uint8_t> lctx[3];    // level contexts (cul | dc << 6) at 4x4 granularity per plane
    std::vector<uint8_t> pal;        // c8 * r8 * 8: palette colours of each cell's block
    bool palette_on = palette_enabled();
    int lctx_w[3] = {0, 0, 0}, lctx_h[3] = {0, 0, 0};
    int level_idx = 8;
    uint64_t frames = 0;
    // levels of the block at mi (r, c) of size bsl, plane 0..2 (raster [row][col])
    int16_t* unit_lev(int r, int c, int bsl, int plane) const;
    FrameView view() const;

   private:
    void intra_block(int r, int c, int bsl, const TileRect& t);
    void inter_unit(int ux, int uy, int mv_row, int mv_col);
    void inter_block(int r, int c, int bsl, int mv_row, int mv_col);
    void key_partition(int r, int c, int bsl, const TileRect& t, bool decide);
    void set_cells(int r, int c, int bsl, const BlkInfo& b);
    void set_lctx(int plane, int x4, int y4, int n4, uint8_t v);
    void set_palette(int r, int c, int bsl, const uint8_t* col);
};

}  // namespace av1
}  // namespace sk
