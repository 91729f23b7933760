// JPEG stripe encoder session (pixelflux output_mode 0): per-stripe damage,
// paint-over at a higher quality once a stripe is static, complete JPEG image per
// stripe. Packets are [frame_id u16 BE][y u16 BE][JPEG]; the server prefixes
// 0x03 0x00 (selkies.py:2873-2874, client header selkies-core.js:2908-2923).
#pragma once
#include <stdint.h>
#include <vector>
#include "jpeg_core.h"
#include "h264_frame.h"  // EncodedPacket

namespace sk {
namespace jpeg {

struct JpegConfig {
    int width = 1920, height = 1080;
    int stripe_height = 64;   // multiple of 16 (one MCU row = 16 px)
    int quality = 40;
    int paint_quality = 90;
    int use_paint_over = 1;
    int paint_over_trigger = 15;
};

struct JpegStripeState {
    int static_frames = 0;
    int painted = 1;
    int need_send = 1;
    int key_seq = 0;   // last keyframe-request sequence applied (GPU backend)
};

// Per-stripe send decision shared by both backends: -1 skip, 0 send at
// `quality` (damaged / keyframe request), 1 send once at `paint_quality` after
// `paint_over_trigger` static frames.
// Runs on the host (CPU backend) and on the device (k_decide) alike.
SK_HD int jpeg_plan_stripe(JpegStripeState& S, bool dirty, int use_paint_over, int paint_over_trigger) {
    if (dirty || S.need_send) {
        S.static_frames = 0;
        S.painted = 0;
        S.need_send = 0;
        return 0;
    }
    S.static_frames++;
    if (use_paint_over && !S.painted && S.static_frames >= paint_over_trigger) {
        S.painted = 1;
        return 1;
    }
    return -1;
}

// Geometry + header cache shared by both backends.
struct JpegLayout {
    int W = 0, H = 0, stripe_h = 0, num_stripes = 0, mcu_w = 0;
    int stride_y = 0, stride_c = 0, plane_h = 0;
    void init(const JpegConfig& c) {
        W = c.width;
        H = c.height;
        stripe_h = c.stripe_height;
        num_stripes = (H + stripe_h - 1) / stripe_h;
        mcu_w = (W + 15) / 16;
        stride_y = mcu_w * 16;
        stride_c = mcu_w * 8;
        plane_h = num_stripes * stripe_h;
    }
    int stripe_y(int s) const { return s * stripe_h; }
    int stripe_pix_h(int s) const {
        int h = H - s * stripe_h;
        return h < stripe_h ? h : stripe_h;
    }
    int stripe_mcu_rows(int s) const { return (stripe_pix_h(s) + 15) / 16; }
};

// SOI, APP0 (JFIF), DQT, SOF0, DHT, SOS for a w x h image at the given tables.
void build_jpeg_header(int w, int h, const JpegTables& t, std::vector<uint8_t>& out);

class CpuJpegEncoder {
   public:
    explicit CpuJpegEncoder(const JpegConfig& c);
    void request_keyframe();
    void encode(const uint8_t* bgrx, int stride, uint16_t frame_id, std::vector<h264::EncodedPacket>& out);
    // Encodes one stripe's JPEG (test hook).
    void encode_stripe(const uint8_t* bgrx, int stride, int s, const JpegTables& t, std::vector<uint8_t>& out);

    JpegConfig cfg;
    JpegLayout L;
    JpegTables tab[2];  // [0] normal quality, [1] paint-over quality
    std::vector<JpegStripeState> st;
    std::vector<uint8_t> prev;  // previous frame (BGRx rows) for damage
    bool first = true;
};

// Planes of one stripe (used by the CPU path and the tests).
void jpeg_convert_stripe(const uint8_t* bgrx, int stride, const JpegLayout& L, int s, uint8_t* y,
                         uint8_t* cb, uint8_t* cr);

}  // namespace jpeg
}  // namespace sk
