// CPU reference JPEG stripe encoder (use_cpu path and golden model of the HIP
// kernels in csrc/kernels/jpeg_kernels.hip).
#include "jpeg_encoder.h"
#include "h264_core.h"  // BitWriter
#include <string.h>
#include <algorithm>

namespace sk {
namespace jpeg {

static void put16(std::vector<uint8_t>& o, int v) {
    o.push_back((uint8_t)(v >> 8));
    o.push_back((uint8_t)v);
}

void build_jpeg_header(int w, int h, const JpegTables& t, std::vector<uint8_t>& o) {
    o.push_back(0xFF); o.push_back(0xD8);                    // SOI
    o.push_back(0xFF); o.push_back(0xE0); put16(o, 16);      // APP0 JFIF
    const uint8_t jfif[] = {'J', 'F', 'I', 'F', 0, 1, 1, 0, 0, 1, 0, 1, 0, 0};
    o.insert(o.end(), jfif, jfif + sizeof(jfif));
    o.push_back(0xFF); o.push_back(0xDB); put16(o, 2 + 2 * 65);  // DQT
    for (int c = 0; c < 2; c++) {
        o.push_back((uint8_t)c);
        for (int k = 0; k < 64; k++) o.push_back((uint8_t)t.q[c][JPEG_ZIGZAG[k]]);
    }
    o.push_back(0xFF); o.push_back(0xC0); put16(o, 17);      // SOF0
    o.push_back(8); put16(o, h); put16(o, w); o.push_back(3);
    o.push_back(1); o.push_back(0x22); o.push_back(0);
    o.push_back(2); o.push_back(0x11); o.push_back(1);
    o.push_back(3); o.push_back(0x11); o.push_back(1);
    struct H { int cls_id; const uint8_t* bits; const uint8_t* vals; int n; } hs[4] = {
        {0x00, JPEG_DC_LUMA_BITS, JPEG_DC_VALS, 12}, {0x10, JPEG_AC_LUMA_BITS, JPEG_AC_LUMA_VALS, 162},
        {0x01, JPEG_DC_CHROMA_BITS, JPEG_DC_VALS, 12}, {0x11, JPEG_AC_CHROMA_BITS, JPEG_AC_CHROMA_VALS, 162}};
    int len = 2;
    for (auto& x : hs) len += 17 + x.n;
    o.push_back(0xFF); o.push_back(0xC4); put16(o, len);     // DHT
    for (auto& x : hs) {
        o.push_back((uint8_t)x.cls_id);
        o.insert(o.end(), x.bits, x.bits + 16);
        o.insert(o.end(), x.vals, x.vals + x.n);
    }
    o.push_back(0xFF); o.push_back(0xDA); put16(o, 12);      // SOS
    o.push_back(3);
    o.push_back(1); o.push_back(0x00);
    o.push_back(2); o.push_back(0x11);
    o.push_back(3); o.push_back(0x11);
    o.push_back(0); o.push_back(63); o.push_back(0);
}

void jpeg_convert_stripe(const uint8_t* bgrx, int stride, const JpegLayout& L, int s, uint8_t* Y,
                         uint8_t* Cb, uint8_t* Cr) {
    const int y0 = L.stripe_y(s), rows = L.stripe_mcu_rows(s) * 16;
    for (int qy = 0; qy < rows / 2; qy++)
        for (int qx = 0; qx < L.stride_c; qx++) {
            int rs = 0, gs = 0, bs = 0;
            for (int j = 0; j < 2; j++)
                for (int i = 0; i < 2; i++) {
                    int py = std::min(y0 + 2 * qy + j, L.H - 1), px = std::min(2 * qx + i, L.W - 1);
                    const uint8_t* p = bgrx + (size_t)py * stride + 4 * px;
                    int yy, cb, cr;
                    rgb_to_ycc(p[2], p[1], p[0], &yy, &cb, &cr);
                    Y[(size_t)(2 * qy + j) * L.stride_y + 2 * qx + i] = (uint8_t)sk_clip255(yy);
                    rs += p[2]; gs += p[1]; bs += p[0];
                }
            int yy, cb, cr;
            rgb_to_ycc((rs + 2) >> 2, (gs + 2) >> 2, (bs + 2) >> 2, &yy, &cb, &cr);
            Cb[(size_t)qy * L.stride_c + qx] = (uint8_t)sk_clip255(cb);
            Cr[(size_t)qy * L.stride_c + qx] = (uint8_t)sk_clip255(cr);
        }
}

CpuJpegEncoder::CpuJpegEncoder(const JpegConfig& c) : cfg(c) {
    L.init(cfg);
    build_tables(cfg.quality, tab[0]);
    build_tables(cfg.paint_quality, tab[1]);
    st.assign(L.num_stripes, JpegStripeState());
    prev.assign((size_t)L.W * L.H * 4, 0);
}

void CpuJpegEncoder::request_keyframe() {
    for (auto& s : st) s.need_send = 1;
}

void CpuJpegEncoder::encode_stripe(const uint8_t* bgrx, int stride, int s, const JpegTables& t,
                                   std::vector<uint8_t>& out) {
    const int mrows = L.stripe_mcu_rows(s);
    std::vector<uint8_t> Y((size_t)L.stride_y * mrows * 16), Cb((size_t)L.stride_c * mrows * 8),
        Cr((size_t)L.stride_c * mrows * 8);
    jpeg_convert_stripe(bgrx, stride, L, s, Y.data(), Cb.data(), Cr.data());
    build_jpeg_header(L.W, L.stripe_pix_h(s), t, out);
    std::vector<uint8_t> bits((size_t)L.mcu_w * mrows * 6 * 256 + 16, 0);
    h264::BitWriter w(bits.data());
    int pred[3] = {0, 0, 0};
    int16_t zz[64];
    for (int my = 0; my < mrows; my++)
        for (int mx = 0; mx < L.mcu_w; mx++) {
            for (int b = 0; b < 6; b++) {
                const uint8_t* px;
                int strd, comp = b < 4 ? 0 : b - 3;
                if (b < 4) {
                    px = &Y[(size_t)(my * 16 + (b >> 1) * 8) * L.stride_y + mx * 16 + (b & 1) * 8];
                    strd = L.stride_y;
                } else {
                    const std::vector<uint8_t>& P = b == 4 ? Cb : Cr;
                    px = &P[(size_t)(my * 8) * L.stride_c + mx * 8];
                    strd = L.stride_c;
                }
                fdct_quant(px, strd, t.q[comp ? 1 : 0], zz);
                int diff = zz[0] - pred[comp];
                pred[comp] = zz[0];
                huff_block(w, zz, diff, t, comp ? 1 : 0);
            }
        }
    while (w.pos & 7) w.put1(1);  // pad with 1-bits
    size_t n = w.pos / 8;
    for (size_t i = 0; i < n; i++) {  // byte stuffing
        out.push_back(bits[i]);
        if (bits[i] == 0xFF) out.push_back(0x00);
    }
    out.push_back(0xFF);
    out.push_back(0xD9);  // EOI
}

void CpuJpegEncoder::encode(const uint8_t* bgrx, int stride, uint16_t frame_id,
                            std::vector<h264::EncodedPacket>& out) {
    for (int s = 0; s < L.num_stripes; s++) {
        int y0 = L.stripe_y(s), h = L.stripe_pix_h(s);
        bool dirty = first;
        for (int y = y0; y < y0 + h && !dirty; y++)
            dirty = memcmp(bgrx + (size_t)y * stride, &prev[(size_t)y * L.W * 4], (size_t)L.W * 4) != 0;
        const int which = jpeg_plan_stripe(st[s], dirty, cfg.use_paint_over, cfg.paint_over_trigger);
        if (which < 0) continue;
        h264::EncodedPacket pk;
        pk.y = y0;
        pk.w = L.W;
        pk.h = h;
        pk.key = 1;
        pk.data = {(uint8_t)(frame_id >> 8), (uint8_t)frame_id, (uint8_t)(y0 >> 8), (uint8_t)y0};
        encode_stripe(bgrx, stride, s, tab[which], pk.data);
        out.push_back(std::move(pk));
    }
    for (int y = 0; y < L.H; y++) memcpy(&prev[(size_t)y * L.W * 4], bgrx + (size_t)y * stride, (size_t)L.W * 4);
    first = false;
}

}  // namespace jpeg
}  // namespace sk
