// Host-code sanitizer harness: the CPU reference encoders
// (H.264 incl. deblocking and the stripe controller, JPEG) and the telephony
// codecs, built with -fsanitize=address,undefined by tests/test_sanitizers.py
// and driven through odd geometries, escalation QPs, keyframes and noise.
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

#include "h264_frame.h"
#include "jpeg_encoder.h"
#include "sk_api.h"

static void fill(std::vector<uint8_t>& f, int w, int h, int t, int kind) {
    uint32_t s = 12345u + 7u * (uint32_t)t;
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            uint8_t* p = &f[((size_t)y * w + x) * 4];
            if (kind == 0) {   // moving gradient + box
                const bool box = x >= (t * 5) % w && x < (t * 5) % w + w / 4 && y > h / 3 && y < h / 2;
                p[0] = box ? 240 : (uint8_t)(x + t);
                p[1] = box ? 40 : (uint8_t)(y * 2);
                p[2] = (uint8_t)(x ^ y);
            } else {           // noise
                for (int c = 0; c < 3; c++) {
                    s = s * 1664525u + 1013904223u;
                    p[c] = (uint8_t)(s >> 24);
                }
            }
            p[3] = 255;
        }
}

int main() {
    size_t bytes = 0;
    const int geoms[][3] = {{130, 70, 48}, {160, 96, 32}, {64, 64, 64}};
    for (auto& gm : geoms) {
        for (int fullframe = 0; fullframe < 2; fullframe++)
            for (int deblock = 0; deblock < 2; deblock++) {
                sk::h264::EncoderConfig c;
                c.width = gm[0];
                c.height = gm[1];
                c.stripe_height = gm[2];
                c.fullframe = fullframe;
                c.deblock = deblock;
                c.qp = fullframe ? 4 : 28;   // QP 4 on noise forces MB-level escalation
                c.paint_qp = 20;
                c.paint_over_trigger = 2;
                c.paint_over_burst = 1;
                sk::h264::CpuH264Encoder enc(c);
                std::vector<uint8_t> f((size_t)c.width * c.height * 4);
                std::vector<sk::h264::EncodedPacket> out;
                for (int t = 0; t < 6; t++) {
                    fill(f, c.width, c.height, t < 4 ? t : 3, (t + fullframe) % 3 == 2);
                    if (t == 4) enc.request_keyframe();
                    out.clear();
                    enc.encode(f.data(), c.width * 4, (uint16_t)t, out);
                    for (auto& p : out) bytes += p.data.size();
                }
            }
        sk::jpeg::JpegConfig jc;
        jc.width = gm[0];
        jc.height = gm[1];
        jc.stripe_height = 16 * ((gm[2] + 15) / 16);
        sk::jpeg::CpuJpegEncoder je(jc);
        std::vector<uint8_t> f((size_t)jc.width * jc.height * 4);
        std::vector<sk::h264::EncodedPacket> out;
        for (int t = 0; t < 4; t++) {
            fill(f, jc.width, jc.height, t, t == 3);
            out.clear();
            je.encode(f.data(), jc.width * 4, (uint16_t)t, out);
            for (auto& p : out) bytes += p.data.size();
        }
    }
    // telephony codecs
    std::vector<int16_t> pcm(3200), back(3200);
    for (int i = 0; i < 3200; i++) pcm[i] = (int16_t)((i * 977) % 65536 - 32768);
    std::vector<uint8_t> code(3200);
    for (int alaw = 0; alaw < 2; alaw++) {
        sk_g711_encode(alaw, pcm.data(), 3200, code.data());
        sk_g711_decode(alaw, code.data(), 3200, back.data());
    }
    void* e = sk_g722_create();
    void* d = sk_g722_create();
    int n = sk_g722_encode(e, pcm.data(), 3200, code.data());
    sk_g722_decode(d, code.data(), n, back.data());
    sk_g722_destroy(e);
    sk_g722_destroy(d);
    printf("sanitized run ok: %zu bytes\n", bytes);
    return 0;
}
