// Telephony audio codecs of the WebRTC stack: G.711 (PCMU / PCMA, ITU-T G.711)
// and G.722 at 64 kbit/s (ITU-T G.722: two-band QMF + sub-band ADPCM).
//
// Parity target: the vendored aiortc codecs of the reference
// (src/selkies/webrtc/codecs/g711.py, g722.py), which delegate to native code
// (audioop / libavcodec). These are plain host C++ — a few kbit/s of audio gain
// nothing from the GPU — exported through the C ABI in runtime/sk_api.h.
#include <stdint.h>
#include <string.h>
#include <algorithm>

#include "../runtime/sk_api.h"

namespace {

// ---------------------------------------------------------------------------
// G.711. Segment (exponent) search on the magnitude, 4-bit mantissa.
inline uint8_t ulaw_encode(int16_t pcm) {
    constexpr int kBias = 0x84, kClip = 32635;
    int mag = pcm < 0 ? -(int)pcm : (int)pcm;
    const uint8_t sign = pcm < 0 ? 0x80 : 0x00;
    mag = std::min(mag, kClip) + kBias;
    int exp = 7;
    for (int m = 0x4000; exp > 0 && !(mag & m); m >>= 1) exp--;
    const int mant = (mag >> (exp + 3)) & 0x0F;
    return (uint8_t)~(sign | (exp << 4) | mant);
}

inline int16_t ulaw_decode(uint8_t code) {
    code = (uint8_t)~code;
    const int exp = (code >> 4) & 7, mant = code & 0x0F;
    const int mag = (((mant << 3) + 0x84) << exp) - 0x84;
    return (int16_t)((code & 0x80) ? -mag : mag);
}

inline uint8_t alaw_encode(int16_t pcm) {
    int mag = pcm < 0 ? -((int)pcm + 1) : (int)pcm;   // one's complement style magnitude
    const uint8_t sign = pcm >= 0 ? 0x80 : 0x00;
    mag >>= 3;                                          // 13-bit
    uint8_t out;
    if (mag < 32) {
        out = (uint8_t)(mag >> 1);
    } else {
        int exp = 1;
        while ((mag >> (exp + 5)) > 0 && exp < 7) exp++;
        out = (uint8_t)((exp << 4) | ((mag >> exp) & 0x0F));
    }
    return (uint8_t)((out | sign) ^ 0x55);
}

inline int16_t alaw_decode(uint8_t code) {
    code ^= 0x55;
    const int exp = (code >> 4) & 7, mant = code & 0x0F;
    int mag = exp == 0 ? (mant << 4) + 8 : ((mant << 4) + 0x108) << (exp - 1);
    return (int16_t)((code & 0x80) ? mag : -mag);
}

// ---------------------------------------------------------------------------
// G.722. Tables of ITU-T G.722 (quantiser decision levels, inverse quantiser
// outputs, log-scale factor adaptation, QMF coefficients).
constexpr int kQ6[32] = {0,    35,   72,   110,  150,  190,  233,  276,  323,  370,  422,
                         473,  530,  587,  650,  714,  786,  858,  940,  1023, 1121, 1219,
                         1339, 1458, 1612, 1765, 1980, 2195, 2557, 2919, 0,    0};
constexpr int kIln[32] = {0,  63, 62, 31, 30, 29, 28, 27, 26, 25, 24, 23, 22, 21, 20, 19,
                          18, 17, 16, 15, 14, 13, 12, 11, 10, 9,  8,  7,  6,  5,  4,  0};
constexpr int kIlp[32] = {0,  61, 60, 59, 58, 57, 56, 55, 54, 53, 52, 51, 50, 49, 48, 47,
                          46, 45, 44, 43, 42, 41, 40, 39, 38, 37, 36, 35, 34, 33, 32, 0};
constexpr int kWl[8] = {-60, -30, 58, 172, 334, 538, 1198, 3042};
constexpr int kRl42[16] = {0, 7, 6, 5, 4, 3, 2, 1, 7, 6, 5, 4, 3, 2, 1, 0};
constexpr int kIlb[32] = {2048, 2093, 2139, 2186, 2233, 2282, 2332, 2383, 2435, 2489, 2543,
                          2599, 2656, 2714, 2774, 2834, 2896, 2960, 3025, 3091, 3158, 3228,
                          3298, 3371, 3444, 3520, 3597, 3676, 3756, 3838, 3922, 4008};
constexpr int kQm4[16] = {0,     -20456, -12896, -8968, -6288, -4240, -2584, -1200,
                          20456, 12896,  8968,   6288,  4240,  2584,  1200,  0};
constexpr int kQm6[64] = {-136,   -136,   -136,   -136,   -24808, -21904, -19008, -16704, -14984, -13512, -12280,
                          -11192, -10232, -9360,  -8576,  -7856,  -7192,  -6576,  -6000,  -5456,  -4944,  -4464,
                          -4008,  -3576,  -3168,  -2776,  -2400,  -2032,  -1688,  -1360,  -1040,  -728,   24808,
                          21904,  19008,  16704,  14984,  13512,  12280,  11192,  10232,  9360,   8576,   7856,
                          7192,   6576,   6000,   5456,   4944,   4464,   4008,   3576,   3168,   2776,   2400,
                          2032,   1688,   1360,   1040,   728,    432,    136,    -432,   -136};
constexpr int kQm2[4] = {-7408, -1616, 7408, 1616};
constexpr int kIhn[3] = {0, 1, 0};
constexpr int kIhp[3] = {0, 3, 2};
constexpr int kWh[3] = {0, -214, 798};
constexpr int kRh2[4] = {2, 1, 2, 1};
constexpr int kQmf[12] = {3, -11, 12, 32, -210, 951, 3876, -805, 362, -156, 53, -11};

inline int sat16(int v) { return std::min(32767, std::max(-32768, v)); }

// One sub-band's adaptive predictor (2 poles, 6 zeros) and scale factor.
struct Band {
    int s = 0, sp = 0, sz = 0;
    int r[3] = {0, 0, 0};
    int a[3] = {0, 0, 0}, ap[3] = {0, 0, 0};
    int p[3] = {0, 0, 0};
    int d[7] = {0, 0, 0, 0, 0, 0, 0};
    int b[7] = {0, 0, 0, 0, 0, 0, 0}, bp[7] = {0, 0, 0, 0, 0, 0, 0};
    int sg[7] = {0, 0, 0, 0, 0, 0, 0};
    int nb = 0, det = 0;

    // Scale factor: log-domain leak + table increment, then the linear step size.
    void adapt_scale(int inc, int nb_max, int shift_base) {
        nb = std::min(std::max(((nb * 127) >> 7) + inc, 0), nb_max);
        const int i = (nb >> 6) & 31, sh = shift_base - (nb >> 11);
        det = (sh < 0 ? kIlb[i] << -sh : kIlb[i] >> sh) << 2;
    }

    // Predictor update with the quantised difference dq (RECONS, PARREC, UPPOL2,
    // UPPOL1, UPZERO, DELAYA, FILTEP, FILTEZ, PREDIC).
    void update(int dq) {
        d[0] = dq;
        r[0] = sat16(s + dq);
        p[0] = sat16(sz + dq);
        for (int i = 0; i < 3; i++) sg[i] = p[i] >> 15;
        // second pole
        int w1 = sat16(a[1] * 4);
        int w2 = sg[0] == sg[1] ? -w1 : w1;
        w2 = std::min(w2, 32767);
        int w3 = (sg[0] == sg[2] ? 128 : -128) + (w2 >> 7) + ((a[2] * 32512) >> 15);
        ap[2] = std::min(std::max(w3, -12288), 12288);
        // first pole
        ap[1] = sat16((sg[0] == sg[1] ? 192 : -192) + ((a[1] * 32640) >> 15));
        const int lim = sat16(15360 - ap[2]);
        ap[1] = std::min(std::max(ap[1], -lim), lim);
        // zeros: sign-sign LMS
        const int step = dq == 0 ? 0 : 128;
        sg[0] = dq >> 15;
        for (int i = 1; i < 7; i++) {
            sg[i] = d[i] >> 15;
            bp[i] = sat16((sg[i] == sg[0] ? step : -step) + ((b[i] * 32640) >> 15));
        }
        for (int i = 6; i > 0; i--) {
            d[i] = d[i - 1];
            b[i] = bp[i];
        }
        for (int i = 2; i > 0; i--) {
            r[i] = r[i - 1];
            p[i] = p[i - 1];
            a[i] = ap[i];
        }
        sp = sat16(((a[1] * sat16(r[1] + r[1])) >> 15) + ((a[2] * sat16(r[2] + r[2])) >> 15));
        int z = 0;
        for (int i = 6; i > 0; i--) z += (b[i] * sat16(d[i] + d[i])) >> 15;
        sz = sat16(z);
        s = sat16(sp + sz);
    }
};

struct G722State {
    Band band[2];
    int x[24] = {};   // QMF delay line
    G722State() {
        band[0].det = 32;
        band[1].det = 8;
    }
};

int g722_encode(G722State& st, const int16_t* pcm, int n, uint8_t* out) {
    int o = 0;
    for (int j = 0; j + 1 < n; j += 2) {
        memmove(st.x, st.x + 2, 22 * sizeof(int));
        st.x[22] = pcm[j];
        st.x[23] = pcm[j + 1];
        int odd = 0, even = 0;
        for (int i = 0; i < 12; i++) {
            odd += st.x[2 * i] * kQmf[i];
            even += st.x[2 * i + 1] * kQmf[11 - i];
        }
        const int xlow = (even + odd) >> 14, xhigh = (even - odd) >> 14;

        Band& L = st.band[0];
        const int el = sat16(xlow - L.s);
        const int wl = el >= 0 ? el : -(el + 1);
        int i = 1;
        while (i < 30 && wl >= ((kQ6[i] * L.det) >> 12)) i++;
        const int ilow = el < 0 ? kIln[i] : kIlp[i];
        const int ril = ilow >> 2;
        const int dlow = (L.det * kQm4[ril]) >> 15;
        L.adapt_scale(kWl[kRl42[ril]], 18432, 8);
        L.update(dlow);

        Band& Hb = st.band[1];
        const int eh = sat16(xhigh - Hb.s);
        const int wh = eh >= 0 ? eh : -(eh + 1);
        const int mih = wh >= ((564 * Hb.det) >> 12) ? 2 : 1;
        const int ihigh = eh < 0 ? kIhn[mih] : kIhp[mih];
        const int dhigh = (Hb.det * kQm2[ihigh]) >> 15;
        Hb.adapt_scale(kWh[kRh2[ihigh]], 22528, 10);
        Hb.update(dhigh);

        out[o++] = (uint8_t)((ihigh << 6) | ilow);
    }
    return o;
}

int g722_decode(G722State& st, const uint8_t* in, int n, int16_t* pcm) {
    int o = 0;
    for (int j = 0; j < n; j++) {
        const int code = in[j];
        const int ilow = code & 0x3F, ihigh = (code >> 6) & 3;

        Band& L = st.band[0];
        const int ril = ilow >> 2;
        const int rlow = std::min(std::max(L.s + ((L.det * kQm6[ilow]) >> 15), -16384), 16383);
        const int dlow = (L.det * kQm4[ril]) >> 15;
        L.adapt_scale(kWl[kRl42[ril]], 18432, 8);
        L.update(dlow);

        Band& Hb = st.band[1];
        const int dhigh = (Hb.det * kQm2[ihigh]) >> 15;
        const int rhigh = std::min(std::max(dhigh + Hb.s, -16384), 16383);
        Hb.adapt_scale(kWh[kRh2[ihigh]], 22528, 10);
        Hb.update(dhigh);

        memmove(st.x, st.x + 2, 22 * sizeof(int));
        st.x[22] = rlow + rhigh;
        st.x[23] = rlow - rhigh;
        // the receive QMF interleaves the odd-tap sum first, then the even-tap sum
        int odd = 0, even = 0;
        for (int i = 0; i < 12; i++) {
            even += st.x[2 * i] * kQmf[i];
            odd += st.x[2 * i + 1] * kQmf[11 - i];
        }
        pcm[o++] = (int16_t)sat16(odd >> 11);
        pcm[o++] = (int16_t)sat16(even >> 11);
    }
    return o;
}

}  // namespace

extern "C" {

int sk_g711_encode(int alaw, const int16_t* pcm, int n, uint8_t* out) {
    for (int i = 0; i < n; i++) out[i] = alaw ? alaw_encode(pcm[i]) : ulaw_encode(pcm[i]);
    return n;
}

int sk_g711_decode(int alaw, const uint8_t* in, int n, int16_t* pcm) {
    for (int i = 0; i < n; i++) pcm[i] = alaw ? alaw_decode(in[i]) : ulaw_decode(in[i]);
    return n;
}

void* sk_g722_create(void) { return new G722State(); }
void sk_g722_destroy(void* h) { delete static_cast<G722State*>(h); }

// 16 kHz PCM (n even) -> n / 2 bytes
int sk_g722_encode(void* h, const int16_t* pcm, int n, uint8_t* out) {
    return g722_encode(*static_cast<G722State*>(h), pcm, n, out);
}

// n bytes -> 2n samples of 16 kHz PCM
int sk_g722_decode(void* h, const uint8_t* in, int n, int16_t* pcm) {
    return g722_decode(*static_cast<G722State*>(h), in, n, pcm);
}

}  // extern "C"
