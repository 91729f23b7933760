// AV1 multi-symbol arithmetic encoder (the entropy coder of BASELINE config 5's AV1
// path; AV1 spec 8.2 "symbol decoding process" is the normative decoder side,
// mirrored independently in selkies_gstreamer_amd/models/av1/entropy.py).
//
// Status: the coder, CDF adaptation, booleans and literals are complete and
// round-trip through the independent spec-model decoder (tests/test_av1_entropy.py).
// An AV1 bitstream additionally starts every frame from the normative default CDF
// tables (thousands of values) that no file on this image holds and nothing here
// could check, so no AV1 elementary stream is produced yet (docs/components.md).
//
// CDFs are held the way the spec writes them: cdf[0..N-1] cumulative (x 32768),
// cdf[N-1] == 32768, cdf[N] = adaptation counter. The coder works on 15-bit
// probabilities with the spec's EC_PROB_SHIFT / EC_MIN_PROB interval rule; `low`
// is a 64-bit window, settled 16-bit chunks carry-propagate at finish().
#pragma once
#include <cstdint>
#include <vector>

#include "sk_common.h"

namespace sk::av1 {

constexpr int kProbShift = 6;   // EC_PROB_SHIFT
constexpr int kMinProb = 4;     // EC_MIN_PROB

// Spec update_cdf (8.2.7 / 4.10.x): adapt towards the coded symbol.
SK_HD void update_cdf(uint16_t* cdf, int n, int symbol) {
    const int cnt = cdf[n];
    const int rate = 3 + (cnt > 15) + (cnt > 31) + (n > 3 ? 2 : (n > 1 ? 1 : 0));   // Min(FloorLog2(N), 2)
    for (int i = 0; i < n - 1; i++) {
        const int target = i >= symbol ? 32768 : 0;
        if (target < cdf[i]) cdf[i] -= (uint16_t)((cdf[i] - target) >> rate);
        else cdf[i] += (uint16_t)((target - cdf[i]) >> rate);
    }
    if (cnt < 32) cdf[n] = (uint16_t)(cnt + 1);
}

// Sink: anything with SK_HD void push(uint16_t) receiving settled bytes (bit 8 =
// pending carry); finish() leaves the carry resolution to carry_bytes().
template <class Sink>
class SymbolCoder {
public:
    SK_HD explicit SymbolCoder(Sink& sink) : sink_(sink) {}

    // Codes `s` (0 <= s < n) with the cumulative CDF `cdf` (n entries + counter).
    SK_HD void encode(const uint16_t* cdf, int n, int s) {
        const uint32_t r = rng_;
        // the decoder's interval boundary for symbol k: v(k) = ((r >> 8) * (f(k) >> 6) >> 1) + 4 * (n - k - 1)
        // with f(k) = 32768 - cdf[k]; symbol s owns [v(s), v(s - 1)) (v(-1) = r) counted from the top
        const uint32_t fh = 32768u - cdf[s];
        const uint32_t v = s < n - 1 ? (((r >> 8) * (fh >> kProbShift)) >> (7 - kProbShift)) + kMinProb * (n - s - 1) : 0;
        uint32_t u = r;
        if (s > 0) {
            const uint32_t fl = 32768u - cdf[s - 1];
            u = (((r >> 8) * (fl >> kProbShift)) >> (7 - kProbShift)) + kMinProb * (n - s);
        }
        // the decoder compares against the complemented value: larger v = lower interval
        low_ += r - u;
        normalize(u - v);
    }

    SK_HD void encode_adapt(uint16_t* cdf, int n, int s) {
        encode(cdf, n, s);
        update_cdf(cdf, n, s);
    }

    // read_bool: a fixed 50 % binary symbol (spec L(1) / read_literal)
    SK_HD void bool_(int b) {
        const uint16_t half[3] = {16384, 32768, 0};
        encode(half, 2, b ? 1 : 0);
    }
    SK_HD void literal(uint32_t v, int bits) {
        for (int i = bits - 1; i >= 0; i--) bool_((v >> i) & 1);
    }

    // Spec exit process: the decoder reads the bits after the final symbol as
    // padding; emit enough of `low` that every continuation decodes identically
    // (low rounded up to a multiple of 2^14 inside [low, low + rng)).
    SK_HD void finish() {
        int c = cnt_;
        const uint64_t m = 0x3fffu;
        uint64_t e = ((low_ + m) & ~m) | (m + 1);
        int s = c + 10;
        if (s > 0) {
            uint64_t n = (1ull << (c + 16)) - 1;
            do {
                sink_.push((uint16_t)(e >> (c + 16)));
                e &= n;
                s -= 8;
                n >>= 8;
                c -= 8;
            } while (s > 0);
        }
    }

private:
    SK_HD void normalize(uint32_t rng) {
        const int d = 15 - (31 - __builtin_clz(rng));   // renormalise rng to [2^15, 2^16)
        int c = cnt_;
        int s = c + d;
        if (s >= 0) {   // a byte (or two) of low settled: keep it with its pending carry
            c += 16;
            uint64_t m = (1ull << c) - 1;
            if (s >= 8) {
                sink_.push((uint16_t)(low_ >> c));
                low_ &= m;
                c -= 8;
                m >>= 8;
            }
            sink_.push((uint16_t)(low_ >> c));
            s = c + d - 24;
            low_ &= m;
        }
        low_ <<= d;
        rng_ = rng << d;
        cnt_ = s;
    }

    Sink& sink_;
    uint64_t low_ = 0;
    uint32_t rng_ = 0x8000;
    int cnt_ = -9;
};

// Settled chunks (9 bits: byte + carry) -> bytes, carries propagated backwards.
SK_HD void carry_bytes(const uint16_t* chunks, int n, uint8_t* out) {
    uint32_t carry = 0;
    for (int i = n - 1; i >= 0; i--) {
        carry += chunks[i];
        out[i] = (uint8_t)carry;
        carry >>= 8;
    }
}

struct VectorSink {
    std::vector<uint16_t> v;
    void push(uint16_t x) { v.push_back(x); }
};

// Host convenience: the whole stream as bytes.
class SymbolEncoder {
public:
    SymbolEncoder() : coder_(sink_) {}
    void encode(const uint16_t* cdf, int n, int s) { coder_.encode(cdf, n, s); }
    void encode_adapt(uint16_t* cdf, int n, int s) { coder_.encode_adapt(cdf, n, s); }
    void bool_(int b) { coder_.bool_(b); }
    void literal(uint32_t v, int bits) { coder_.literal(v, bits); }
    std::vector<uint8_t> finish() {
        coder_.finish();
        std::vector<uint8_t> out(sink_.v.size());
        if (!out.empty()) carry_bytes(sink_.v.data(), (int)sink_.v.size(), out.data());
        return out;
    }

private:
    VectorSink sink_;
    SymbolCoder<VectorSink> coder_;
};

}  // namespace sk::av1
