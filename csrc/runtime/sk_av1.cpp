// C ABI of the AV1 entropy coder (codec/av1_ec.h) for the round-trip tests against
// the independent spec-model decoder (models/av1/entropy.py).
#include <cstring>
#include <vector>

#include "../codec/av1_ec.h"
#include "sk_api.h"

extern "C" {

// Codes n symbols: symbol i uses context ctx[i] (of n_ctx contexts, each with
// nsym[c] symbols and CDF cdfs[c * 17 .. c * 17 + nsym[c]] incl. the counter),
// adapting the CDFs when `adapt`; kind[i] = 0 symbol, 1 bool (sym = 0/1),
// 2 literal of ctx[i] bits. Returns the byte count (or -needed if cap is short).
int sk_av1_ec_encode(const int32_t* kind, const int32_t* ctx, const int32_t* sym, int n, uint16_t* cdfs,
                     const int32_t* nsym, int adapt, uint8_t* out, int cap) {
    sk::av1::SymbolEncoder enc;
    for (int i = 0; i < n; i++) {
        if (kind[i] == 1) {
            enc.bool_(sym[i]);
        } else if (kind[i] == 2) {
            enc.literal((uint32_t)sym[i], ctx[i]);
        } else {
            uint16_t* cdf = cdfs + (size_t)ctx[i] * 17;
            if (adapt) enc.encode_adapt(cdf, nsym[ctx[i]], sym[i]);
            else enc.encode(cdf, nsym[ctx[i]], sym[i]);
        }
    }
    std::vector<uint8_t> b = enc.finish();
    if ((int)b.size() > cap) return -(int)b.size();
    if (!b.empty()) std::memcpy(out, b.data(), b.size());
    return (int)b.size();
}

}  // extern "C"
