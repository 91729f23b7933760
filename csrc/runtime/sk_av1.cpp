// C ABI of the AV1 entropy coder (codec/av1_ec.h) for the round-trip tests against
// the independent spec-model decoder (models/av1/entropy.py).
#include <cstring>
#include <vector>

#include "../codec/av1_core.h"
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

// Adaptive CDF arrays of the default context for token-stream tests: field i ->
// (offset of its first CDF in u16 units, symbols N, number of CDFs, CDF stride in
// u16). Returns the number of fields when i is out of range.
int sk_av1_cdf_field(int i, int32_t* off, int32_t* nsym, int32_t* count, int32_t* stride) {
    using sk::av1::CdfContext;
    const CdfContext& c = sk::av1::AV1_DEFAULT_CDF[0];
    struct F { const uint16_t* p; int n, stride; size_t bytes; };
#define SK_FIELD(f, n, st) F{(const uint16_t*)&c.f, n, st, sizeof(c.f)}
    const F fs[] = {SK_FIELD(kf_y_mode, 13, 14),    SK_FIELD(uv_mode_cfl_allowed, 14, 15), SK_FIELD(partition_w16, 10, 11),
                    SK_FIELD(partition_w8, 4, 11),  SK_FIELD(eob_pt_16, 5, 6),             SK_FIELD(eob_pt_1024, 11, 12),
                    SK_FIELD(coeff_base, 4, 5),     SK_FIELD(coeff_br, 4, 5),              SK_FIELD(coeff_base_eob, 3, 4),
                    SK_FIELD(txb_skip, 2, 3),       SK_FIELD(skip, 2, 3),                  SK_FIELD(mv_joint, 4, 5)};
#undef SK_FIELD
    const int nf = (int)(sizeof(fs) / sizeof(fs[0]));
    if (i < 0 || i >= nf) return nf;
    *off = (int32_t)(fs[i].p - (const uint16_t*)&c);
    *nsym = fs[i].n;
    *stride = fs[i].stride;
    *count = (int32_t)(fs[i].bytes / (2 * fs[i].stride));
    return nf;
}

// Host replay of a token stream (av1_core.h token format) through SymbolCoder with
// the default CDFs of qidx: the reference for the GPU coder k_av1_ec.
int sk_av1_ec_tokens_cpu(const uint32_t* tok, int n, int qidx, uint8_t* out, int cap) {
    sk::av1::CdfContext cx = sk::av1::AV1_DEFAULT_CDF[sk::av1::coef_qctx(qidx)];
    sk::av1::VectorSink sink;
    sk::av1::SymbolCoder<sk::av1::VectorSink> coder(sink);
    for (int i = 0; i < n; i++) sk::av1::code_token(coder, (uint16_t*)&cx, tok[i]);
    coder.finish();
    const int m = (int)sink.v.size();
    if (m > cap) return -m;
    if (m) sk::av1::carry_bytes(sink.v.data(), m, out);
    return m;
}

// Interval words of k_av1_cdf (av1_kernels.hip) for a token stream, on the host:
// words[i] for symbol and gathered tokens, the token itself for literals.
int sk_av1_cdf_words_cpu(const uint32_t* tok, int n, int qidx, uint32_t* words) {
    using namespace sk::av1;
    CdfContext cx = AV1_DEFAULT_CDF[coef_qctx(qidx)];
    uint16_t* cdfs = (uint16_t*)&cx;
    auto word = [](uint32_t clo, uint32_t chi, int nn, int s) {
        const uint32_t fh = s < nn - 1 ? (32768u - chi) >> kProbShift : 0u;
        const uint32_t fl = s > 0 ? (32768u - clo) >> kProbShift : 0u;
        return fh | fl << 10 | (uint32_t)(nn - s) << 20 | (s > 0 ? 1u << 25 : 0u);
    };
    for (int i = 0; i < n; i++) {
        const uint32_t t = tok[i], kind = t >> 30;
        uint16_t* c = cdfs + (t & 0x3fffff);
        if (kind == 0) {
            const int nn = (int)((t >> 26) & 15) + 1, s = (int)((t >> 22) & 15);
            words[i] = word(s > 0 ? c[s - 1] : 0, c[s], nn, s);
            update_cdf(c, nn, s);
        } else if (kind == 1) {
            words[i] = t;   // literal tokens are their own word
        } else {
            uint16_t c2[3];
            gather_partition_cdf(c, ((t >> 29) & 1) == 0, c2);
            const int v = (int)((t >> 28) & 1);
            words[i] = word(c2[0], v ? 32768u : c2[0], 2, v);
        }
    }
    return n;
}

}  // extern "C"
