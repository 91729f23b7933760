// Chunk-parallel CABAC coding of one substream (an HEVC CTB-row substream), exact.
//
// The arithmetic coder is linear in its code value: with V the unbounded "low" register
// and T the number of renormalisation shifts so far, every bin does
//     V <- (V + a) * 2^k + c          (a, c, k depend only on the range and the bin),
// so the substream's final value is the sum, over any split of the bins into chunks, of
// each chunk's own value coded from V = 0 -- provided each chunk starts from its true
// range -- shifted by the number of shifts after the chunk. The range evolves
// independently of V. That gives four parallel phases (kernels/hevc_kernels.hip):
//   1. context modelling: per (row, context) chain of state transitions (the states a
//      serial coder would see), written back as "modelled" entries (LPS state, is-LPS);
//   2. range maps: per chunk (= CTB), the end range and shift count for every start range;
//   3. composition: per row, start range and bit offset of every chunk (a map lookup each);
//   4. chunk coding: per chunk, the HM coder from V = 0 with the chunk's start range and bit
//      offset, fully flushed; its bytes are the chunk's exclusive bytes plus a 2-byte tail
//      that overlaps the next chunk and is added (with carries) in a final merge.
// Stream bit i of the substream is bit T_f + 8 - i of the final value; a chunk starting at
// stream bit t with K shifts covers stream bits [t, t + K + 9).
// Host model: pc_code_row_host() (codec/hevc_cpu.cpp, SK_HEVC_PCABAC=1 and the tests).
#pragma once
#include <stdint.h>
#include "hevc_core.h"

namespace sk {
namespace hevc {

constexpr uint32_t kPcModeled = 0x4000u;   // modelled context bin: bits 0..5 LPS state, bit 6 is-LPS
constexpr int kPcCtxOff = 144;             // per-CU context offsets: CTX_COUNT + 1 entries, padded
static_assert(kPcCtxOff >= CTX_COUNT + 1 && kPcCtxOff % 4 == 0 && kPcCtxOff <= 192,
              "k_pc_sort: three counters per lane, 64 lanes");

// Renormalisation shift of a range 1..510: doublings until it is >= 256.
SK_HD int pc_renorm(uint32_t r) {
    const int k = __builtin_clz(r) - 23;
    return k > 0 ? k : 0;
}

// Modelled entry of context bin `bin` under state byte s (9.3.4.2); advances s.
SK_HD uint16_t pc_model(uint8_t& s, int bin) {
    const int st = s >> 1, lp = bin ^ (s & 1);
    ctx_update(s, bin);
    return (uint16_t)(kPcModeled | (lp << 6) | st);
}

// Range-only step of one entry (modelled context bin, bypass run or terminating bin):
// returns the renormalisation shift (for a bypass run: its length).
SK_HD int pc_range_step(uint32_t e, uint32_t& r) {
    if ((e & 0xC000u) == kPcModeled) {
        const uint32_t lps = CABAC_LPS[e & 63u][(r >> 6) & 3];
        const uint32_t nr = (e & 64u) ? lps : r - lps;
        const int k = pc_renorm(nr);
        r = nr << k;
        return k;
    }
    if (e & 0x8000u) return (int)((e >> 12) & 7u) + 1;
    r -= 2;   // terminating bin
    if ((e >> 8) & 1u) {
        r = 256;
        return 7;
    }
    if (r < 256) {
        r <<= 1;
        return 1;
    }
    return 0;
}

// Host LPS row lookup for PcCoder::code.
struct PcLpsTable {
    SK_HD uint32_t operator()(uint32_t st) const {
        return (uint32_t)CABAC_LPS[st][0] | ((uint32_t)CABAC_LPS[st][1] << 8) | ((uint32_t)CABAC_LPS[st][2] << 16) |
               ((uint32_t)CABAC_LPS[st][3] << 24);
    }
};

// HM arithmetic coder over modelled entries, started from V = 0 with range r at bit
// offset o (0..7) inside its first byte; flush() emits every remaining bit of V.
struct PcCoder {
    uint32_t low, range, buffered;
    int bits_left, nbuf;
    SK_HD void start(uint32_t r, int o) {
        low = 0;
        range = r;
        bits_left = 23 - o;
        nbuf = 0;
        buffered = 0xff;
    }
    template <class Emit>
    SK_HD void write_out(Emit& emit) {
        const uint32_t lead = low >> (24 - bits_left);
        bits_left += 8;
        low &= 0xffffffffu >> bits_left;
        if (lead == 0xff) {
            nbuf++;
        } else if (nbuf > 0) {
            const uint32_t carry = lead >> 8;
            emit((buffered + carry) & 0xffu);
            buffered = lead & 0xff;
            const uint32_t fill = (0xff + carry) & 0xff;
            while (nbuf > 1) {
                emit(fill);
                nbuf--;
            }
        } else {
            nbuf = 1;
            buffered = lead;
        }
    }
    // lps4(state): the state's four LPS ranges packed in bytes (q = 0..3)
    template <class Emit, class Lps>
    SK_HD void code(uint32_t e, Emit& emit, Lps& lps4) {
        if ((e & 0xC000u) == kPcModeled) {
            const uint32_t lps = (lps4(e & 63u) >> ((range >> 3) & 24u)) & 0xffu;
            const uint32_t rmps = range - lps;
            uint32_t nr = rmps;
            if (e & 64u) {
                low += rmps;
                nr = lps;
            }
            const int k = pc_renorm(nr);
            low <<= k;
            range = nr << k;
            bits_left -= k;
        } else if (e & 0x8000u) {
            const int n = (int)((e >> 12) & 7u) + 1;
            low = (low << n) + range * (e & 0xffu);
            bits_left -= n;
        } else {
            range -= 2;
            if ((e >> 8) & 1u) {
                low += range;
                low <<= 7;
                range = 2 << 7;
                bits_left -= 7;
            } else if (range < 256) {
                low <<= 1;
                range <<= 1;
                bits_left--;
            }
        }
        if (bits_left < 12) write_out(emit);
    }
    template <class Emit>
    SK_HD void flush(Emit& emit) {
        const int m = 32 - bits_left;   // bits of V not yet emitted (bits_left >= 12: m <= 20)
        const uint32_t c = low >> m;    // carry into the outstanding bytes
        if (nbuf > 0) {
            emit((buffered + c) & 0xffu);
            const uint32_t fill = c ? 0x00u : 0xffu;
            while (nbuf > 1) {
                emit(fill);
                nbuf--;
            }
        }
        uint32_t v = low & ((1u << m) - 1);
        int left = m;
        while (left >= 8) {
            emit((v >> (left - 8)) & 0xffu);
            left -= 8;
        }
        if (left > 0) emit((v << (8 - left)) & 0xffu);
    }
};

}  // namespace hevc
}  // namespace sk
