// H.265 high-level syntax shared by the CPU reference and the GPU slice assembly:
// a bit writer, the slice segment header (7.3.6.1) with WPP entry points, and
// emulation prevention (7.4.2). Parameter sets (VPS/SPS/PPS) are host-only
// (hevc_params.cpp).
#pragma once
#include "sk_common.h"

namespace sk {
namespace hevc {

// MSB-first bit writer into a zero-initialised byte buffer.
struct HBitWriter {
    uint8_t* buf;
    uint32_t pos;   // bits
    SK_HD void put1(int b) {
        if (b) buf[pos >> 3] |= (uint8_t)(0x80u >> (pos & 7));
        pos++;
    }
    SK_HD void put(uint32_t v, int n) {
        for (int i = n - 1; i >= 0; i--) put1((v >> i) & 1);
    }
    SK_HD void ue(uint32_t v) {
        const uint32_t x = v + 1;
        int len = 0;
        while ((x >> len) > 1) len++;
        put(0, len);
        put(x, len + 1);
    }
    SK_HD void se(int v) { ue(v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * v)); }
    SK_HD void align_one() {   // byte_alignment() / rbsp_trailing_bits(): '1' then zeros
        put1(1);
        while (pos & 7) put1(0);
    }
};

constexpr int kNalIdrWRadl = 19, kNalTrailR = 1, kNalVps = 32, kNalSps = 33, kNalPps = 34;
constexpr int kLog2MaxPocLsb = 16;

struct SliceHeader {
    int first_slice;      // first_slice_segment_in_pic_flag
    int idr;              // nal_unit_type IDR_W_RADL (else TRAIL_R)
    int address;          // slice_segment_address (CTB raster address)
    int address_bits;     // Ceil(Log2(PicSizeInCtbsY))
    int slice_type;       // 1 = P, 2 = I
    int poc_lsb;
    int qp_delta;         // SliceQpY - 26
    int num_entry;        // num_entry_point_offsets
    const int* entry;     // EP-escaped substream sizes in bytes (entry_point_offset_minus1 + 1)
};

SK_HD int bit_length(uint32_t v) {
    int n = 0;
    while (v >> n) n++;
    return n;
}

// Writes the slice segment header RBSP (including byte_alignment()) into a zeroed
// buffer; returns its size in bytes.
SK_HD int write_slice_header(uint8_t* buf, const SliceHeader& h) {
    HBitWriter w{buf, 0};
    w.put1(h.first_slice);
    if (h.idr) w.put1(0);                  // no_output_of_prior_pics_flag
    w.ue(0);                               // slice_pic_parameter_set_id
    if (!h.first_slice) w.put((uint32_t)h.address, h.address_bits);
    w.ue((uint32_t)h.slice_type);
    if (!h.idr) {
        w.put((uint32_t)h.poc_lsb, kLog2MaxPocLsb);
        w.put1(1);                         // short_term_ref_pic_set_sps_flag (the SPS's one RPS)
    }
    w.put1(1);                             // slice_sao_luma_flag (per-CTB decisions, hevc_sao.h)
    w.put1(1);                             // slice_sao_chroma_flag
    if (h.slice_type == 1) {
        w.put1(0);                         // num_ref_idx_active_override_flag
        w.ue(0);                           // five_minus_max_num_merge_cand
    }
    w.se(h.qp_delta);
    w.ue((uint32_t)h.num_entry);
    if (h.num_entry > 0) {
        uint32_t mx = 0;
        for (int i = 0; i < h.num_entry; i++) mx = mx > (uint32_t)(h.entry[i] - 1) ? mx : (uint32_t)(h.entry[i] - 1);
        const int len = bit_length(mx) > 0 ? bit_length(mx) : 1;
        w.ue((uint32_t)(len - 1));         // offset_len_minus1
        for (int i = 0; i < h.num_entry; i++) w.put((uint32_t)(h.entry[i] - 1), len);
    }
    w.align_one();
    return (int)(w.pos >> 3);
}

// Emulation prevention of one independent piece (the byte before it is non-zero):
// returns the escaped size; writes when out != nullptr.
SK_HD int ep_escape(const uint8_t* in, int n, uint8_t* out) {
    int zeros = 0, o = 0;
    for (int i = 0; i < n; i++) {
        const uint8_t b = in[i];
        if (zeros >= 2 && b <= 3) {
            if (out) out[o] = 3;
            o++;
            zeros = 0;
        }
        if (out) out[o] = b;
        o++;
        zeros = b == 0 ? zeros + 1 : 0;
    }
    return o;
}

}  // namespace hevc
}  // namespace sk
