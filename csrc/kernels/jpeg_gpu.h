// Device-side interface of the gfx950 JPEG stripe kernels (jpeg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../codec/jpeg_encoder.h"

namespace sk {
namespace jpeg {
namespace gpu {

// Worst case per 8x8 block: DC 22 bits + 63 AC symbols of <= 26 bits + EOB,
// doubled for 0xFF00 stuffing.
constexpr int kMaxBlockBytes = 416;
constexpr int kTileBytes = 4096;        // byte-stuffing tile (one workgroup)
constexpr int kBlockWords = 56;         // LDS words per block bitstring (<= 1695 bits)

struct JpegArgs {
    int W, H, stripe_h, num_stripes, mcu_w;
    int blocks_per_stripe;        // blocks of a full-height stripe (slot stride)
    const uint8_t* cur;           // BGRx frame (device), `stride` bytes per row
    const uint8_t* prev;          // previous frame (device) for damage
    int stride;
    // Frame-parity double buffers (the host swaps them per hipGraph): k_damage
    // writes dirty_in, every k_blocks workgroup evaluates the stripe plan from
    // state_in (deterministic, no cross-workgroup sync), workgroup 0 of each
    // stripe publishes state_out / action / host_action and clears dirty_out.
    int* dirty_in;
    int* dirty_out;
    const JpegStripeState* state_in;
    JpegStripeState* state_out;
    int* action;                  // [num_stripes] -1 skip, 0 quality, 1 paint quality (device)
    int* host_action;             // host-mapped copy of `action` for packet assembly
    const volatile int* key_seq;  // host-mapped keyframe-request counter (read once per frame)
    int* key_now;                 // device copy of key_seq for this frame
    int use_paint_over, paint_over_trigger;
    const JpegTables* tabs;       // [2]
    int16_t* coef;                // [num_stripes * blocks_per_stripe * 64] zig-zag levels
    int16_t* dc;                  // [.. blocks] quantised DC
    int16_t* dcdiff;              // [.. blocks] DC difference (coding order)
    int* ac_bits;                 // [.. blocks] AC + EOB bits
    int* blk_off;                 // [.. blocks] bit offset inside the stripe
    int* stripe_bits;             // [num_stripes] entropy-coded bits
    uint32_t* bits;               // [num_stripes * bits_slot_words] big-endian bit buffer
    int bits_slot_words;
    int* tile_ff;                 // [num_stripes * max_tiles] 0xFF count per stuffing tile
    int max_tiles;
    uint8_t* host_out;            // host-mapped [num_stripes * out_slot]
    int* host_size;               // host-mapped [num_stripes]
    int out_slot;
};

// damage -> blocks(+plan) -> scan -> write -> ffcount -> stuff (one graph per parity)
void launch_frame(const JpegArgs& a, hipStream_t s);

}  // namespace gpu
}  // namespace jpeg
}  // namespace sk
