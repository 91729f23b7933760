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
    int* stripe_dirty;            // [num_stripes] (k_decide clears it for the next frame)
    int* action;                  // [num_stripes] -1 skip, 0 quality, 1 paint quality (device)
    int* host_action;             // host-mapped copy of `action` for packet assembly
    JpegStripeState* state;       // [num_stripes] damage / paint-over state (device resident)
    int* ctl;                     // [0] first frame, [1] keyframe seq seen, [2] stripe counter, [32*(s+1)] WG counters (one cache line each)
    const volatile int* key_seq;  // host-mapped keyframe-request counter
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

// damage(+decide) is launched directly after the upload; blocks -> scan ->
// write -> ffcount -> stuff are captured in a graph.
void launch_damage(const JpegArgs& a, hipStream_t s);
void launch_encode(const JpegArgs& a, hipStream_t s);

}  // namespace gpu
}  // namespace jpeg
}  // namespace sk
