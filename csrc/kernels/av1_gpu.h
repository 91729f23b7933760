// Device buffers and launch interface of the HIP AV1 back end. It runs after the
// H.264 front end (k_convert_damage, k_plan, k_me_mfma, k_motion_search, k_decide)
// on the same FrameArgs and before k_commit (reference / motion-field update).
#pragma once
#include <hip/hip_runtime.h>
#include "h264_gpu.h"
#include "../codec/av1_core.h"
#include "../codec/av1_lf.h"
#include "../codec/av1_cdef.h"

namespace sk {
namespace av1 {
namespace gpu {

constexpr int kLevPerUnit = 384;
constexpr int kTokCap = 4096;        // tokens per 16x16 unit slot (worst case ~3.3k, see tok_bound)
constexpr int kTileChunkCap = 1 << 20;

struct Av1Args {
    h264::gpu::FrameArgs f;   // planes, geometry (mb = 16x16 unit), tasks, motion field
    Av1Geo geo;
    BlkInfo* blk;             // [r8][c8]
    uint8_t* pal;             // [r8][c8][8] palette colours of each cell's block (key frames)
    int palette;              // palette coding of key frames enabled (av1_encoder.h palette_enabled)
    int* pal_rate;            // [r8][c8] key frames: palette_rate2 of the block at that origin cell
                              // (k_av1_intra_modes; its colour count rides in BlkInfo.pad1 until
                              // k_av1_intra_rec decides)
    int16_t* lev;             // [units][kLevPerUnit]
    uint8_t* lctx[3];         // level contexts per plane (4x4 units), strides lctx_w
    int lctx_w[3];
    uint32_t* tok;            // [units][kTokCap]
    int* tok_n;               // [units]
    uint32_t* tokc;           // [tiles][tile_tok_cap]: each tile's tokens in coding order
    uint32_t* pw;             // [tiles][tile_tok_cap]: interval word of each symbol token (k_av1_cdf)
    int tile_tok_cap;
    int* tok_off;             // [units] offset of the unit's tokens in its tile's stream
    int* tile_ntok;           // [tiles]
    int* frame;               // device: [0] key, [1] qidx
    int* frame_host;          // host-mapped copy of frame[0..2]
    h264::gpu::Planes cdef_in;   // the deblocked picture CDEF reads (k_av1_cdef writes f.rec)
    const uint8_t* qidx_of_qp;   // [52]
    int tile_cap;             // byte capacity per tile
    // block-parallel coder (k_av1_ec_*): per block 128 candidate (exit rng, shift count)
    // maps and {first token, end, entry rng, shift prefix}; per tile the big integer low
    // as 64-bit digit sums (ecv), its carried 32-bit digits (ecf) and its total shift
    uint2* ecmap;             // [ec_max_blocks][128]
    int4* ecblk;              // [ec_max_blocks]
    int ec_max_blocks;
    unsigned long long* ecv;  // [tiles][ec_vcap]
    uint32_t* ecf;            // [tiles][ec_vcap]
    int ec_vcap;
    int* tile_bits;           // [tiles] total shift D (-1: over capacity)
    int* tile_size;           // device [tiles] bytes
    uint8_t* out_host;        // host-mapped tile bytes, concatenated [out_cap]
    int out_cap;
    int* out_size_host;       // host-mapped [tiles] bytes (-1: did not fit out_cap)
};

// redo: the K10 re-code flag (CBR sessions): the coding kernels run a second time,
// gated on it, after k_rc_guard_sizes checked the frame against its cap; nullptr: one pass.
void launch_backend(const Av1Args& a, hipStream_t s, int* redo = nullptr);
// Sizes of the coder's block maps and big-integer digits for tiles of tile_bytes.
void ec_buffers(int tiles, int tile_bytes, int* max_blocks, int* vcap);

}  // namespace gpu
}  // namespace av1
}  // namespace sk
