// Device buffers and launch interface of the HIP HEVC back end. It runs after the
// H.264 front end (k_convert_damage, k_plan, k_me_mfma, k_motion_search, k_decide)
// on the same FrameArgs and before k_commit (reference / motion-field update).
#pragma once
#include <hip/hip_runtime.h>
#include "h264_gpu.h"
#include "../codec/hevc_core.h"
#include "../codec/hevc_syntax.h"
#include "../codec/hevc_pcabac.h"
#include "../codec/hevc_sao.h"

namespace sk {
namespace hevc {
namespace gpu {

// Geometry: f.mb_w x f.mb_h are the 16x16 units (the front end's macroblocks); the CTBs
// (32x32) are cw x ch, slices rows_per_slice CTB rows (f.rows_per_slice is in units).
// Per-unit arrays are indexed by unit (uy * mb_w + ux); the chunk-parallel coder's chunks
// are the units of a CTB row in coding order (UnitGrid::chunk_unit).
struct HevcArgs {
    h264::gpu::FrameArgs f;     // planes, geometry (mb = unit), tasks, motion field
    int cw, ch, rps;            // CTBs per row / column, CTB rows per slice
    CuInfo* cus;                // [units]
    int16_t* coefs;             // [units][kCoefPerCu]
    uint16_t* bins;             // [units][kCuBinCap]
    int* bin_n;                 // [units]
    uint8_t* sync;              // [ch][CTX_COUNT] WPP context states at each row start
    uint8_t* sub;               // [ch][sub_stride] CABAC substreams (one per CTB row)
    int sub_stride;
    int* sub_size;              // [ch] bytes
    int* sub_esc;               // [ch] bytes after emulation prevention
    int* row_off;               // [ch] byte offset of the row's substream inside its slice NAL
    uint8_t* out_host;          // host-mapped slice slots [num_slices][out_slot]
    int* out_size;              // host-mapped [num_slices]: NAL bytes (> out_slot: in out_dev)
    uint8_t* out_dev;           // device fallback slots [num_slices][out_dev_slot]
    int out_slot, out_dev_slot;
    int addr_bits;
    unsigned long long* dbg;    // optional (SK_STAMPS): per CTB row [cycles, entries, bytes, 0]
    int reg_steps;              // k_hevc_intra: 4x4 TUs in registers (default; SK_HEVC_REG_STEPS=0: LDS batches)
    // chunk-parallel substream coding (codec/hevc_pcabac.h), chunk = unit
    uint16_t* srt;              // [units][kCuBinCap] the unit's context bins sorted by context: index << 1 | bin
    uint16_t* coff;             // [ch][kPcCtxOff][2 * mb_w] start of each context's run in srt, per chunk (last = count)
    uint32_t* rmap;             // [units][256] end range | shifts << 9, per start range 256..511
    uint32_t* cu_t;             // [units] stream bit offset of the unit's chunk inside its row substream
    uint16_t* cu_r;             // [units] start range of the chunk
    uint8_t* tail;              // [units][2] the chunk's two bytes overlapping the next chunk
    uint32_t* row_bits;         // [ch] shifts of the whole row (T_f)
    // SAO (codec/hevc_sao.h) on the deblocked reconstruction
    SaoStats* sao_stats;        // [ctbs][3] Y, Cb, Cr (CTB = 32x32)
    SaoParams* sao_own;         // [ctbs] each CTB's own decision (k_hevc_sao_stats)
    long long* sao_cost;        // [ctbs] its cost
    long long* sao_md;          // [ctbs][kSaoMd] merge-candidate distortions (sao_merge_dists)
    SaoParams* sao;             // [ctbs] final parameters after the row merge pass (k_hevc_sao_row)
    h264::gpu::Planes sao_tmp;  // filtered samples of the CTBs SAO changes, copied back into f.rec
    // intra slices cut every CTB row into seg_k slices (SliceMap, hevc_core.h); the
    // substream arrays (sync, sub_size, sub_esc, row_off, row_bits) hold mb_h * seg_k
    // slots (slot = cy * seg_k + k, k = 0 for whole rows); segment k of CTB row cy codes its
    // substream at sub + cy * sub_stride + x0 * 4 * kSubstreamCtbBytes + 64 * k
    int seg_k;
    int pc_seg;                 // k_pc_model: shortest speculative chain segment (SK_HEVC_PC_SEG, default 32)
};

// redo: the K10 re-code flag (CBR sessions): the coding kernels run a second time,
// gated on it, after k_rc_guard_sizes checked the frame against its cap; nullptr: one pass.
void launch_backend(const HevcArgs& a, hipStream_t s, int* redo = nullptr);

}  // namespace gpu
}  // namespace hevc
}  // namespace sk
