// K10 rate control, shared by the CPU reference controller and the GPU one
// (k_rc_qp after the motion search, k_rc_account after the bitstream), so both
// backends choose the same QP for the same frame.
//
// Modes (reference parity):
//  * CQP  - h264_crf mapped to a constant QP (the round-2 behaviour).
//  * CRF  - the reference's default (CRF 25, src/selkies/settings.py:48, passed to
//           pixelflux at selkies.py:2941): a complexity-adaptive QP around the CRF
//           value. The frame complexity is the motion-compensated SAD per coded
//           macroblock; frames busier than the running average get a coarser QP
//           (x264's qcompress 0.6 curve, QP offset 2.4 * log2(C / C_avg)), quiet
//           frames a finer one.
//  * CBR  - bitrate with a VBV of 1.5 frame intervals (legacy/gstwebrtc_app.py:101-105,
//           630-637: vbv-buf-capacity in frame periods). A leaky-bucket decoder
//           buffer drains one frame budget per frame; each frame's target keeps the
//           buffer near half full and P frames below 1.25x the budget. The QP comes
//           from the previous frame of the same type through the log-linear model
//           bits ~ C * 2^(-QP/6): QP = QP_prev + 6 log2((bits_prev / C_prev) * C / target).
// Integer-only (Q8 log2 with an 8-bit linear mantissa): bit-exact on host and device.
#pragma once
#include "sk_common.h"

namespace sk {
namespace h264 {

enum RcMode : int32_t { RC_CQP = 0, RC_CRF = 1, RC_CBR = 2 };

// Re-code passes an encoder may add to a frame over its per-frame cap (rc_redo_step):
// HEVC two (a scene cut coded at QP 0 needs ~26 QP), H.264 one, AV1 two below 4K (a
// burst - a window opening - can start at 40x the budget; one slope-guessed step left
// 1080p desktop frames at 2-3x) and one at 4K (it sits at the top of its quantiser range
// on 4K120 content, where a further pass rarely gains, and a third 4K pass would cost the
// frame interval). pixels: luma samples per frame.
constexpr int kMaxRecodes = 2;
SK_HD int rc_max_recodes(int codec, int pixels = 0) {
    return codec == 1 ? 2 : (codec == 2 && pixels < 3840 * 2160 / 2 ? 2 : 1);
}

struct RcState {
    int32_t mode, base_qp, qp_min, qp_max;
    int32_t budget;          // CBR bits per frame
    int32_t vbv_size;        // CBR bits
    int32_t fullness;        // bits in the virtual decoder buffer after the last frame
    int32_t frames;          // frames accounted
    int32_t last_qp[2];      // [0] inter frames, [1] intra frames
    int32_t last_bits[2];
    int32_t last_cplx[2];    // complexity per coded MB (x16)
    int32_t cplx_ema;        // CRF: running complexity reference (x16), 0 = none yet
    int32_t cur_qp, cur_intra, cur_cplx;   // the frame in flight (set by rc_frame_qp)
    int32_t max_p_bits;      // statistics: largest inter frame since reset
    int32_t seq;             // GPU: host set_rate() counter applied
    int32_t cur_valid;       // rc_frame_qp chose this frame's QP (its size trains the model)
    int32_t pixels;          // luma samples per frame
    int32_t cur_idr;         // the frame in flight is a planned key frame
    int32_t redos;           // statistics: frames coded twice by the CBR guard
    int32_t qp_floor;        // CBR: inter QP (Q8) at which a frame overflowed recently (0: none)
    int32_t floor_age;       // frames since the floor last moved (it decays 1 QP per 16 frames)
    int32_t last_mbs[2];     // rate-controlled macroblocks of the model frames
    int32_t cur_mbs;         // ... of the frame in flight
    int32_t vbv_ms;          // CBR buffer in ms (0: 1.5 frame intervals), kept across set_rate()
    int32_t last_qpf[2];     // fractional QP (Q8) of the model frames
    int32_t cur_qpf;         // ... of the frame in flight: slices dither between its two QPs
    int32_t cur_redo;        // re-code passes of the frame in flight (rc_redo)
    int32_t redo_qpf;        // ... the fractional QP and payload bits of its pass before the
    int32_t redo_bits;       //     last one (valid when cur_redo > 0)
    int32_t codec;           // EncoderConfig::codec (rc_qp_min_for, rc_redo_step)
    int32_t lam_boost;       // HEVC: QPs above 51 of the frame in flight, added to the RD model's lambda
};
static_assert(sizeof(RcState) == 152, "RcState layout");

SK_HD int rc_ilog2_q8(uint32_t x) {   // log2(x) * 256, linear mantissa; 0 for x <= 1
    if (x <= 1) return 0;
    int m = 31 - __builtin_clz(x);
    const uint32_t frac = m >= 8 ? (x >> (m - 8)) & 255u : (x << (8 - m)) & 255u;
    return m * 256 + (int)frac;
}

// HEVC CBR continues past QP 51: a controller QP 51 + b codes at QP 51 with the RD
// model's lambda b QPs higher (hevc_core.h rd_lambda_q8), so the TU zeroing drops every
// residual that does not pay for itself at that rate - 4K motion content at 20 Mbit/s
// overflowed its frames 1.9x at QP 51. The model, the steps and the re-code passes run on
// the extended scale as on the real one.
constexpr int kLamBoostMax = 18;
SK_HD int rc_lam_boost(int qpf) { return qpf > (51 << 8) ? ((qpf + 128) >> 8) - 51 : 0; }

// vbv_ms: the CBR buffer. 0 = 1.5 frame intervals, the reference's low-latency
// setting for its H.264 / H.265 encoders (legacy/gstwebrtc_app.py:100-104); AV1
// passes 120 ms, svtav1enc's buf-optimal-sz (gstwebrtc_app.py:738).
// Finest controller QP per codec (EncoderConfig::codec). H.264 stops at 10. HEVC and AV1
// go down to 0 like x265's qpmin / svtav1enc's min-qp: transform skip / IDTX and the
// residual trees code a desktop at QP 10 in ~0.65 (HEVC) / ~0.7 (AV1) of a 1080p60 budget
// at 16 Mbit/s, so CBR needs finer QPs to reach the rate (the per-frame guard bounds what
// a burst coded that fine costs). AV1 maps the QP to the qindex of the same step.
SK_HD int rc_qp_min_for(int codec) { return codec == 0 ? 10 : 0; }

// codec: EncoderConfig::codec (0 H.264, 1 HEVC, 2 AV1).
SK_HD void rc_init(RcState& rc, int mode, int base_qp, int bitrate_kbps, float fps, int pixels, int vbv_ms = 0,
                   int codec = 0) {
    rc = RcState{};
    rc.vbv_ms = vbv_ms;
    rc.pixels = pixels;
    rc.mode = mode;
    rc.base_qp = base_qp;
    rc.codec = codec;
    rc.qp_min = rc_qp_min_for(codec);
    rc.qp_max = codec == 1 ? 51 + kLamBoostMax : 51;
    const double f = fps > 0 ? fps : 60.0;
    rc.budget = (int32_t)(bitrate_kbps * 1000.0 / f);
    const long long vbv = vbv_ms > 0 ? (long long)bitrate_kbps * vbv_ms : 0;   // bits
    rc.vbv_size = vbv > rc.budget + rc.budget / 2 ? (int32_t)(vbv > (1ll << 30) ? (1ll << 30) : vbv)
                                                  : rc.budget + rc.budget / 2;   // >= 1.5 frame intervals
    rc.fullness = rc.vbv_size / 2;
    rc.last_qp[0] = rc.last_qp[1] = base_qp;
    rc.last_qpf[0] = rc.last_qpf[1] = rc.cur_qpf = base_qp << 8;
}

// Slice QP of a controller QP: the coded range ends at 51 (HEVC's controller QPs above it
// are lambda boosts, rc_lam_boost).
SK_HD int rc_clamp_qp(const RcState& rc, int qp) { return sk_clip(qp, rc.qp_min, sk_min(rc.qp_max, 51)); }


// Per-frame cap of a non-key frame. A short buffer (vbv_ms 0: 1.5 frame intervals, the
// reference's x264enc / x265enc setting, legacy/gstwebrtc_app.py:101-105, 633): the VBV
// itself. A long buffer (AV1: 120 ms, svtav1enc buf-optimal-sz, :738) is a leaky bucket:
// the frame may fill the buffer but not overflow it (fullness + bits - budget <= size),
// and never above 2.5 budgets (svtav1enc maxsection-pct=250): an empty buffer lets a busy
// frame through at up to 2.5 budgets, a full one holds it to one budget.
// A little under the cap because the packets add stripe headers and NAL framing (~2 %
// at 1080p). Key frames (IDR) may use 4 budgets (their target is 3).
SK_HD long long rc_frame_cap(const RcState& rc, bool key) {
    if (key) return 4ll * rc.budget;
    if (rc.vbv_ms > 0) {
        const long long room = (long long)rc.vbv_size - rc.fullness + rc.budget;   // >= budget
        return sk_min(room, 5ll * rc.budget / 2) - rc.budget / 32;
    }
    return (long long)rc.vbv_size - rc.budget / 16;
}

// QP whose lambda prices motion vectors in the motion search, which runs before the
// frame's QP is chosen: under CRF / CBR the QP of the last rate-controlled inter frame
// (the search at the configured QP picks ragged, expensive vectors when the
// controller runs far coarser), else the planned QP.
SK_HD int rc_me_qp(const RcState& rc, int plan_qp) {
    return (rc.mode != RC_CQP && rc.last_bits[0] > 0) ? rc.last_qp[0] : plan_qp;
}

// QP of the frame about to be coded, fractional (Q8, also left in rc.cur_qpf): the
// slices dither between its two integer QPs (rc_dither_qp), because screen content
// has cliffs - sharp text at one contrast crosses the dead zone within one QP (1080p
// synthetic desktop, H.264: 0.35 budgets at QP 44, above 1.4 at QP 43) - and a
// whole-frame QP then cannot use the budget. cplx_sum: sum of the complexity measure
// over coded_mbs measured MBs (ME SAD for inter frames, source activity for intra);
// mbs: all rate-controlled MBs of the frame (the model scales with their number:
// striped sessions code only the stripes that changed).
SK_HD int rc_frame_qpf(RcState& rc, long long cplx_sum, int coded_mbs, bool intra, bool idr = false, int mbs = 0) {
    const int k = intra ? 1 : 0;
    long long c64 = coded_mbs > 0 ? (cplx_sum * 16) / coded_mbs : 0;
    int cplx = (int)(c64 > (1 << 28) ? (1 << 28) : c64);
    const bool known = cplx > 0;   // planned key frames have no motion search: complexity unknown
    int qp = rc.base_qp << 8;
    if (rc.mode == RC_CRF) {
        if (!intra) {
            if (rc.cplx_ema > 0) {
                const int d = rc_ilog2_q8((uint32_t)cplx) - rc_ilog2_q8((uint32_t)rc.cplx_ema);   // Q8
                const int off = (d * 24 + (d >= 0 ? 1280 : -1280)) / 2560;   // round(2.4 * d / 256)
                qp = (rc.base_qp + sk_clip(off, -3, 6)) << 8;
            }
            rc.cplx_ema = rc.cplx_ema > 0 ? rc.cplx_ema + (cplx - rc.cplx_ema) / 8 : cplx;
        }
    } else if (rc.mode == RC_CBR) {
        int target = rc.budget + (rc.vbv_size / 2 - rc.fullness) / 4;
        // key frames (IDR) may use 3 budgets and are paid back by the frames after
        // them; every other frame, scene-cut intra pictures included, stays under 1.25x.
        // A long buffer (AV1's 120 ms) drains an under-full buffer back towards half full
        // at up to 1.5 budgets per frame (its frames vary +-30 % at one qindex, under the
        // 2.5-budget cap) and never aims above the budget when it is over half full.
        if (idr) target = sk_max(target, 3 * rc.budget);
        else if (rc.vbv_ms > 0) target = sk_min(target, rc.budget + rc.budget / 2);
        else target = sk_min(target, rc.budget + rc.budget / 4);
        target = sk_max(target, rc.budget / 4);
        if (target < 64) target = 64;
        if (rc.last_bits[k] > 0) {
            // screen content is steeper than 6 QP per halving (sharp text: whole
            // coefficient runs cross the dead zone together): 5 QP per halving up,
            // and at most 2 QP finer per frame so a quiet frame cannot set up a burst
            const int dc = (known && rc.last_cplx[k] > 0)   // complexity ratio only when both were measured
                               ? rc_ilog2_q8((uint32_t)cplx) - rc_ilog2_q8((uint32_t)rc.last_cplx[k]) : 0;
            const int dm = (mbs > 0 && rc.last_mbs[k] > 0)   // coded area ratio
                               ? rc_ilog2_q8((uint32_t)mbs) - rc_ilog2_q8((uint32_t)rc.last_mbs[k]) : 0;
            // a large complexity drop (the ordinary frame after a burst: a window opened,
            // a page of text arrived) moves the QP finer at once, outside the per-frame
            // limits below: at 2 QP (AV1: half a QP) per frame the frames after every burst
            // ran at 0.4-0.7 of the budget for a quarter second
            const int dc_down = dc < -128 ? dc : 0;
            const int d = rc_ilog2_q8((uint32_t)rc.last_bits[k]) + (dc - dc_down) + dm - rc_ilog2_q8((uint32_t)target);
            // a long buffer (AV1, vbv_ms) absorbs a misprediction, so its inter frames move
            // gently: 3 QP per halving and at most a quarter QP finer per frame. At the top
            // of AV1's quantiser range an inter frame's size doubles every ~2-3 QP (it
            // re-codes what the coarser frames before it lost): larger steps oscillate
            // (half a QP finer per frame: the per-frame cap catches an overshoot, and a
            // quarter QP left the stream at 0.5-0.7 of its rate for seconds after a burst)
            const bool gentle = rc.vbv_ms > 0 && !intra;
            const int dq = gentle ? 3 * d : (d >= 0 ? 6 * d : 5 * d);   // Q8 QP
            // ... except far below the target (under half of it: the frames after a
            // key frame coded at the top of the range ran at 0.1-0.4 of the budget for the
            // first 40 frames at half a QP per frame): 1.5 QP per frame
            const int fine = gentle ? (d < -(1 << 8) ? -384 : -128) : -512;
            // a complexity drop moves a long-buffer session at most 1 QP at once (the motion
            // search's complexity of screen content swings while the coded size does not)
            const int drop = gentle ? sk_max(3 * dc_down, -256) : 5 * dc_down;
            qp = rc.last_qpf[k] + sk_clip(dq, fine, (intra ? 16 : 10) << 8) + drop;
            // screen content can jump several-fold within one QP (glyph edges crossing the
            // dead zone together): stay above the QP that last overflowed the buffer
            if (!intra && rc.qp_floor > qp) qp = rc.qp_floor;
        } else if (intra && known) {
            // no intra model yet, the activity measured (sum |Y - mean| per MB): about
            // 0.049 bits per unit of activity at QP 39 (dense synthetic text, H.264 and
            // AV1 alike), 5 QP per halving
            const long long tb = ((long long)target << 10) / sk_max(mbs > 0 ? mbs : coded_mbs, 1);   // bits/MB x1024
            const uint32_t est = (uint32_t)sk_min((long long)cplx * 3 + cplx / 8, (long long)1 << 30);   // (0.049 / 16) x1024
            const int d = rc_ilog2_q8(sk_max(est, 2u)) - rc_ilog2_q8((uint32_t)sk_min(sk_max(tb, 2ll), 1ll << 30));
            qp = (39 << 8) + 5 * d;
        } else if (intra) {
            // no intra model and no activity: start from the bits per pixel the budget
            // allows (~0.6 bpp at QP 25 for desktop content, 6 QP per halving)
            const int bpp_q8 = (int)(((long long)target * 256) / sk_max(rc.pixels, 1));   // target bpp x256
            const int d = rc_ilog2_q8(154) - rc_ilog2_q8((uint32_t)sk_max(bpp_q8, 1));  // log2(0.6 / bpp)
            qp = ((25 << 8) + 6 * d + 128) & ~255;
        } else {
            qp = rc.last_qpf[1] + 512;   // first inter frame: a little coarser than the key frame
        }
    }
    qp = sk_clip(qp, rc.qp_min << 8, rc.qp_max << 8);
    rc.cur_qpf = qp;
    rc.cur_qp = (qp + 128) >> 8;
    rc.cur_intra = intra;
    rc.cur_cplx = known ? cplx : 0;   // 0: not measured
    rc.cur_valid = 1;
    rc.cur_idr = idr ? 1 : 0;
    rc.cur_mbs = mbs;
    rc.cur_redo = 0;
    rc.lam_boost = rc_lam_boost(qp);
    return qp;
}

// Integer QP of the i-th rate-controlled slice of a frame at fractional QP qpf: an
// error-diffusion dither, so a fraction f of the slices runs at the coarser QP.
SK_HD int rc_dither_qp(int qpf, int i) {
    const int lo = qpf >> 8, f = qpf & 255;
    return lo + ((((i + 1) * f + 128) >> 8) - ((i * f + 128) >> 8));
}

// A burst: the frame in flight is far busier than the last inter frame (a window
// opening, a page of new text), measured by the motion search before coding.
SK_HD bool rc_burst(const RcState& rc) {
    return rc.cur_cplx > 0 && rc.last_cplx[0] > 0 && 2 * (long long)rc.cur_cplx > 3 * (long long)rc.last_cplx[0];
}

// CBR guard (per-frame cap, rc_frame_cap): a frame whose payload exceeds its cap is
// coded once more, coarser by the QP step this returns (0: keep it). The first step
// assumes the model's 6 QP per halving towards the target; a further one uses the
// slope the frame itself showed between its last two passes (screen content is far
// flatter or steeper than 6 QP per halving). Every codec runs it (H.264 k_rc_guard,
// HEVC / AV1 k_rc_guard_sizes, the CPU encoders alike). When the last pass still
// overflows at QP 51 the frame is sent as coded: the encoder keeps no B frames or
// frame drops, the buffer accounting (rc_account) clamps at the VBV and the next
// frames pay it back.
SK_HD int rc_redo_step(const RcState& rc, long long frame_bits) {
    if (rc.mode != RC_CBR || !rc.cur_valid) return 0;
    // HEVC / AV1 key frames are not re-coded: their intra pass is the longest of the
    // picture (a second one doubled the 4K key-frame latency); the frames after a key
    // frame pay its overshoot back through the buffer, as they pay its planned 3 budgets
    if (rc.cur_idr && rc.codec != 0) return 0;
    if (rc.cur_redo >= rc_max_recodes(rc.codec, rc.pixels)) return 0;
    const long long cap = rc_frame_cap(rc, rc.cur_idr != 0);
    if (frame_bits <= cap) return 0;
    const uint32_t b = (uint32_t)(frame_bits > (1ll << 30) ? (1ll << 30) : frame_bits);
    const int target = sk_max(rc.cur_idr ? 3 * rc.budget : rc.budget, 1);
    const int d = rc_ilog2_q8(b) - rc_ilog2_q8((uint32_t)target);   // Q8 halvings, > 0
    // Q8 QP per halving: 6, except AV1 below QP 24, where screen content measured ~2 QP
    // per halving (1.65 -> 0.37 budgets over 4 QP at QP 17): 6 sent a 2x overflow to a
    // third of the budget there (at QP 40+ it still needs the 6)
    int slope = rc.codec == 2 && rc.cur_qpf < (24 << 8) && !rc_burst(rc) ? 3 << 8 : 6 << 8;
    if (rc.cur_redo > 0) {
        const int dq = rc.cur_qpf - rc.redo_qpf;
        const int dl = rc_ilog2_q8((uint32_t)sk_max(rc.redo_bits, 2)) - rc_ilog2_q8(b);
        slope = (dq > 0 && dl > 0) ? sk_clip((int)(((long long)dq << 8) / dl), 3 << 8, 24 << 8) : 24 << 8;
    }
    return sk_clip((int)(((long long)slope * d + 32768) >> 16), 2, 24);
}

// Model point of a re-coded inter frame: the QP at which its content meets the budget,
// interpolated in log size between its last two passes (extrapolated at their slope
// past the coarser one). Training the model on the coarse re-code itself left the next
// frames several QP too coarse (screen content falls 10x within 4 QP); the first pass
// alone would repeat the overflow.
SK_HD int rc_redo_model_qpf(const RcState& rc, int bits, int target) {
    const int l1 = rc_ilog2_q8((uint32_t)sk_max(rc.redo_bits, 2)), l2 = rc_ilog2_q8((uint32_t)sk_max(bits, 2));
    const int lt = rc_ilog2_q8((uint32_t)sk_max(target, 2));
    const int dq = rc.cur_qpf - rc.redo_qpf;
    if (dq <= 0 || l1 <= l2) return rc.cur_qpf;
    const long long q = (long long)rc.redo_qpf + (long long)dq * (l1 - lt) / (l1 - l2);
    return (int)sk_min(sk_max(q, (long long)rc.qp_min << 8), (long long)rc.qp_max << 8);
}

// The frame in flight (first pass at cur_qp) overflowed: remember its QP as a floor
// for the inter frames after it.
SK_HD void rc_raise_floor(RcState& rc) {
    if (rc.cur_intra) return;
    // a burst (complexity well above the last inter frame's) overflows at any QP the
    // buffer allows for ordinary frames: re-code it, but keep the floor where it is
    if (rc_burst(rc)) return;
    // a quarter QP above the QP that overflowed: the dither reaches the cliff's edge
    rc.qp_floor = sk_max(rc.qp_floor, rc.cur_qpf + 64);
    rc.floor_age = 0;
}

// After the frame: its coded size.
SK_HD void rc_account(RcState& rc, long long frame_bits) {
    const int k = rc.cur_intra ? 1 : 0;
    const int bits = (int)(frame_bits > (1ll << 30) ? (1ll << 30) : frame_bits);
    // frames whose QP the controller did not choose (all static) do not train the model
    if (rc.cur_valid) {   // last_cplx 0: not measured (the next prediction assumes no change)
        if (rc.cur_redo > 0 && !rc.cur_intra) {   // re-coded: the budget point (rc_redo_model_qpf)
            const int q = rc_redo_model_qpf(rc, bits, rc.budget);
            rc.last_qpf[k] = q;
            rc.last_qp[k] = (q + 128) >> 8;
            rc.last_bits[k] = sk_max(rc.budget, 1);
        } else {
            rc.last_qp[k] = rc.cur_qp;
            rc.last_qpf[k] = rc.cur_qpf;
            rc.last_bits[k] = bits > 0 ? bits : 1;
        }
        rc.last_cplx[k] = rc.cur_cplx;
        rc.last_mbs[k] = rc.cur_mbs;
    }
    if (rc.mode == RC_CBR) {
        // an overflow (a key frame far above the buffer) is written off after one
        // frame instead of starving the frames behind it for seconds
        long long f = (long long)rc.fullness + bits - rc.budget;
        rc.fullness = (int32_t)(f < 0 ? 0 : (f > rc.vbv_size ? rc.vbv_size : f));
    }
    if (rc.cur_valid && !rc.cur_intra && bits > rc.max_p_bits) rc.max_p_bits = bits;
    if (rc.qp_floor > 0) {
        // 1 QP per 16 frames (3.75 QP a second at 60 fps); an inter frame coded AT the
        // floor (not above it, not re-coded) in 3/4 of its budget or less says the cliff
        // has passed: half a QP per frame (1080p synthetic desktop, H.264 16 Mbit/s: 7 s
        // at 0.3-0.6 budgets under the slow decay alone)
        const bool at_floor = rc.cur_valid && !rc.cur_intra && rc.cur_qpf <= rc.qp_floor;
        const int step = (at_floor && 4ll * bits < 3ll * rc.budget) ? 128 : 16;
        rc.qp_floor = rc.qp_floor - step > (rc.qp_min << 8) ? rc.qp_floor - step : 0;
        rc.floor_age++;
    }
    rc.cur_valid = 0;
    rc.frames++;
}

}  // namespace h264
}  // namespace sk
