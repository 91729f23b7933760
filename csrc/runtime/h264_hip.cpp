// HIP backend of the H.264 stripe encoder: owns the per-session HBM buffers,
// the stream, pinned staging, and drives the gfx950 kernels
// (csrc/kernels/h264_kernels.hip). Frame flow:
//   H2D(BGRx) -> [K1/K3 convert+damage, k_plan (stripe controller on the GPU),
//   K4 ME, decide, K6 inter, K5/K6 intra, K8 CAVLC, K9 slice assembly into
//   host-mapped packet slots, commit] (one hipGraph per src/prev parity)
//   -> one sync -> packets. No host decision sits inside a frame.
#include "encoder_iface.h"
#include "trace.h"
#include "../kernels/h264_gpu.h"
#include "../kernels/hevc_gpu.h"
#include "../kernels/av1_gpu.h"
#include "../codec/av1_encoder.h"
#include "../kernels/runtime_kernels.h"
#include "../codec/hevc_encoder.h"
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string.h>
#include <string>
#include <thread>
#include <vector>
#include <atomic>

namespace sk {
namespace {

#define HIPCHECK(x)                                                                     \
    do {                                                                                \
        hipError_t e__ = (x);                                                           \
        if (e__ != hipSuccess)                                                          \
            throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e__)); \
    } while (0)

using namespace h264;

class HipBackend : public EncoderBackend {
   public:
    HipBackend(const EncoderConfig& c, int device) : cfg_(c), device_(device) {
        if (cfg_.codec == 2) av1::cbr_config(cfg_);   // AV1 CBR as the CPU encoder (av1_encoder.h)
        if (cfg_.codec == 1) {   // HEVC: CBR without scene-cut intra slices, stripes of whole CTB rows (hevc_encoder.h)
            hevc::cbr_config(cfg_);
            hevc::hevc_geometry(cfg_);
        }
        g_.init(cfg_);
        ctl_.init(cfg_, g_);
        HIPCHECK(hipSetDevice(device_));
        warm_copy_engines(device_);
        HIPCHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
        for (auto& e : ev_) HIPCHECK(hipEventCreate(&e));
        for (auto& e : ev_copy_) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        if (cfg_.shared_copy) copy_stream_ = device_copy_stream(device_);
        alloc();
        if (cfg_.codec == 1) alloc_hevc();
        if (cfg_.codec == 2) alloc_av1();
    }
    ~HipBackend() override {
        hipSetDevice(device_);
        for (auto& gx : graph_exec_)
            if (gx) hipGraphExecDestroy(gx);
        for (auto& gx : post_exec_)
            if (gx) hipGraphExecDestroy(gx);
        for (void* p : dev_allocs_) hipFree(p);
        for (void* p : host_allocs_) hipHostFree(p);
        for (auto& e : ev_) hipEventDestroy(e);
        for (auto& e : ev_copy_) hipEventDestroy(e);
        if (ev_ext_) hipEventDestroy(ev_ext_);
        for (auto* b : bgrx_dev_)
            if (b) hipFree(b);
        hipStreamDestroy(stream_);
        if (up_stream_) hipStreamDestroy(up_stream_);
    }

    // Picked up by k_plan at the start of the next frame.
    void request_keyframe() override { __atomic_fetch_add(h_key_seq_, 1, __ATOMIC_SEQ_CST); }
    // Host-mapped overrides, read by k_plan at the start of the next frame.
    void set_qp(int qp, int paint_qp) override {
        if (qp > 0) __atomic_store_n(&h_key_seq_[1], qp, __ATOMIC_SEQ_CST);
        if (paint_qp > 0) __atomic_store_n(&h_key_seq_[2], paint_qp, __ATOMIC_SEQ_CST);
    }
    // K10: picked up by k_rc_qp at the next frame (a change counter tells it apart).
    void set_rate(int mode, int kbps) override {
        cfg_.rc_mode = mode;   // graphs re-captured with / without the CBR guard (launch)
        __atomic_store_n(&h_key_seq_[3], mode, __ATOMIC_SEQ_CST);
        __atomic_store_n(&h_key_seq_[4], kbps, __ATOMIC_SEQ_CST);
        __atomic_fetch_add(&h_key_seq_[5], 1, __ATOMIC_SEQ_CST);
    }
    int64_t rc_stats(int32_t* out, int n) override {
        HIPCHECK(hipSetDevice(device_));
        HIPCHECK(hipStreamSynchronize(stream_));
        RcState rc;
        copy_now(&rc, args_.rc, sizeof(rc));
        const int k = n < (int)(sizeof(rc) / 4) ? n : (int)(sizeof(rc) / 4);
        memcpy(out, &rc, (size_t)k * 4);
        return k;
    }

    int encode(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        submit(bgrx, stride, frame_id);
        return finish();
    }

    int submit(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        if (upload(bgrx, stride, frame_id) < 0) return -1;
        return launch();
    }

    // Stage a frame: H2D into the input buffer of the frame's parity on the copy
    // stream. May be called while the previous frame is still encoding (its upload
    // then overlaps that frame's kernels); launch() comes after finish() of it.
    double upload_fraction() const override {
        const long long t = up_rows_total_.load();
        return t ? (double)up_rows_copied_.load() / (double)t : 1.0;
    }
    void set_upload_rows(const int* r, int n) override {
        up_next_known_ = n >= 0;
        up_next_.assign(r && n > 0 ? r : nullptr, r && n > 0 ? r + 2 * n : nullptr);
    }

    // Damage-driven upload: bgrx_dev_[q] holds the frame uploaded two frames ago, so the
    // rows that changed since then (this frame's damage and the previous frame's) are
    // copied; everything else is already on the device. Full copy when either damage is
    // unknown, the buffer was never filled or the frame is scaled on the device.
    void upload_copy(int q, const uint8_t* bgrx, int stride, size_t in_bytes, hipStream_t cs) {
        const int rows = (int)(in_bytes / (size_t)stride);
        const bool partial = up_valid_[q] && up_next_known_ && up_prev_known_ && !args_.scaled;
        if (!partial) {
            HIPCHECK(hipMemcpyAsync(bgrx_dev_[q], bgrx, in_bytes, hipMemcpyDefault, cs));
        } else {
            // union of the two damage lists on 16-row bands, copied as maximal row ranges
            for (const auto& r : upload_ranges({&up_next_, &up_prev_}, rows)) {
                HIPCHECK(hipMemcpyAsync(bgrx_dev_[q] + (size_t)r.first * stride, bgrx + (size_t)r.first * stride,
                                        (size_t)(r.second - r.first) * stride, hipMemcpyDefault, cs));
                up_rows_copied_ += r.second - r.first;
            }
        }
        if (!partial) up_rows_copied_ += rows;
        up_rows_total_ += rows;
        up_valid_[q] = true;
        up_prev_known_ = up_next_known_;
        up_prev_.swap(up_next_);
        up_next_known_ = false;   // one damage report per upload
        up_next_.clear();
    }

    // Planar input: the planes are staged (2D copies, H2D or D2D) into this parity's
    // staging buffer in the packed layout k_yuv_damage reads; the graphs are captured
    // per input kind (BGRx / I420 / NV12).
    int encode_yuv(const YuvInput& in, int on_device, uint16_t frame_id) override {
        if (upload_yuv(in, on_device, frame_id) < 0) return -1;
        if (launch() < 0) return -1;
        return finish();
    }

    int upload_yuv(const YuvInput& in, int on_device, uint16_t frame_id) {
        trace::Range frame_range("h264.upload_yuv");
        HIPCHECK(hipSetDevice(device_));
        if (args_.scaled) {
            set_last_error("planar input cannot be resampled (src size != encoder size)");
            return -1;
        }
        if (inflight() >= 2) {
            set_last_error("upload(): two frames in flight; finish() the oldest first");
            return -1;
        }
        const int W = g_.W, H = g_.H, cw = (W + 1) / 2, ch = (H + 1) / 2;
        const size_t need = (size_t)W * H + (size_t)2 * cw * ch;
        if (!yuv_dev_[0] || yuv_mode_ != in.fmt) {
            HIPCHECK(hipStreamSynchronize(stream_));
            if (!yuv_dev_[0])
                for (auto& b : yuv_dev_) b = dmalloc<uint8_t>(need, false);
            invalidate_graphs();
            yuv_mode_ = in.fmt;
        }
        const int q = launched_ & 1;
        HIPCHECK(hipEventRecord(ev_[3 * q], stream_));
        const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
        uint8_t* d = yuv_dev_[q];
        HIPCHECK(hipMemcpy2DAsync(d, W, in.p[0], in.stride[0], W, H, k, stream_));
        if (in.fmt == YUV_NV12) {
            HIPCHECK(hipMemcpy2DAsync(d + (size_t)W * H, 2 * cw, in.p[1], in.stride[1], 2 * cw, ch, k, stream_));
        } else {
            HIPCHECK(hipMemcpy2DAsync(d + (size_t)W * H, cw, in.p[1], in.stride[1], cw, ch, k, stream_));
            HIPCHECK(hipMemcpy2DAsync(d + (size_t)W * H + (size_t)cw * ch, cw, in.p[2], in.stride[2], cw, ch, k,
                                      stream_));
        }
        up_valid_[0] = up_valid_[1] = false;   // the BGRx buffers no longer hold the last frames
        staged_on_main_ = true;
        staged_ = true;
        staged_frame_ = frame_id;
        return 0;
    }

    int upload(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        trace::Range frame_range("h264.upload");
        HIPCHECK(hipSetDevice(device_));
        if (yuv_mode_) {   // back to BGRx input: graphs with k_convert_damage
            HIPCHECK(hipStreamSynchronize(stream_));
            invalidate_graphs();
            yuv_mode_ = 0;
        }
        const size_t in_bytes = (size_t)stride * (args_.scaled ? args_.scale.src_h : g_.H);
        if (in_bytes > bgrx_cap_ || stride != args_.bgrx_stride) {
            HIPCHECK(hipStreamSynchronize(stream_));   // geometry change: drain, then reallocate
            if (in_bytes > bgrx_cap_) {
                for (auto*& b : bgrx_dev_) {
                    if (b) hipFree(b);
                    HIPCHECK(hipMalloc(&b, in_bytes));
                }
                bgrx_cap_ = in_bytes;
            }
            up_valid_[0] = up_valid_[1] = false;
            invalidate_graphs();
            args_.bgrx_stride = stride;
        }
        if (inflight() >= 2) {
            set_last_error("upload(): two frames in flight; finish() the oldest first");
            return -1;
        }
        const int q = launched_ & 1;   // parity this frame is launched with
        // A re-upload before launch (the staged frame was never launched) overwrites
        // bgrx_dev_[q] again: the two-frames-ago invariant of upload_copy no longer holds
        // for either parity, so the next two uploads are full copies.
        if (staged_) up_valid_[0] = up_valid_[1] = false;
        // Nothing in flight: copy on the encoder's own stream (no cross-stream wait).
        // Overlapped upload, or bands of one frame: the device's shared copy stream, so
        // the uploads of all encoders on this GPU run back to back at full PCIe rate
        // instead of contending (one copy queue, not one per session). Copies behind
        // kernels on one stream stall in a fresh process until warm_copy_engines() ran.
        hipStream_t cs = stream_;
        // Overlapped upload of a session: its own upload stream (the copies of many
        // sessions then spread over the SDMA engines; SK_SHARED_UPLOAD=1 funnels them
        // through the device's one shared copy stream instead).
        if (copy_stream_) cs = copy_stream_;
        else if (inflight() && upload_mode_ != 0) cs = upload_mode_ == 2 ? device_copy_stream(device_) : upload_stream();
        if (ext_wait_) {   // wait_stream(): the source is written by another stream's queued work
            HIPCHECK(hipStreamWaitEvent(cs, ev_ext_, 0));
            ext_wait_ = false;
        }
        // the last reader of bgrx_dev_[q] is the graph two frames back: finished
        HIPCHECK(hipEventRecord(ev_[3 * q], cs));
        // hipMemcpyDefault: the frame may be host memory (capture) or device memory (a band
        // scattered to this GPU over RCCL, parallel/dist_banded.py)
        upload_copy(q, bgrx, stride, in_bytes, cs);
        if (cs != stream_) HIPCHECK(hipEventRecord(ev_copy_[q], cs));
        staged_on_main_ = cs == stream_;
        staged_ = true;
        staged_frame_ = frame_id;
        return 0;
    }

    int wait_stream(void* stream) override {
        HIPCHECK(hipSetDevice(device_));
        if (!ev_ext_) HIPCHECK(hipEventCreateWithFlags(&ev_ext_, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(ev_ext_, (hipStream_t)stream));
        ext_wait_ = true;
        return 0;
    }

    int launch() override {
        if (!staged_ || inflight() >= 2) {
            set_last_error("launch() needs one uploaded frame and at most one frame in flight");
            return -1;
        }
        trace::Range frame_range("h264.launch");
        HIPCHECK(hipSetDevice(device_));
        const int p = launched_ & 1;
        parity_ = p;
        if ((cfg_.rc_mode == RC_CBR) != graph_guard_) {   // K10 CBR guard in / out of the graphs
            HIPCHECK(hipStreamSynchronize(stream_));
            invalidate_graphs();
            graph_guard_ = cfg_.rc_mode == RC_CBR;
        }
        set_parity_args(args_.bgrx_stride);   // bgrx = bgrx_dev_[p], host outputs of parity p
        // host-mapped, read by this frame's k_plan: per parity, because with two frames
        // in flight the previous frame's k_plan may not have run yet
        h_frame_params_[p][0] = staged_frame_;
        // keyframe request counter and QP overrides as of this launch: a request made
        // before launch(n) applies to frame n even when frame n-1 has not planned yet
        for (int i = 0; i < 6; i++) h_key_snap_[p][i] = __atomic_load_n(&h_key_seq_[i], __ATOMIC_SEQ_CST);
        frame_of_[p] = staged_frame_;
        memcpy(ov_params_host_[p], ov_pending_, sizeof(ov_pending_));   // read by this frame's graph
        if (!staged_on_main_) HIPCHECK(hipStreamWaitEvent(stream_, ev_copy_[p], 0));
        HIPCHECK(hipEventRecord(ev_[3 * p + 1], stream_));
        // convert/damage -> plan -> ME -> code -> CAVLC -> assembly -> commit: one graph,
        // one sync; k_decide leaves the final slice decisions in h_tasks_[p].
        // MV field / reference update and K7 deblocking run after the packets are done:
        // the host only waits for ev_[3p+2]; the next frame's work queues behind the update.
        // (An event record captured inside one fused graph did not order the host wait
        // after part 0 on ROCm 7: packets read back empty. Two launches it is.)
        run_graph(graph_exec_[p], 0);
        HIPCHECK(hipEventRecord(ev_[3 * p + 2], stream_));
        run_graph(post_exec_[p], 1);
        staged_ = false;
        launched_++;
        parity_ = launched_ & 1;
        return 0;
    }

    // Oldest frame in flight: wait for its packets. Up to two frames may be in flight
    // (launch(n+1) before finish(n)): the GPU then runs frame n+1's graph while the
    // host assembles frame n's packets, with no idle gap between the two graphs.
    int finish() override {
        if (inflight() <= 0) {
            set_last_error("finish() without a launched frame");
            return -1;
        }
        const int p = finished_ & 1;
        {
            trace::Range r("h264.wait");
            HIPCHECK(hipEventSynchronize(ev_[3 * p + 2]));
        }
        {
            trace::Range r("h264.packets");
            packets_.clear();
            build_packets(p, frame_of_[p]);
        }
        finished_++;
        float t0 = 0, t1 = 0;
        hipEventElapsedTime(&t0, ev_[3 * p], ev_[3 * p + 1]);
        hipEventElapsedTime(&t1, ev_[3 * p + 1], ev_[3 * p + 2]);
        stage_ms_[0] = t0;
        stage_ms_[1] = t1;
        return (int)packets_.size();
    }

    int64_t state_bytes() override { return (int64_t)h264::state_bytes(g_); }

    // Copies `n` bytes between this encoder's device buffer and a caller buffer
    // that is device (on_device) or host memory.
    void xfer(void* dst, const void* src, size_t n, bool to_caller, int on_device) {
        const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice
                                          : (to_caller ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice);
        HIPCHECK(hipMemcpyAsync(dst, src, n, k, stream_));
    }

    int export_state(void* dst, int on_device) override {
        HIPCHECK(hipSetDevice(device_));
        HIPCHECK(hipStreamSynchronize(stream_));
        const int ns = g_.num_slices;
        int ctl[4];
        std::vector<StripeState> st(ns + 1);
        std::vector<SliceTask> tasks(ns);
        copy_now(ctl, args_.plan_ctl, sizeof(ctl));
        copy_now(st.data(), args_.plan_state, sizeof(StripeState) * (ns + 1));
        copy_now(tasks.data(), args_.tasks, sizeof(SliceTask) * ns);
        if (ctl[1] == 1) {   // apply the commit k_plan would run at the next frame
            if (cfg_.fullframe) {
                bool idr = ns > 0;
                for (int s = 0; s < ns; s++) idr &= tasks[s].final_action == ACT_I && tasks[s].idr_on_intra;
                commit_picture(st[ns], idr, cfg_.num_refs > 1 ? 2 : 1);
            } else {
                for (int s = 0; s < ns; s++) commit_stripe(st[s], tasks[s].final_action, cfg_.num_refs > 1 ? 2 : 1);
            }
        }
        const int qp = h_key_seq_[1] > 0 ? h_key_seq_[1] : cfg_.qp;
        const int pqp = h_key_seq_[2] > 0 ? h_key_seq_[2] : cfg_.paint_qp;
        std::vector<uint8_t> head(state_head_bytes(g_));
        StateHeader h;
        state_header(cfg_, g_, ctl[1] != 0, qp, pqp, h);
        memcpy(head.data(), &h, sizeof(h));
        memcpy(head.data() + sizeof(h), st.data(), sizeof(StripeState) * (ns + 1));
        copy_now(head.data() + sizeof(h) + sizeof(StripeState) * (ns + 1), args_.rc, sizeof(RcState));   // K10
        uint8_t* o = static_cast<uint8_t*>(dst);
        if (on_device) HIPCHECK(hipMemcpyAsync(o, head.data(), head.size(), hipMemcpyHostToDevice, stream_));
        else memcpy(o, head.data(), head.size());
        o += head.size();
        const size_t ny = (size_t)g_.stride_y * g_.plane_h_y, nc = (size_t)g_.stride_c * g_.plane_h_c;
        const gpu::Planes& last_src = planes_src_[parity_ ^ 1];
        for (const gpu::Planes* pl : {(const gpu::Planes*)&args_.ref, (const gpu::Planes*)&args_.ref1, &last_src}) {
            xfer(o, pl->y, ny, true, on_device); o += ny;
            xfer(o, pl->u, nc, true, on_device); o += nc;
            xfer(o, pl->v, nc, true, on_device); o += nc;
        }
        xfer(o, args_.mvfield, sizeof(int16_t) * 2 * (size_t)g_.num_mbs(), true, on_device);
        HIPCHECK(hipStreamSynchronize(stream_));
        return 0;
    }

    int import_state(const void* src, int on_device) override {
        HIPCHECK(hipSetDevice(device_));
        HIPCHECK(hipStreamSynchronize(stream_));
        const int ns = g_.num_slices;
        std::vector<uint8_t> head(state_head_bytes(g_));
        const uint8_t* i = static_cast<const uint8_t*>(src);
        if (on_device) copy_now(head.data(), i, head.size());
        else memcpy(head.data(), i, head.size());
        StateHeader h;
        memcpy(&h, head.data(), sizeof(h));
        if (!state_header_matches(cfg_, g_, h)) {
            set_last_error("encoder state does not match this encoder's geometry / codec");
            return -1;
        }
        xfer(args_.plan_state, i + sizeof(StateHeader), sizeof(StripeState) * (ns + 1), false, on_device);
        {   // K10 state; its set_rate() counter is this encoder's, so k_rc_qp keeps it
            RcState rc;
            memcpy(&rc, head.data() + sizeof(StateHeader) + sizeof(StripeState) * (ns + 1), sizeof(rc));
            rc.seq = __atomic_load_n(&h_key_seq_[5], __ATOMIC_SEQ_CST);
            HIPCHECK(hipMemcpyAsync(args_.rc, &rc, sizeof(rc), hipMemcpyHostToDevice, stream_));
            HIPCHECK(hipStreamSynchronize(stream_));
        }
        i += head.size();
        const size_t ny = (size_t)g_.stride_y * g_.plane_h_y, nc = (size_t)g_.stride_c * g_.plane_h_c;
        const gpu::Planes& last_src = planes_src_[parity_ ^ 1];
        for (const gpu::Planes* pl : {(const gpu::Planes*)&args_.ref, (const gpu::Planes*)&args_.ref1, &last_src}) {
            xfer(pl->y, i, ny, false, on_device); i += ny;
            xfer(pl->u, i, nc, false, on_device); i += nc;
            xfer(pl->v, i, nc, false, on_device); i += nc;
        }
        xfer(args_.mvfield, i, sizeof(int16_t) * 2 * (size_t)g_.num_mbs(), false, on_device);
        // controller: committed state (2), and the host keyframe counter as already seen
        int ctl[2] = {__atomic_load_n(&h_key_seq_[0], __ATOMIC_SEQ_CST), h.started ? 2 : 0};
        HIPCHECK(hipMemcpyAsync(args_.plan_ctl, ctl, sizeof(ctl), hipMemcpyHostToDevice, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
        __atomic_store_n(&h_key_seq_[1], h.qp, __ATOMIC_SEQ_CST);
        __atomic_store_n(&h_key_seq_[2], h.paint_qp, __ATOMIC_SEQ_CST);
        return 0;
    }

    int stage_times(float* dst, int n) override {
        int k = n < 2 ? n : 2;
        for (int i = 0; i < k; i++) dst[i] = stage_ms_[i] * 1000.f;
        return k;
    }

    int set_overlay_image(int slot, const uint8_t* bgra, int w, int h) override {
        if (slot < 0 || slot >= kOverlaySlots || w < 0 || h < 0 || w > kOverlayMaxDim || h > kOverlayMaxDim) return -1;
        HIPCHECK(hipSetDevice(device_));
        const size_t n = (size_t)w * h * 4;
        if (!ov_stage_) ov_stage_ = hmalloc<uint8_t>((size_t)kOverlayMaxDim * kOverlayMaxDim * 4);
        HIPCHECK(hipStreamSynchronize(stream_));   // frames in flight may still read the old image
        if (n) {
            memcpy(ov_stage_, bgra, n);
            HIPCHECK(hipMemcpyAsync(ov_img_dev_[slot], ov_stage_, n, hipMemcpyHostToDevice, stream_));
            HIPCHECK(hipStreamSynchronize(stream_));
        }
        ov_pending_[slot].w = w;
        ov_pending_[slot].h = h;
        if (!n) ov_pending_[slot].on = 0;
        return 0;
    }
    int set_overlay_pos(int slot, int on, int x, int y, int tdx, int tdy) override {
        if (slot < 0 || slot >= kOverlaySlots) return -1;
        OverlayParams& o = ov_pending_[slot];
        o.on = on && o.w > 0 && o.h > 0;
        o.x = x;
        o.y = y;
        o.tdx = tdx > 0 ? tdx : 0;
        o.tdy = tdy > 0 ? tdy : 0;
        return 0;
    }

    int64_t debug_buffer(const char* name, void* dst, int64_t cap) override {
        HIPCHECK(hipSetDevice(device_));
        HIPCHECK(hipStreamSynchronize(stream_));
        std::string s(name);
        const void* p = nullptr;
        int64_t n = 0;
        size_t ny = (size_t)g_.stride_y * g_.plane_h_y, nc = (size_t)g_.stride_c * g_.plane_h_c;
        // after a frame the parity flipped: the last source is in `prev` of the next frame
        const gpu::Planes& last_src = parity_ ? planes_src_[0] : planes_src_[1];
        if (s == "src_y") { p = last_src.y; n = (int64_t)ny; }
        else if (s == "src_u") { p = last_src.u; n = (int64_t)nc; }
        else if (s == "src_v") { p = last_src.v; n = (int64_t)nc; }
        else if (s == "ref_y") { p = args_.ref.y; n = (int64_t)ny; }
        else if (s == "ref_u") { p = args_.ref.u; n = (int64_t)nc; }
        else if (s == "ref_v") { p = args_.ref.v; n = (int64_t)nc; }
        else if (s == "ref1_y") { p = args_.ref1.y; n = (int64_t)ny; }
        else if (s == "fs_mv") { p = args_.fs_mv; n = (int64_t)g_.num_mbs() * 4; }
        else if (s == "mbs") { p = args_.mbs; n = (int64_t)g_.num_mbs() * sizeof(MbInfo); }
        else if (s == "blk" && cfg_.codec == 2) { p = aargs_.blk; n = (int64_t)av1_geo_.c8 * av1_geo_.r8 * sizeof(av1::BlkInfo); }
        else if (s == "levels" && cfg_.codec == 2) { p = aargs_.lev; n = (int64_t)g_.num_mbs() * av1::gpu::kLevPerUnit * 2; }
        else if (s == "tok_n" && cfg_.codec == 2) { p = aargs_.tok_n; n = (int64_t)g_.num_mbs() * 4; }
        else if (s == "tokc" && cfg_.codec == 2) { p = aargs_.tokc; n = (int64_t)av1_geo_.tile_cols * av1_geo_.tile_rows * aargs_.tile_tok_cap * 4; }
        else if (s == "tile_ntok" && cfg_.codec == 2) { p = aargs_.tile_ntok; n = (int64_t)av1_geo_.tile_cols * av1_geo_.tile_rows * 4; }
        else if (s == "frame" && cfg_.codec == 2) { p = aargs_.frame; n = 16; }   // key, qidx, lf level, -
        else if (s == "tile_size" && cfg_.codec == 2) { p = aargs_.tile_size; n = (int64_t)av1_geo_.tile_cols * av1_geo_.tile_rows * 4; }
        else if (s == "av1_geo" && cfg_.codec == 2) {
            if (dst && cap >= (int64_t)sizeof(av1_geo_)) memcpy(dst, &av1_geo_, sizeof(av1_geo_));
            return (int64_t)sizeof(av1_geo_);
        }
        else if (s == "coefs" && cfg_.codec == 1) { p = hargs_.coefs; n = (int64_t)g_.num_mbs() * hevc::kCoefPerCu * 2; }
        else if (s == "cus" && cfg_.codec == 1) { p = hargs_.cus; n = (int64_t)g_.num_mbs() * sizeof(hevc::CuInfo); }
        else if (s == "sao" && cfg_.codec == 1) { p = hargs_.sao; n = (int64_t)hargs_.cw * hargs_.ch * sizeof(hevc::SaoParams); }
        else if (s == "bin_n" && cfg_.codec == 1) { p = hargs_.bin_n; n = (int64_t)g_.num_mbs() * 4; }
        else if (s == "cu_t" && cfg_.codec == 1) { p = hargs_.cu_t; n = (int64_t)g_.num_mbs() * 4; }
        else if (s == "cu_r" && cfg_.codec == 1) { p = hargs_.cu_r; n = (int64_t)g_.num_mbs() * 2; }
        else if (s == "tail" && cfg_.codec == 1) { p = hargs_.tail; n = (int64_t)g_.num_mbs() * 2; }
        else if (s == "sub" && cfg_.codec == 1) { p = hargs_.sub; n = (int64_t)hargs_.ch * hargs_.sub_stride; }
        else if (s == "sub_size" && cfg_.codec == 1) { p = hargs_.sub_size; n = (int64_t)hargs_.ch * hargs_.seg_k * 4; }
        else if (s == "row_bits" && cfg_.codec == 1) { p = hargs_.row_bits; n = (int64_t)hargs_.ch * hargs_.seg_k * 4; }
        else if (s == "hevc_stamps" && cfg_.codec == 1) { if (!hargs_.dbg) return -1; p = hargs_.dbg; n = (int64_t)hargs_.ch * 32; }
        else if (s == "coefs") { p = args_.coefs; n = (int64_t)g_.num_mbs() * kCoefPerMb * 2; }
        else if (s == "me") { p = args_.me; n = (int64_t)g_.num_mbs() * sizeof(MeResult); }
        else if (s == "mb_dirty") { p = args_.mb_dirty; n = g_.num_mbs(); }
        else if (s == "aq") { p = args_.aq; n = g_.num_mbs(); }
        else if (s == "stamps") { if (!args_.dbg) return -1; p = args_.dbg; n = (64 * 16 + 256) * 8; }
        else if (s == "tasks") {
            n = (int64_t)g_.num_slices * sizeof(SliceTask);
            if (dst && cap >= n) memcpy(dst, h_tasks_[(finished_ + 1) & 1], (size_t)n);   // last finished
            return n;
        } else return -1;
        if (dst && cap >= n) HIPCHECK(hipMemcpyAsync(dst, p, (size_t)n, hipMemcpyDeviceToHost, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
        return n;
    }

   private:
    template <class T>
    T* dmalloc(size_t count, bool zero = true) {
        void* p = nullptr;
        HIPCHECK(hipMalloc(&p, count * sizeof(T)));
        if (zero) HIPCHECK(hipMemsetAsync(p, 0, count * sizeof(T), stream_));
        dev_allocs_.push_back(p);
        return (T*)p;
    }
    template <class T>
    T* hmalloc(size_t count, unsigned flags = hipHostMallocDefault) {
        void* p = nullptr;
        HIPCHECK(hipHostMalloc(&p, count * sizeof(T), flags));
        memset(p, 0, count * sizeof(T));
        host_allocs_.push_back(p);
        return (T*)p;
    }

    gpu::Planes make_planes() {
        size_t ny = (size_t)g_.stride_y * g_.plane_h_y, nc = (size_t)g_.stride_c * g_.plane_h_c;
        gpu::Planes p;
        p.y = dmalloc<uint8_t>(ny);
        p.u = dmalloc<uint8_t>(nc);
        p.v = dmalloc<uint8_t>(nc);
        return p;
    }

    void alloc() {
        const int nmb = g_.num_mbs(), ns = g_.num_slices;
        planes_src_[0] = make_planes();
        planes_src_[1] = make_planes();
        gpu::FrameArgs& a = args_;
        memset(&a, 0, sizeof(a));
        a.W = g_.W; a.H = g_.H; a.mb_w = g_.mb_w; a.mb_h = g_.mb_h;
        a.stride_y = g_.stride_y; a.stride_c = g_.stride_c;
        a.num_slices = ns; a.rows_per_slice = g_.rows_per_slice; a.fullframe = cfg_.fullframe;
        a.full_range = cfg_.full_range; a.me_range = cfg_.me_range; a.me_iters = cfg_.me_iters;
        a.deblock = cfg_.codec == 0 ? cfg_.deblock : 0;   // HEVC / AV1 filter in their own back ends
        a.me_full = cfg_.me_full;
        a.aq_strength = cfg_.codec == 1 ? 0 : cfg_.aq_strength;
        a.subpel = cfg_.codec == 2 ? 0 : cfg_.subpel;   // AV1 keeps integer vectors (av1_encoder.h front_config)
        a.intra4x4 = cfg_.codec == 1 ? 0 : cfg_.intra4x4;
        a.aq = dmalloc<int8_t>(nmb);
        for (int k = 0; k < kOverlaySlots; k++) {
            ov_img_dev_[k] = dmalloc<uint8_t>((size_t)kOverlayMaxDim * kOverlayMaxDim * 4);
            a.ov_img[k] = ov_img_dev_[k];
            ov_params_host_[k] = hmalloc<OverlayParams>(kOverlaySlots);   // [parity][slot]
        }
        ov_params_dev_ = dmalloc<OverlayParams>(kOverlaySlots);
        a.ov = ov_params_dev_;
        memset(ov_pending_, 0, sizeof(ov_pending_));
        a.num_refs = cfg_.num_refs > 1 ? 2 : 1;
        a.scaled = (cfg_.src_width > 0 && cfg_.src_width != cfg_.width) ||
                   (cfg_.src_height > 0 && cfg_.src_height != cfg_.height);
        if (a.scaled)
            a.scale = scale_params(cfg_.src_width > 0 ? cfg_.src_width : cfg_.width,
                                   cfg_.src_height > 0 ? cfg_.src_height : cfg_.height, cfg_.width, cfg_.height);
        a.ref = make_planes();
        a.ref1 = make_planes();
        a.rec = make_planes();
        a.mb_dirty = dmalloc<uint8_t>(nmb);
        void* dd = nullptr;
        a.stripe_dirty = dmalloc<int>(ns);
        a.plan_ctl = dmalloc<int>(4);
        a.plan_cfg = plan_config(cfg_);
        {
            std::vector<StripeState> init(ns + 1);  // need_idr on every stripe and the picture
            a.plan_state = dmalloc<StripeState>(ns + 1);
            HIPCHECK(hipMemcpyAsync(a.plan_state, init.data(), sizeof(StripeState) * (ns + 1),
                                    hipMemcpyHostToDevice, stream_));
            HIPCHECK(hipStreamSynchronize(stream_));
        }
        h_key_seq_ = hmalloc<int>(16, hipHostMallocCoherent);   // written by request_keyframe/set_qp
        for (int p = 0; p < 2; p++) {   // per-parity snapshot taken at launch, read by k_plan
            h_key_snap_[p] = hmalloc<int>(8, hipHostMallocCoherent);
            HIPCHECK(hipHostGetDevicePointer(&dd, h_key_snap_[p], 0));
            key_snap_dev_[p] = (const int*)dd;
        }
        a.key_seq_host = key_snap_dev_[0];
        a.key_dev = dmalloc<int>(8);
        a.tasks = dmalloc<SliceTask>(ns);
        a.me = dmalloc<MeResult>(nmb);
        a.mvfield = dmalloc<int16_t>(2 * nmb);
        a.fs_mv = dmalloc<int16_t>(2 * nmb);
        {   // K10 rate control state (ratecontrol.h), initialised like the CPU controller's
            RcState rc;
            rc_init(rc, cfg_.rc_mode, cfg_.qp, cfg_.bitrate_kbps, cfg_.fps, cfg_.width * cfg_.height, cfg_.vbv_ms, cfg_.codec);
            a.rc = dmalloc<RcState>(1);
            copy_now(a.rc, &rc, sizeof(rc));
            a.rc_slice = dmalloc<long long>(2 * (size_t)ns);
            a.rc_redo = dmalloc<int>(1);
            a.gate = nullptr;
            a.rc_fps = cfg_.fps;
            h_key_seq_[3] = cfg_.rc_mode;
            h_key_seq_[4] = cfg_.bitrate_kbps;
        }
        a.db = dmalloc<DbInfo>(nmb);
        a.dbe = dmalloc<uint4>((size_t)3 * nmb);
        a.mbs = dmalloc<MbInfo>(nmb);
        a.coefs = dmalloc<int16_t>((size_t)nmb * kCoefPerMb);
        a.mb_bits = dmalloc<uint32_t>((size_t)nmb * (gpu::kMbSlotBytes / 4));
        a.mb_nbits = dmalloc<int>(nmb);
        int max_slice_mbs = g_.rows_per_slice * g_.mb_w;
        // K5: split I slices put one NAL per sub-slice (h264_encoder.h intra_split)
        const bool can_split = cfg_.codec == 0 && g_.mb_w > kIntraSubMbs;
        a.nal_per_slice = can_split ? max_nals_per_slice(g_.rows_per_slice, g_.mb_w) : 1;
        a.sub_rbsp_words = (kIntraSubMbs * gpu::kMbSlotBytes + 1024) / 4;
        a.rbsp_slot_words = std::max((max_slice_mbs * gpu::kMbSlotBytes + 1024) / 4,
                                     can_split ? a.nal_per_slice * a.sub_rbsp_words : 0);
        a.rbsp = dmalloc<uint32_t>((size_t)ns * a.rbsp_slot_words);
        a.mb_off = dmalloc<int>(nmb);
        a.slice_info = dmalloc<int>(4 * (size_t)ns * a.nal_per_slice);
        a.max_tiles = (a.rbsp_slot_words * 4 + 4095) / 4096;
        a.tile_nz = dmalloc<int>((size_t)ns * a.nal_per_slice * a.max_tiles);
        a.tile_ins = dmalloc<int>((size_t)ns * a.nal_per_slice * a.max_tiles);
        // worst case: header + SPS/PPS + 3/2 emulation-prevention growth, 64-byte multiple
        size_t slot = ((size_t)a.rbsp_slot_words * 4 * 3 / 2 + 1024 + 63) & ~(size_t)63;
        a.out_slot_bytes = (int)slot;
        void* dptr = nullptr;
        for (int p = 0; p < 2; p++) {   // host outputs per parity (two frames in flight)
            host_out_[p] = hmalloc<uint8_t>(slot * ns);
            h_out_size_[p] = hmalloc<int>(ns);
            HIPCHECK(hipHostGetDevicePointer(&dptr, host_out_[p], 0));
            host_out_dev_[p] = (uint8_t*)dptr;
            HIPCHECK(hipHostGetDevicePointer(&dptr, h_out_size_[p], 0));
            host_size_dev_[p] = (int*)dptr;
        }
        // parameter sets
        std::vector<std::vector<uint8_t>> ps;
        if (cfg_.fullframe) {
            ps.resize(1);
            build_parameter_sets(g_.W, g_.H, cfg_.full_range, cfg_.fps, ps[0], cfg_.num_refs);
        } else {
            ps.resize(ns);
            for (int s = 0; s < ns; s++) build_parameter_sets(g_.W, g_.slice_pix_h(s), cfg_.full_range, cfg_.fps, ps[s], cfg_.num_refs);
        }
        param_sets_ = ps;
        a.param_set_stride = 256;
        std::vector<uint8_t> flat((size_t)ns * 256, 0);
        std::vector<int> lens(ns, 0);
        for (int s = 0; s < ns; s++) {
            const std::vector<uint8_t>& v = ps[cfg_.fullframe ? 0 : s];
            if (v.size() > 256) throw std::runtime_error("parameter sets too large");
            memcpy(&flat[(size_t)s * 256], v.data(), v.size());
            lens[s] = (int)v.size();
        }
        uint8_t* dps = dmalloc<uint8_t>(flat.size());
        HIPCHECK(hipMemcpyAsync(dps, flat.data(), flat.size(), hipMemcpyHostToDevice, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
        int* dlen = dmalloc<int>(ns);
        HIPCHECK(hipMemcpyAsync(dlen, lens.data(), sizeof(int) * ns, hipMemcpyHostToDevice, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
        a.param_sets = dps;
        a.param_set_len = dlen;
        CavlcTables* ct = dmalloc<CavlcTables>(1);
        HIPCHECK(hipMemcpyAsync(ct, &host_cavlc_tables(), sizeof(CavlcTables), hipMemcpyHostToDevice, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
        a.cavlc_tabs = ct;
        d_frame_params_ = dmalloc<int>(4);
        if (getenv("SK_STAMPS")) a.dbg = dmalloc<unsigned long long>(64 * 16 + 256);
        a.frame_params_dev = d_frame_params_;
        for (int p = 0; p < 2; p++) {
            h_tasks_[p] = hmalloc<SliceTask>(ns, hipHostMallocCoherent);  // final decisions from k_decide
            HIPCHECK(hipHostGetDevicePointer(&dd, h_tasks_[p], 0));
            tasks_host_dev_[p] = (SliceTask*)dd;
            h_frame_params_[p] = hmalloc<int>(4, hipHostMallocCoherent);
            HIPCHECK(hipHostGetDevicePointer(&dd, h_frame_params_[p], 0));
            frame_params_dev_host_[p] = (const int*)dd;
        }
    }

    void set_parity_args(int stride) {
        args_.yuv = yuv_dev_[parity_];
        args_.yuv_fmt = yuv_mode_;
        args_.bgrx = bgrx_dev_[parity_];
        args_.bgrx_stride = stride;
        args_.src = planes_src_[parity_];
        args_.prev = planes_src_[parity_ ^ 1];
        args_.host_out = host_out_dev_[parity_];
        args_.host_size = host_size_dev_[parity_];
        args_.tasks_host = tasks_host_dev_[parity_];
        args_.frame_params_host = frame_params_dev_host_[parity_];
        args_.key_seq_host = key_snap_dev_[parity_];
    }

    void invalidate_graphs() {
        for (auto* set : {graph_exec_, post_exec_})
            for (int i = 0; i < 2; i++)
                if (set[i]) { hipGraphExecDestroy(set[i]); set[i] = nullptr; }
    }

    // part 0: convert/damage -> ... -> packets; part 1: commit (+ deblocking).
    // rbsp is self-cleaning (k_ep_write); stripe flags are cleared by k_plan.
    void enqueue(int part) {
        if (part == 0) {
            // this frame's overlay placement (host copy written at launch()) -> device
            HIPCHECK(hipMemcpyAsync(ov_params_dev_, ov_params_host_[parity_], sizeof(OverlayParams) * kOverlaySlots,
                                    hipMemcpyHostToDevice, stream_));
            gpu::launch_convert_damage(args_, stream_);
            if (cfg_.codec == 2) {
                gpu::launch_frontend(args_, stream_);
                av1::gpu::Av1Args aa = aargs_;
                aa.f = args_;
                aa.frame_host = av1_frame_dev_[parity_];
                aa.out_host = av1_out_dev_[parity_];
                aa.out_size_host = av1_size_dev_[parity_];
                av1::gpu::launch_backend(aa, stream_, graph_guard_ ? args_.rc_redo : nullptr);
                gpu::launch_rc_account(args_, aa.tile_size, av1_geo_.tile_cols * av1_geo_.tile_rows, 1, 0, stream_);
            } else if (cfg_.codec == 1) {
                gpu::launch_frontend(args_, stream_);
                hevc::gpu::HevcArgs ha = hargs_;
                ha.f = args_;
                ha.out_host = hevc_out_dev_[parity_];
                ha.out_size = hevc_size_dev_[parity_];
                ha.out_dev = hevc_fallback_[parity_];
                hevc::gpu::launch_backend(ha, stream_, graph_guard_ ? args_.rc_redo : nullptr);
                gpu::launch_rc_account(args_, ha.sub_size, ha.ch * ha.seg_k, 1, 0, stream_);
            } else {
                gpu::launch_encode(args_, stream_, graph_guard_);
            }
        } else {
            gpu::launch_commit(args_, stream_);
        }
    }

    void run_graph(hipGraphExec_t& gx, int part) {
        if (!use_graphs_) {
            enqueue(part);
            return;
        }
        if (!gx) {
            hipGraph_t graph;
            HIPCHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeRelaxed));
            enqueue(part);
            HIPCHECK(hipStreamEndCapture(stream_, &graph));
            HIPCHECK(hipGraphInstantiate(&gx, graph, nullptr, nullptr, 0));
            hipGraphDestroy(graph);
        }
        HIPCHECK(hipGraphLaunch(gx, stream_));
    }

    // HEVC back-end buffers (hevc_gpu.h): CU decisions, levels, bin slots, WPP states,
    // one substream slot per CTB row, host-mapped slice slots + device fallback.
    void alloc_hevc() {
        const int n = g_.num_mbs(), ns = g_.num_slices;
        hevc::Geo geo;
        geo.init(g_);
        hevc::gpu::HevcArgs& h = hargs_;
        memset(&h, 0, sizeof(h));
        h.cw = geo.ctb_w;
        h.ch = geo.ctb_h;
        h.rps = geo.rows_per_slice;
        if (g_.rows_per_slice & 1) throw std::runtime_error("HEVC: stripes must be whole CTB rows");
        const int nc = geo.ctbs();
        h.cus = dmalloc<hevc::CuInfo>(n);
        h.coefs = dmalloc<int16_t>((size_t)n * hevc::kCoefPerCu);
        h.bins = dmalloc<uint16_t>((size_t)n * hevc::kCuBinCap, false);
        h.bin_n = dmalloc<int>(n);
        // intra slices: seg_k slices per CTB row (hevc_core.h SliceMap); per-substream
        // arrays hold ch * seg_k slots
        h.seg_k = hevc::intra_seg_k(h.cw, h.ch);
        if (h.rps * h.seg_k > 256) throw std::runtime_error("HEVC: more than 256 row segments per slice");
        const size_t slots = (size_t)h.ch * h.seg_k;
        h.sync = dmalloc<uint8_t>(slots * hevc::CTX_COUNT);
        h.sub_stride = h.cw * 4 * hevc::kSubstreamCtbBytes + 64 * h.seg_k + 64;
        h.sub = dmalloc<uint8_t>((size_t)h.ch * h.sub_stride, false);
        h.sub_size = dmalloc<int>(slots);
        h.sub_esc = dmalloc<int>(slots);
        h.row_off = dmalloc<int>(slots);
        h.addr_bits = geo.addr_bits;
        if (2 * g_.mb_w > 1024) throw std::runtime_error("HEVC: more than 1024 units per CTB row (8K) is not supported");
        h.srt = dmalloc<uint16_t>((size_t)n * hevc::kCuBinCap, false);
        h.coff = dmalloc<uint16_t>((size_t)h.ch * hevc::kPcCtxOff * 2 * g_.mb_w, false);
        h.rmap = dmalloc<uint32_t>((size_t)n * 256, false);
        h.cu_t = dmalloc<uint32_t>(n);
        h.cu_r = dmalloc<uint16_t>(n);
        h.tail = dmalloc<uint8_t>((size_t)n * 2);
        h.row_bits = dmalloc<uint32_t>(slots);
        h.sao_stats = dmalloc<hevc::SaoStats>((size_t)3 * nc, false);
        h.sao_own = dmalloc<hevc::SaoParams>(nc);
        h.sao_cost = dmalloc<long long>(nc);
        h.sao_md = dmalloc<long long>((size_t)nc * hevc::kSaoMd);
        h.sao = dmalloc<hevc::SaoParams>(nc);
        h.sao_tmp.y = dmalloc<uint8_t>((size_t)g_.stride_y * g_.mb_h * 16, false);
        h.sao_tmp.u = dmalloc<uint8_t>((size_t)g_.stride_c * g_.mb_h * 8, false);
        h.sao_tmp.v = dmalloc<uint8_t>((size_t)g_.stride_c * g_.mb_h * 8, false);
        // host slot: 1.5 KB per CTB (far above practical rates); larger slices go to the
        // device fallback slot (worst case: 3/2 emulation growth of the substream bound)
        h.out_slot = (g_.rows_per_slice * g_.mb_w * 1536 + 4096 + 63) & ~63;
        h.out_dev_slot = (int)(((size_t)h.rps * h.sub_stride * 3 / 2 + 4096 + 63) & ~(size_t)63);
        void* dptr = nullptr;
        for (int p = 0; p < 2; p++) {
            hevc_out_[p] = hmalloc<uint8_t>((size_t)h.out_slot * ns);
            hevc_size_[p] = hmalloc<int>(ns, hipHostMallocCoherent);
            HIPCHECK(hipHostGetDevicePointer(&dptr, hevc_out_[p], 0));
            hevc_out_dev_[p] = (uint8_t*)dptr;
            HIPCHECK(hipHostGetDevicePointer(&dptr, hevc_size_[p], 0));
            hevc_size_dev_[p] = (int*)dptr;
            hevc_fallback_[p] = dmalloc<uint8_t>((size_t)h.out_dev_slot * ns, false);
        }
        HIPCHECK(hipStreamSynchronize(stream_));
        if (getenv("SK_STAMPS")) h.dbg = dmalloc<unsigned long long>((size_t)4 * h.ch);
        h.reg_steps = getenv("SK_HEVC_REG_STEPS") ? atoi(getenv("SK_HEVC_REG_STEPS")) : 1;
        h.pc_seg = getenv("SK_HEVC_PC_SEG") ? sk_max(atoi(getenv("SK_HEVC_PC_SEG")), 1) : 32;
        hevc_params_.clear();
        hevc::build_parameter_sets(g_.W, g_.H, cfg_.full_range, cfg_.fps, hevc_params_);
    }

    // AV1 back-end buffers (av1_gpu.h): cells, levels, level contexts, token slots per
    // 16x16 unit, block-parallel coder state per tile, host-mapped frame info and tile bytes.
    void alloc_av1() {
        const int n = g_.num_mbs();
        av1::gpu::Av1Args& a = aargs_;
        memset(&a, 0, sizeof(a));
        const int sbc = (g_.W + 63) / 64, sbr = (g_.H + 63) / 64;
        int ac, ar;
        av1::auto_tiles(sbc, sbr, &ac, &ar);
        const int tc = cfg_.tile_cols_log2 >= 0 ? cfg_.tile_cols_log2 : ac;
        const int tr = cfg_.tile_rows_log2 >= 0 ? cfg_.tile_rows_log2 : ar;
        av1::geo_init(av1_geo_, g_.W, g_.H, tc, tr);
        a.geo = av1_geo_;
        a.blk = dmalloc<av1::BlkInfo>((size_t)av1_geo_.c8 * av1_geo_.r8);
        a.pal = dmalloc<uint8_t>((size_t)av1_geo_.c8 * av1_geo_.r8 * 8);
        a.palette = av1::palette_enabled() ? 1 : 0;
        a.pal_rate = dmalloc<int>((size_t)av1_geo_.c8 * av1_geo_.r8);
        a.lev = dmalloc<int16_t>((size_t)n * av1::gpu::kLevPerUnit);
        a.lctx_w[0] = av1_geo_.mi_cols;
        a.lctx_w[1] = a.lctx_w[2] = av1_geo_.mi_cols >> 1;
        a.lctx[0] = dmalloc<uint8_t>((size_t)av1_geo_.mi_cols * av1_geo_.mi_rows);
        a.lctx[1] = dmalloc<uint8_t>((size_t)(av1_geo_.mi_cols >> 1) * (av1_geo_.mi_rows >> 1));
        a.lctx[2] = dmalloc<uint8_t>((size_t)(av1_geo_.mi_cols >> 1) * (av1_geo_.mi_rows >> 1));
        a.tok = dmalloc<uint32_t>((size_t)n * av1::gpu::kTokCap, false);
        a.tok_n = dmalloc<int>(n);
        a.frame = dmalloc<int>(4);
        a.cdef_in.y = dmalloc<uint8_t>((size_t)g_.stride_y * g_.mb_h * 16, false);
        a.cdef_in.u = dmalloc<uint8_t>((size_t)g_.stride_c * g_.mb_h * 8, false);
        a.cdef_in.v = dmalloc<uint8_t>((size_t)g_.stride_c * g_.mb_h * 8, false);
        const int tiles = av1_geo_.tile_cols * av1_geo_.tile_rows;
        // tile bytes: 4 KB per unit of the largest tile (incompressible content codes
        // below ~1.5 bytes per sample)
        const int tile_units = (av1_geo_.tile_w_sb * 4) * (av1_geo_.tile_h_sb * 4);
        a.tile_tok_cap = tile_units * av1::gpu::kTokCap;
        a.tokc = dmalloc<uint32_t>((size_t)tiles * a.tile_tok_cap, false);
        // + per-wave junk slots of k_av1_cdf (words of tokens a wave does not own)
        a.pw = dmalloc<uint32_t>((size_t)tiles * a.tile_tok_cap + (size_t)tiles * 16 * 64, false);
        a.tok_off = dmalloc<int>(n);
        a.tile_ntok = dmalloc<int>(tiles);
        a.tile_cap = tile_units * 4096;
        if (tiles > 64) throw std::runtime_error("AV1: at most 64 tiles");
        av1::gpu::ec_buffers(tiles, a.tile_cap, &a.ec_max_blocks, &a.ec_vcap);
        a.ecmap = dmalloc<uint2>((size_t)a.ec_max_blocks * 128, false);
        a.ecblk = dmalloc<int4>((size_t)a.ec_max_blocks, false);
        a.ecv = dmalloc<unsigned long long>((size_t)tiles * a.ec_vcap, false);
        a.ecf = dmalloc<uint32_t>((size_t)tiles * a.ec_vcap, false);
        a.tile_bits = dmalloc<int>(tiles);
        a.tile_size = dmalloc<int>(tiles);
        a.out_cap = g_.W * g_.H * 3 + 4096;
        std::vector<uint8_t> q(52);
        for (int i = 0; i < 52; i++) q[i] = (uint8_t)av1::qidx_for_qp(i);
        uint8_t* dq = dmalloc<uint8_t>(52);
        copy_now(dq, q.data(), 52);
        a.qidx_of_qp = dq;
        void* dptr = nullptr;
        for (int p = 0; p < 2; p++) {
            av1_out_[p] = hmalloc<uint8_t>((size_t)a.out_cap);
            av1_size_[p] = hmalloc<int>(tiles, hipHostMallocCoherent);
            av1_frame_[p] = hmalloc<int>(4, hipHostMallocCoherent);
            HIPCHECK(hipHostGetDevicePointer(&dptr, av1_out_[p], 0));
            av1_out_dev_[p] = (uint8_t*)dptr;
            HIPCHECK(hipHostGetDevicePointer(&dptr, av1_size_[p], 0));
            av1_size_dev_[p] = (int*)dptr;
            HIPCHECK(hipHostGetDevicePointer(&dptr, av1_frame_[p], 0));
            av1_frame_dev_[p] = (int*)dptr;
        }
        HIPCHECK(hipStreamSynchronize(stream_));
        av1_level_ = av1::choose_level_idx(g_.W, g_.H, cfg_.fps);
    }

    void build_packets_av1(int par, uint16_t frame_id) {
        const int tiles = av1_geo_.tile_cols * av1_geo_.tile_rows;
        av1::FrameParams fp;
        fp.key = av1_frame_[par][0];
        fp.qidx = av1_frame_[par][1];
        fp.lf_level = av1_frame_[par][2];
        fp.screen = fp.key && aargs_.palette;
        std::vector<std::vector<uint8_t>> tl(tiles);
        size_t off = 0;
        for (int t = 0; t < tiles; t++) {
            const int n = av1_size_[par][t];
            if (n < 0) throw std::runtime_error("AV1 tile exceeded its output capacity");
            tl[t].assign(av1_out_[par] + off, av1_out_[par] + off + n);
            off += (size_t)n;
        }
        size_t maxsz = 1;
        for (int t = 0; t + 1 < tiles; t++) maxsz = std::max(maxsz, tl[t].size());
        fp.tile_size_bytes = maxsz <= 0x100 ? 1 : (maxsz <= 0x10000 ? 2 : (maxsz <= 0x1000000 ? 3 : 4));
        EncodedPacket pk;
        pk.y = 0; pk.w = g_.W; pk.h = g_.H; pk.key = fp.key;
        pk.data.resize(10);
        write_stripe_header(pk.data.data(), fp.key, frame_id, 0, g_.W, g_.H);
        av1::append_obu(pk.data, 2, nullptr, 0);
        if (fp.key) {
            av1::BitWriter sh;
            av1::write_sequence_header(sh, g_.W, g_.H, av1_level_, cfg_.full_range);
            av1::append_obu(pk.data, 1, sh.buf.data(), sh.buf.size());
        }
        av1::BitWriter fh;
        av1::write_frame_header(fh, av1_geo_, fp);
        std::vector<uint8_t> payload = fh.buf;
        if (tiles > 1) payload.push_back(0);
        for (int t = 0; t < tiles; t++) {
            if (t + 1 < tiles) {
                const uint32_t sz = (uint32_t)tl[t].size() - 1;
                for (int k = 0; k < fp.tile_size_bytes; k++) payload.push_back((uint8_t)(sz >> (8 * k)));
            }
            payload.insert(payload.end(), tl[t].begin(), tl[t].end());
        }
        av1::append_obu(pk.data, 6, payload.data(), payload.size());
        packets_.push_back(std::move(pk));
    }

    void build_packets_hevc(int par, uint16_t frame_id) {
        const SliceTask* h_tasks = h_tasks_[par];
        const int ns = g_.num_slices;
        const bool idr = ctl_.picture_is_idr(h_tasks);
        EncodedPacket pk;
        pk.y = 0; pk.w = g_.W; pk.h = g_.H; pk.key = idr;
        pk.data.resize(10);
        write_stripe_header(pk.data.data(), idr, frame_id, 0, g_.W, g_.H);
        if (idr) pk.data.insert(pk.data.end(), hevc_params_.begin(), hevc_params_.end());
        for (int s = 0; s < ns; s++) {
            const int n = hevc_size_[par][s];
            const size_t o = pk.data.size();
            pk.data.resize(o + (size_t)n);
            if (n <= hargs_.out_slot) {
                memcpy(pk.data.data() + o, hevc_out_[par] + (size_t)s * hargs_.out_slot, (size_t)n);
            } else {   // rare: the slice did not fit its host slot
                copy_now(pk.data.data() + o, hevc_fallback_[par] + (size_t)s * hargs_.out_dev_slot, (size_t)n);
            }
        }
        packets_.push_back(std::move(pk));
    }

    void build_packets(int par, uint16_t frame_id) {
        if (cfg_.codec == 2) {
            build_packets_av1(par, frame_id);
            return;
        }
        if (cfg_.codec == 1) {
            build_packets_hevc(par, frame_id);
            return;
        }
        const uint8_t* host_out = host_out_[par];
        const int* h_out_size = h_out_size_[par];
        const SliceTask* h_tasks = h_tasks_[par];
        const int ns = g_.num_slices;
        std::vector<long> offs(ns);
        for (int s = 0; s < ns; s++) offs[s] = (long)s * args_.out_slot_bytes;
        if (cfg_.fullframe) {
            bool idr = ctl_.picture_is_idr(h_tasks);
            EncodedPacket pk;
            pk.y = 0; pk.w = g_.W; pk.h = g_.H; pk.key = idr;
            pk.data.resize(10);
            write_stripe_header(pk.data.data(), idr, frame_id, 0, g_.W, g_.H);
            if (idr) pk.data.insert(pk.data.end(), param_sets_[0].begin(), param_sets_[0].end());
            for (int s = 0; s < ns; s++) {
                const uint8_t* p = host_out + offs[s];
                pk.data.insert(pk.data.end(), p, p + h_out_size[s]);
            }
            packets_.push_back(std::move(pk));
            return;
        }
        for (int s = 0; s < ns; s++) {
            if (h_tasks[s].final_action == ACT_NONE || h_out_size[s] <= 0) continue;
            EncodedPacket pk;
            pk.y = g_.slice_pix_y(s);
            pk.w = g_.W;
            pk.h = g_.slice_pix_h(s);
            pk.key = h_tasks[s].final_action == ACT_I;
            const uint8_t* p = host_out + offs[s];
            pk.data.assign(p, p + h_out_size[s]);
            packets_.push_back(std::move(pk));
        }
    }

    EncoderConfig cfg_;
    Geometry g_;
    Controller ctl_;
    int device_;
    hevc::gpu::HevcArgs hargs_;
    av1::gpu::Av1Args aargs_;
    av1::Av1Geo av1_geo_;
    int av1_level_ = 8;
    uint8_t* av1_out_[2] = {nullptr, nullptr};
    uint8_t* av1_out_dev_[2] = {nullptr, nullptr};
    int* av1_size_[2] = {nullptr, nullptr};
    int* av1_size_dev_[2] = {nullptr, nullptr};
    int* av1_frame_[2] = {nullptr, nullptr};
    int* av1_frame_dev_[2] = {nullptr, nullptr};
    uint8_t* hevc_out_[2] = {nullptr, nullptr};
    uint8_t* hevc_out_dev_[2] = {nullptr, nullptr};
    int* hevc_size_[2] = {nullptr, nullptr};
    int* hevc_size_dev_[2] = {nullptr, nullptr};
    uint8_t* hevc_fallback_[2] = {nullptr, nullptr};
    std::vector<uint8_t> hevc_params_;
    hipStream_t stream_ = nullptr;
    hipEvent_t ev_[6];   // per parity p: [3p] upload, [3p+1] graph start, [3p+2] packets done
    gpu::FrameArgs args_;
    gpu::Planes planes_src_[2];
    int parity_ = 0;
    uint8_t* bgrx_dev_[2] = {nullptr, nullptr};   // input frame per parity (upload overlaps the other)
    hipEvent_t ev_copy_[2];
    bool staged_ = false, staged_on_main_ = true;
    int launched_ = 0, finished_ = 0;   // frames launched / finished; frame k uses parity k & 1
    int inflight() const { return launched_ - finished_; }
    uint16_t frame_of_[2] = {0, 0};
    uint16_t staged_frame_ = 0;
    size_t bgrx_cap_ = 0;
    // damage-driven upload (set_upload_rows / upload_copy)
    bool up_valid_[2] = {false, false};      // bgrx_dev_[q] holds a complete frame
    bool up_next_known_ = false, up_prev_known_ = false;
    std::vector<int> up_next_, up_prev_;     // row ranges of this frame / the previous one
    std::atomic<long long> up_rows_copied_{0}, up_rows_total_{0};   // read by the stats thread
    uint8_t* host_out_[2] = {nullptr, nullptr};
    uint8_t* host_out_dev_[2] = {nullptr, nullptr};
    int* host_size_dev_[2] = {nullptr, nullptr};
    SliceTask* tasks_host_dev_[2] = {nullptr, nullptr};
    const int* frame_params_dev_host_[2] = {nullptr, nullptr};
    int* h_key_seq_ = nullptr;
    SliceTask* h_tasks_[2] = {nullptr, nullptr};
    int* h_out_size_[2] = {nullptr, nullptr};
    int* h_frame_params_[2] = {nullptr, nullptr};
    int* h_key_snap_[2] = {nullptr, nullptr};
    const int* key_snap_dev_[2] = {nullptr, nullptr};
    int* d_frame_params_ = nullptr;
    std::vector<std::vector<uint8_t>> param_sets_;
    std::vector<void*> dev_allocs_, host_allocs_;
    hipGraphExec_t graph_exec_[2] = {nullptr, nullptr};
    uint8_t* ov_img_dev_[kOverlaySlots] = {};
    OverlayParams* ov_params_dev_ = nullptr;
    OverlayParams* ov_params_host_[2] = {};   // per launch parity: copied into the graph
    OverlayParams ov_pending_[kOverlaySlots];
    uint8_t* ov_stage_ = nullptr;
    hipGraphExec_t post_exec_[2] = {nullptr, nullptr};
    bool use_graphs_ = getenv("SK_NO_GRAPHS") == nullptr;
    // Blocking copies are ordered on the encoder's own stream: a copy on the legacy
    // stream fails while any stream of the process is capturing a graph (several
    // sessions share one process in parallel/multi.py session hosts). No extra stream:
    // every stream takes a slot in the process's round-robin over its hardware queues,
    // and an idle one per session halved the queues the sessions' work spread over
    // (8 x 1080p: 4150 -> 3650 fps).
    void copy_now(void* dst, const void* src, size_t n) {
        HIPCHECK(hipMemcpyAsync(dst, src, n, hipMemcpyDefault, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
    }
    bool graph_guard_ = false;   // the captured H.264 graphs contain the K10 CBR guard
    uint8_t* yuv_dev_[2] = {nullptr, nullptr};   // planar input staging per parity (upload_yuv)
    int yuv_mode_ = 0;                           // YuvFormat of the captured graphs (0: BGRx)
    hipEvent_t ev_ext_ = nullptr;   // wait_stream(): foreign stream's work before the next upload
    bool ext_wait_ = false;
    hipStream_t copy_stream_ = nullptr;   // shared per device (not owned)
    hipStream_t up_stream_ = nullptr;     // this session's upload stream (owned, lazily created)
    // 0: on the session stream (behind the frame in flight), 1: own upload stream,
    // 2: the device's shared copy stream
    int upload_mode_ = getenv("SK_UPLOAD_MODE") ? atoi(getenv("SK_UPLOAD_MODE")) : 2;
    hipStream_t upload_stream() {
        if (!up_stream_) HIPCHECK(hipStreamCreateWithFlags(&up_stream_, hipStreamNonBlocking));
        return up_stream_;
    }

    // One H2D stream per device for encoders created with shared_copy: lives as long
    // as the process (encoders come and go, the stream is reused).
    static hipStream_t device_copy_stream(int device) {
        static std::mutex mu;
        static std::map<int, hipStream_t> streams;
        std::lock_guard<std::mutex> lk(mu);
        auto it = streams.find(device);
        if (it != streams.end()) return it->second;
        hipStream_t s = nullptr;
        HIPCHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        streams[device] = s;
        return s;
    }
    float stage_ms_[4] = {0, 0, 0, 0};
};

}  // namespace

// A fresh process pays a one-time cost when several threads queue SDMA copies behind
// kernels on their streams: during the first ~50 such copies hipMemcpyAsync blocks
// the calling thread, and every other copying thread with it, for 6-9 ms while the
// GPU idles (rocprofv3 --hip-runtime-trace of the 8-session bench: all capture
// threads inside hipMemcpyAsync at once, four times within the first ~40 frames;
// tools/microbench/h2d_stall.cpp reproduces it with 8 threads x (copy + 12 small
// kernels): 46 stalled calls; 0 with HSA_ENABLE_SDMA=0, with copies on kernel-free
// streams, or after this warm-up; profiles/r2_driver_window.md). Whatever the
// runtime grows in that phase is per process, not per stream: the same pattern run
// here from 8 threads on streams of their own, destroyed afterwards, leaves the
// sessions' own streams stall-free. Serving would otherwise pay it inside the first
// second of the first sessions. SK_COPY_WARMUP=0 skips it.
void warm_copy_engines(int device) {
    static std::mutex mu;
    static std::map<int, bool> done;
    std::lock_guard<std::mutex> lk(mu);
    if (done[device]) return;
    done[device] = true;
    const char* env = getenv("SK_COPY_WARMUP");
    if (env && atoi(env) == 0) return;
    const int kThreads = 8, kRounds = 60, kKernels = 12;
    const size_t bytes = (size_t)8 << 20;
    uint8_t* host = nullptr;
    if (hipHostMalloc((void**)&host, bytes, hipHostMallocDefault) != hipSuccess) return;
    for (size_t i = 0; i < bytes; i += 4096) host[i] = 0;
    std::vector<std::thread> th;
    for (int t = 0; t < kThreads; t++)
        th.emplace_back([=] {
            if (hipSetDevice(device) != hipSuccess) return;
            hipStream_t s = nullptr;
            uint8_t* dev = nullptr;
            if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
            if (hipMalloc((void**)&dev, bytes) == hipSuccess) {
                for (int r = 0; r < kRounds; r++) {
                    if (hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s) != hipSuccess) break;
                    for (int k = 0; k < kKernels; k++) launch_touch_pages(dev, 2000, s);
                    if (hipStreamSynchronize(s) != hipSuccess) break;
                }
                hipFree(dev);
            }
            hipStreamDestroy(s);
        });
    for (auto& x : th) x.join();
    hipHostFree(host);
}

EncoderBackend* create_hip_backend(const h264::EncoderConfig& c, int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device)
        throw std::runtime_error("no HIP device available for the gfx950 backend");
    return new HipBackend(c, device);
}

}  // namespace sk
