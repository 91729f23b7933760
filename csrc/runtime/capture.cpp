// Capture session behind the pixelflux-compatible Python API
// (pixelflux/__init__.py): a native thread paced at target_fps grabs the region
// (X11 MIT-SHM or the synthetic desktop), encodes it with the HIP (or CPU
// reference) stripe encoder and hands every stripe packet to a C callback, the
// contract the reference server relies on (selkies.py:2846-2917:
// ScreenCapture.start_capture(settings, StripeCallback(cb)), result.data/.size/
// .frame_id).
#include "sk_api.h"
#include "encoder_iface.h"
#include "trace.h"
#include "../capture/frame_source.h"
#include <atomic>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <chrono>
#include <mutex>
#include <stdio.h>
#include <string.h>
#include <string>
#include <thread>
#include <algorithm>
#include <vector>


namespace sk {

// Sessions currently running per GPU (adjusted by `delta`; returns the new count).
static int device_sessions(int device, int delta) {
    static std::mutex mu;
    static std::map<int, int> count;
    std::lock_guard<std::mutex> g(mu);
    int& c = count[device];
    c += delta;
    return c;
}

class CaptureSession {
   public:
    ~CaptureSession() { stop(); }

    int start(const sk_capture_settings& s, sk_stripe_cb cb, void* user) {
        stop();
        s_ = s;
        display_ = s.display ? s.display : "";
        s_.display = nullptr;
        cb_ = cb;
        user_ = user;
        std::string err;
        const int w = s.capture_width, h = s.capture_height;
        if (w < 16 || h < 16) {
            set_last_error("capture size too small");
            return -1;
        }
        // frame source
        if (s.source <= 0) {
            const char* disp = display_.empty() ? getenv("DISPLAY") : display_.c_str();
            if (disp && *disp) src_ = make_x11_source(disp, s.capture_x, s.capture_y, w, h, s.capture_cursor != 0, &err);
            if (!src_ && s.source == 0) {
                set_last_error("X11 capture unavailable: " + err);
                return -1;
            }
        }
        pool_ = nullptr;
        if (s.source == 4) {   // caller-owned frame pool (benchmarks / replay)
            if (!s.pool || s.pool_frames < 1) {
                set_last_error("pool source needs pool and pool_frames");
                return -1;
            }
            pool_ = s.pool;
            src_ = make_pool_source(s.pool, s.pool_frames, s.pool_stride > 0 ? s.pool_stride : w * 4, h, s.pool_phase);
        }
        if (!src_) src_ = make_synthetic_source(w, h, s.source >= 1 ? s.source - 1 : 0, 0x1234567u);
        src_kind_ = strcmp(src_->name(), "x11-shm") == 0 ? 1.0 : 0.0;
        {
            std::lock_guard<std::mutex> g(step_mu_);
            budget_ = target_ = delivered_ = 0;
        }
        // encoder
        try {
            int backend = s.use_cpu ? 0 : (sk_hip_device_count() > 0 ? 1 : 0);
            int sh = s.stripe_height > 0 ? s.stripe_height : 64;
            if (s.output_mode == 0) {
                jpeg::JpegConfig j;
                j.width = w; j.height = h; j.stripe_height = sh;
                j.quality = s.jpeg_quality; j.paint_quality = s.paint_over_jpeg_quality;
                j.use_paint_over = s.use_paint_over_quality; j.paint_over_trigger = s.paint_over_trigger_frames;
                jcfg_ = j;
                enc_.reset(backend ? create_hip_jpeg_backend(j, s.device) : create_cpu_jpeg_backend(j));
            } else {
                h264::EncoderConfig e;
                e.width = w & ~1; e.height = h & ~1; e.stripe_height = sh;
                if (s.output_width > 0 && s.output_height > 0 && (s.output_width != w || s.output_height != h)) {
                    e.src_width = w;   // K2: resample the capture inside the conversion kernel
                    e.src_height = h;
                    e.width = s.output_width & ~1;
                    e.height = s.output_height & ~1;
                }
                e.fullframe = s.h264_fullframe; e.full_range = s.h264_fullcolor;
                e.qp = sk_clip(s.h264_crf, 0, 51);
                e.paint_qp = sk_clip(s.h264_paintover_crf, 0, 51);
                e.use_paint_over = s.use_paint_over_quality;
                e.paint_over_trigger = s.paint_over_trigger_frames > 0 ? s.paint_over_trigger_frames : 15;
                e.paint_over_burst = s.h264_paintover_burst_frames > 0 ? s.h264_paintover_burst_frames : 5;
                e.streaming_mode = s.h264_streaming_mode;
                e.damage_threshold = s.damage_block_threshold > 0 ? s.damage_block_threshold : 10;
                e.damage_duration = s.damage_block_duration > 0 ? s.damage_block_duration : 20;
                e.fps = (float)(s.target_fps > 0 ? s.target_fps : 60.0);
                e.aq_strength = sk_clip(s.h264_aq_strength, 0, 64);
                e.subpel = s.h264_subpel >= 0 ? 1 : 0;
                if (s.h264_me_full < 0) e.me_full = 0;
                e.intra4x4 = s.h264_intra4x4 > 0 ? 1 : 0;
                e.rc_mode = s.h264_rc_mode >= 0 && s.h264_rc_mode <= 2 ? s.h264_rc_mode : h264::RC_CQP;
                e.bitrate_kbps = s.h264_bitrate_kbps > 0 ? s.h264_bitrate_kbps : 0;
                if (e.rc_mode == h264::RC_CBR && e.bitrate_kbps <= 0) e.rc_mode = h264::RC_CRF;
                if (s.output_mode == 2 || s.output_mode == 3) {   // HEVC / AV1: full-frame pictures
                    e.codec = s.output_mode == 2 ? 1 : 2;
                    e.fullframe = 1;
                    e.aq_strength = 0;
                    e.intra4x4 = 0;
                    e.deblock = 0;   // their own in-loop filters, not the H.264 front end's
                }
                ecfg_ = e;
                enc_.reset(backend ? create_hip_backend(e, s.device) : create_cpu_backend(e));
            }
            backend_ = backend;
        } catch (const std::exception& ex) {
            set_last_error(std::string("encoder init failed: ") + ex.what());
            src_.reset();
            return -1;
        }
        if (!enc_) {
            src_.reset();
            return -1;
        }
        // H.264 / HEVC encoders composite the cursor themselves (K13 overlay slot 1)
        cursor_via_enc_ = s.output_mode != 0;
        cursor_set_ = false;
        cursor_serial_ = 0;
        wm_sent_ = nullptr;
        wm_on_gpu_ = false;
        src_->set_cursor_overlay(cursor_via_enc_);
        running_ = true;
        registered_device_ = s.use_cpu ? -1 : s.device;
        if (registered_device_ >= 0) device_sessions(registered_device_, +1);
        th_ = std::thread([this] { loop(); });
        return 0;
    }

    void stop() {
        running_ = false;
        {
            std::lock_guard<std::mutex> g(step_mu_);
            step_cv_.notify_all();
        }
        if (th_.joinable()) th_.join();
        if (registered_device_ >= 0) device_sessions(registered_device_, -1);
        registered_device_ = -1;
        enc_.reset();
        src_.reset();
    }

    void request_keyframe() { key_req_ = true; }
    void set_qp(int qp, int paint_qp) { qp_req_ = (qp & 0xffff) | (paint_qp & 0xffff) << 16; }

    // Live move of the session's encoder to GPU `device` (load rebalancing across the
    // GPUs of a node, parallel/rebalance.py). The capture thread does it between two
    // frames: a new encoder is created on `device`, the old one's inter-frame state
    // (StateHeader v3: references, damage baseline, MV field, controller, K10 state) is
    // exported into a buffer on the old GPU, copied GPU-to-GPU (peer copy over xGMI)
    // and imported, so the next frame is a P frame continuing the same stream — the
    // client's decoder never sees the move. When the state cannot be carried (JPEG,
    // an export that fails) the new encoder starts with a key frame instead.
    // Returns 0 moved with the stream continued, 1 moved with a key frame, -1 not
    // moved (CPU session, target GPU unusable, timeout; last error says why).
    // The target encoder (allocations, hipGraph capture: the slow part) and the state's
    // staging buffers are made here, on the caller's thread, while the capture thread keeps
    // encoding on the old GPU; between two frames the capture thread only exports,
    // peer-copies and imports the state and swaps encoders. That stall is recorded (stats:
    // move_stall_ms). The old encoder and the staging buffers are released back here too
    // (hipFree synchronises the device: not on the capture thread).
    int move_to(int device, int timeout_ms) {
        if (!running_) {
            set_last_error("capture not running");
            return -1;
        }
        std::unique_ptr<EncoderBackend> nenc;
        if (backend_ && device >= 0 && device < sk_hip_device_count()) {
            try {
                nenc.reset(s_.output_mode == 0 ? create_hip_jpeg_backend(jcfg_, device)
                                               : create_hip_backend(ecfg_, device));
            } catch (const std::exception& ex) {
                set_last_error((std::string("encoder init on the target GPU failed: ") + ex.what()).c_str());
                return -1;
            }
            if (!nenc) {
                set_last_error("encoder init on the target GPU failed");
                return -1;
            }
        }
        std::shared_ptr<void> sa, sb;
        const int sdev = registered_device_;   // where the state is exported (checked again by do_move)
        if (nenc && sdev >= 0) {
            const int64_t n = nenc->state_bytes();
            if (n > 0) {
                sa = dev_buf(sdev, n);
                sb = dev_buf(device, n);
            }
        }
        std::unique_lock<std::mutex> g(move_mu_);
        const uint64_t ticket = ++move_ticket_;
        move_dev_ = device;
        move_enc_ = std::move(nenc);   // null: do_move reports why nothing can move
        move_a_ = std::move(sa);
        move_b_ = std::move(sb);
        move_a_dev_ = sdev;
        move_pending_ = true;   // the loop stops queueing a second frame until it is served
        auto done = [&] { return move_done_ >= ticket || !running_; };
        if (!move_cv_.wait_for(g, std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 10000), done)) {
            if (move_serving_ != ticket) {
                // the capture thread has not reached it: withdraw the request, so no move
                // happens after the caller has been told it failed
                move_done_ = ticket;
                move_pending_ = false;
                set_last_error("move timed out before the capture thread reached it (cancelled)");
            } else {
                set_last_error("move timed out while in progress on the capture thread (it completes there; "
                               "the device reports where the session ended up)");
            }
            return -1;
        }
        if (move_done_ < ticket) {
            set_last_error("capture stopped during the move");
            return -1;
        }
        if (move_rc_ < 0) set_last_error(move_err_);
        const int rc = move_rc_;
        std::unique_ptr<EncoderBackend> old = std::move(move_old_);   // released on this thread
        sa = std::move(move_a_);
        sb = std::move(move_b_);
        g.unlock();
        return rc;
    }
    static std::shared_ptr<void> dev_buf(int dev, int64_t n) {
        void* p = sk_dev_alloc(dev, n);
        if (!p) return nullptr;
        return std::shared_ptr<void>(p, [dev](void* q) { sk_dev_free(dev, q); });
    }
    int device() const { return registered_device_; }
    // K10: switch the rate control mode / CBR target from the next frame
    void set_rate(int mode, int kbps) {
        rate_req_ = (int64_t)1 << 62 | (int64_t)(mode & 0xff) << 32 | (uint32_t)(kbps > 0 ? kbps : 0);
    }
    void set_frame_callback(sk_frame_cb cb, void* user) {
        frame_cb_ = cb;
        frame_user_ = user;
    }

    // Premultiplied BGRA watermark, composited onto every captured frame before
    // encoding. location: 0 top-left, 1 top-right, 2 bottom-left, 3 bottom-right,
    // 4 centre, 5 bouncing (moves 2 px per frame), 6 tiled; < 0 disables.
    // (pixelflux's own enum is not part of the reference tree; this mapping is ours.)
    void set_watermark(const uint8_t* bgra, int w, int h, int location) {
        auto wm = std::make_shared<Watermark>();
        wm->px.assign(bgra, bgra + (size_t)w * h * 4);
        wm->w = w;
        wm->h = h;
        wm->loc = location;
        std::lock_guard<std::mutex> g(mu_);
        wm_ = std::move(wm);
    }

    // Step mode (sk_capture_settings.step_mode): the loop encodes exactly the frames
    // granted here, unpaced, two in flight; wait() blocks until all are delivered.
    void run(int64_t frames) {
        std::lock_guard<std::mutex> g(step_mu_);
        budget_ += frames;
        target_ += frames;
        step_cv_.notify_all();
    }
    int wait(int timeout_ms) {
        std::unique_lock<std::mutex> g(step_mu_);
        auto ok = [&] { return delivered_ >= target_ || !running_; };
        if (timeout_ms < 0) step_cv_.wait(g, ok);
        else if (!step_cv_.wait_for(g, std::chrono::milliseconds(timeout_ms), ok)) return 1;
        return delivered_ >= target_ ? 0 : -1;
    }

    // out: frames, mean encode ms, bytes, packets, source kind, last encode ms, then
    // the per-frame encode-time histogram: counts for le = kHistLe[i] ms and +Inf.
    static constexpr int kHist = 9;
    static constexpr double kHistLe[kHist - 1] = {0.25, 0.5, 1, 2, 4, 8, 16, 33};
    void stats(double* out, int n) {
        std::lock_guard<std::mutex> g(mu_);
        double v[9 + kHist] = {(double)frames_, frames_ ? enc_ms_sum_ / frames_ : 0.0, (double)bytes_,
                               (double)packets_, src_kind_, last_enc_ms_};
        for (int i = 0; i < kHist; i++) v[6 + i] = (double)hist_[i];
        v[6 + kHist] = (double)inflight_max_;   // frames in flight actually used (1 or 2)
        v[7 + kHist] = enc_ ? enc_->upload_fraction() : 1.0;   // rows uploaded / rows captured
        v[8 + kHist] = move_stall_ms_;   // last live move: capture thread time between two frames
        for (int i = 0; i < n && i < 9 + kHist; i++) out[i] = v[i];
    }
    // Capture-to-packets latency (ms) of the most recent frames, oldest first;
    // returns the count copied. reset != 0 clears the record afterwards.
    int latencies(float* out, int cap, int reset) {
        std::lock_guard<std::mutex> g(mu_);
        const int n = (int)std::min<uint64_t>(lat_count_, kLatRing);
        int k = std::min(cap, n);
        for (int i = 0; i < k; i++) out[i] = lat_[(lat_count_ - k + i) % kLatRing];
        if (reset) lat_count_ = 0;
        return k;
    }

   private:
    struct Watermark {
        std::vector<uint8_t> px;
        int w = 0, h = 0, loc = -1;
    };
    using clk = std::chrono::steady_clock;
    struct InFlight {
        uint16_t id;
        clk::time_point t_grab;
    };

    // Grabs, composites the watermark, uploads and launches frame `id`. Returns false
    // when the source has no frame (the caller retries at the next tick).
    bool start_frame(uint16_t id, std::deque<InFlight>& q) {
        int stride = 0;
        const uint8_t* px = nullptr;
        const auto t = clk::now();
        {
            trace::Range r("capture.grab");
            px = src_->grab(&stride);
        }
        if (!px) return false;
        std::shared_ptr<Watermark> wm;
        {
            std::lock_guard<std::mutex> g(mu_);
            wm = wm_;
        }
        const bool have_wm = wm && wm->loc >= 0 && !wm->px.empty();
        if (s_.output_mode != 0 && (have_wm || wm_on_gpu_)) {
            // H.264 / HEVC: K12 inside the encoder's colour conversion (overlay.h); the
            // grab buffer is left untouched
            if (wm.get() != wm_sent_) {
                wm_sent_ = wm.get();
                wm_on_gpu_ = have_wm && enc_->set_overlay_image(0, wm->px.data(), wm->w, wm->h) == 0;
                if (!have_wm) enc_->set_overlay_image(0, nullptr, 0, 0);
            }
            if (wm_on_gpu_) {
                int x, y, tdx, tdy;
                watermark_place(*wm, id, &x, &y, &tdx, &tdy);
                enc_->set_overlay_pos(0, 1, x, y, tdx, tdy);
            }
        }
        // K13: the cursor as encoder overlay slot 1 (sources that report it, X11)
        if (cursor_via_enc_) {
            int cx, cy, cw, ch;
            unsigned long serial = 0;
            if (src_->cursor(&cx, &cy, &cw, &ch, &serial, cursor_serial_, &cursor_px_)) {
                if (serial != cursor_serial_ || !cursor_set_) {
                    cursor_set_ = enc_->set_overlay_image(1, cursor_px_.data(), cw, ch) == 0;
                    cursor_serial_ = serial;
                    if (!cursor_set_) {   // too large for the overlay buffer: draw it on the host
                        enc_->set_overlay_pos(1, 0, 0, 0, 0, 0);   // and drop the stale GPU cursor
                        src_->set_cursor_overlay(false);
                        cursor_via_enc_ = false;
                    }
                }
                if (cursor_set_) enc_->set_overlay_pos(1, 1, cx, cy, 0, 0);
            }
        }
        // JPEG (or an image the encoder cannot hold): blend on the host into the grab
        // buffer (ours: SHM segment / ring; pool frames are never composited)
        bool composited = false;
        if (have_wm && !wm_on_gpu_ && pool_ == nullptr) {
            composite_watermark(const_cast<uint8_t*>(px), stride, id, *wm);
            composited = true;
        }
        // damage-driven upload: only rows the source reports as changed cross PCIe
        if (!composited && src_->damage(&dmg_rows_)) enc_->set_upload_rows(dmg_rows_.data(), (int)dmg_rows_.size() / 2);
        else enc_->set_upload_rows(nullptr, -1);
        try {
            if (enc_->upload(px, stride, id) < 0 || enc_->launch() < 0) return false;
        } catch (const std::exception& ex) {
            set_last_error(ex.what());
            return false;
        }
        q.push_back({id, t});
        return true;
    }

    void deliver(const InFlight& f, int n) {
        const double ms = std::chrono::duration<double, std::milli>(clk::now() - f.t_grab).count();
        size_t bytes = 0;
        std::vector<sk_stripe_result> res((size_t)std::max(n, 0));
        for (int i = 0; i < n; i++) {
            h264::EncodedPacket& p = enc_->packets_[i];
            sk_stripe_result& r = res[i];
            r.type = s_.output_mode == 0 ? 0 : (s_.output_mode >= 2 ? s_.output_mode : 1);
            r.stripe_y_start = p.y;
            r.stripe_height = p.h;
            r.size = (int32_t)p.data.size();
            r.data = p.data.data();
            r.frame_id = f.id;
            r.grab_ns = (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(f.t_grab.time_since_epoch()).count();
            bytes += p.data.size();
        }
        if (frame_cb_) frame_cb_(res.data(), n, frame_user_);   // one call per frame
        else if (cb_)
            for (int i = 0; i < n; i++) cb_(&res[i], user_);      // pixelflux contract: per stripe
        std::lock_guard<std::mutex> g(mu_);
        frames_++;
        int b = 0;
        while (b < kHist - 1 && ms > kHistLe[b]) b++;
        hist_[b]++;
        enc_ms_sum_ += ms;
        last_enc_ms_ = ms;
        bytes_ += bytes;
        packets_ += n > 0 ? n : 0;
        lat_[lat_count_++ % kLatRing] = (float)ms;
    }

    // A granted frame that could not be grabbed/launched counts as delivered (with
    // no packets), so wait() cannot hang on a failing source or encoder.
    void step_failed() {
        std::lock_guard<std::mutex> g(step_mu_);
        delivered_++;
        step_cv_.notify_all();
    }

    // Production loop. Paced (target_fps): grab at each tick, encode, deliver at
    // once (latency first). When the encoder falls behind the tick, or in step
    // mode, frame n+1 is grabbed, uploaded and launched before frame n is
    // finished, so the GPU always has the next frame queued (two in flight; needs
    // a source whose grab buffers survive one more grab, FrameSource::ring()).
    void loop() {
        const double fps = s_.target_fps > 0 ? s_.target_fps : 60.0;
        const auto period = std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(1.0 / fps));
        const bool step = s_.step_mode != 0;
        // Two frames in flight pay off for a session that has its GPU to itself (the
        // copy of frame n+1 overlaps the kernels of frame n). With several sessions
        // on one GPU the others fill those gaps, and the extra queued work only
        // lengthens the in-order hardware queues (GPU_MAX_HW_QUEUES = 4 shared by
        // every stream): measured 5587 fps with one in flight vs 4567 with two, 8
        // sessions at 1080p (profiles/r2_capture_pipeline.md). SK_CAPTURE_INFLIGHT
        // (1 or 2) overrides.
        const char* inflight_env = getenv("SK_CAPTURE_INFLIGHT");
        const int forced = inflight_env ? atoi(inflight_env) : 0;
        auto overlap_now = [&]() {
            if (src_->ring() < 2 || forced == 1) return false;
            return forced == 2 || device_sessions(s_.device, 0) <= 1;
        };
        auto next = clk::now();
        uint16_t frame_id = 0;
        std::deque<InFlight> q;
        auto take_budget = [&](bool block) -> bool {   // step mode: one frame of budget
            std::unique_lock<std::mutex> g(step_mu_);
            if (block) step_cv_.wait_for(g, std::chrono::milliseconds(50), [&] { return budget_ > 0 || !running_; });
            if (budget_ <= 0 || !running_) return false;
            budget_--;
            return true;
        };
        while (running_) {
            if (q.empty()) serve_move();   // a requested GPU move, between two frames
            if (key_req_.exchange(false)) enc_->request_keyframe();
            if (int qq = qp_req_.exchange(0)) enc_->set_qp(qq & 0xffff, qq >> 16), last_qp_ = qq;
            if (int64_t rr = rate_req_.exchange(0))
                enc_->set_rate((int)((rr >> 32) & 0xff), (int)(rr & 0xffffffff)), last_rate_ = rr;
            if (q.empty()) {
                if (step) {
                    if (!take_budget(true)) continue;
                } else {
                    auto now = clk::now();
                    if (next > now) std::this_thread::sleep_until(next);
                    next += period;
                    if (next < clk::now()) next = clk::now();   // behind schedule: do not burst
                }
                // a key-frame request that arrived while this thread waited for the budget /
                // the next tick belongs to the frame about to start, not the one after it
                if (key_req_.exchange(false)) enc_->request_keyframe();
                if (!start_frame(frame_id, q)) {
                    if (step) step_failed();
                    continue;
                }
                frame_id++;
            }
            // queue the next frame behind the one in flight when there is no time to idle
            if (q.size() < 2 && overlap_now() && !move_pending_) {
                bool go = step ? take_budget(false) : clk::now() >= next;
                if (go) {
                    if (!step) {
                        next += period;
                        if (next < clk::now()) next = clk::now();
                    }
                    if (key_req_.exchange(false)) enc_->request_keyframe();
                    if (start_frame(frame_id, q)) frame_id++;
                    else if (step) step_failed();
                }
            }
            if ((int)q.size() > inflight_max_) inflight_max_ = (int)q.size();
            int n = -1;
            try {
                n = enc_->finish();
            } catch (const std::exception& ex) {
                set_last_error(ex.what());
            }
            InFlight f = q.front();
            q.pop_front();
            deliver(f, n);
            if (step) {
                std::lock_guard<std::mutex> g(step_mu_);
                delivered_++;
                step_cv_.notify_all();
            }
        }
        {   // a move requested while stopping is not done
            std::lock_guard<std::mutex> g(move_mu_);
            move_cv_.notify_all();
        }
        while (!q.empty()) {   // drain (the encoder is destroyed after the thread ends)
            try {
                enc_->finish();
            } catch (const std::exception&) {
            }
            q.pop_front();
        }
        std::lock_guard<std::mutex> g(step_mu_);
        step_cv_.notify_all();
    }

    // Capture thread, no frame in flight: performs a pending move_to().
    void serve_move() {
        std::unique_ptr<EncoderBackend> nenc, old;
        std::shared_ptr<void> a, b;
        int dev, adev;
        uint64_t ticket;
        {
            std::lock_guard<std::mutex> g(move_mu_);
            if (move_done_ >= move_ticket_) return;   // none pending, or withdrawn by a timed-out caller
            move_pending_ = false;
            dev = move_dev_;
            ticket = move_ticket_;
            move_serving_ = ticket;
            nenc = std::move(move_enc_);
            a = std::move(move_a_);
            b = std::move(move_b_);
            adev = move_a_dev_;
        }
        std::string err;
        const auto t0 = clk::now();
        const int rc = do_move(dev, std::move(nenc), adev == s_.device ? a.get() : nullptr, b.get(), &old, &err);
        {
            std::lock_guard<std::mutex> gs(mu_);
            move_stall_ms_ = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
        }
        std::lock_guard<std::mutex> g(move_mu_);
        move_old_ = std::move(old);   // the caller releases them (a timed-out caller: the next move / close)
        move_a_ = std::move(a);
        move_b_ = std::move(b);
        move_rc_ = rc;
        move_err_ = err;
        move_done_ = std::max(move_done_, ticket);   // a withdrawn later ticket stays withdrawn
        move_cv_.notify_all();
    }

    // sa / sb: staging buffers made by move_to's caller on the old / new GPU (null: made here).
    // The replaced encoder goes to *old (released by the caller, off this thread).
    int do_move(int dev, std::unique_ptr<EncoderBackend> nenc, void* sa, void* sb,
                std::unique_ptr<EncoderBackend>* old, std::string* err) {
        trace::Range r("capture.move");
        if (!backend_ || dev < 0 || dev >= sk_hip_device_count() || !nenc) {
            *err = backend_ ? "no such GPU" : "CPU session: nothing to move";
            return -1;
        }
        bool carried = false;
        std::string why;
        const int64_t n = enc_->state_bytes();
        if (n <= 0) {
            why = "the encoder keeps no inter-frame state";
        } else if (nenc->state_bytes() != n) {
            why = "state sizes differ";
        } else {
            std::shared_ptr<void> own_a, own_b;   // fallback staging (no buffers from the caller)
            if (!sa) own_a = dev_buf(s_.device, n);
            if (!sb) own_b = dev_buf(dev, n);
            void* a = sa ? sa : own_a.get();
            void* b = sb ? sb : own_b.get();
            try {
                if (!a || !b) why = "device buffers: " + std::string(sk_last_error());
                else if (enc_->export_state(a, 1) != 0) why = "export: " + std::string(sk_last_error());
                else if (sk_dev_copy(dev, b, a, n, 3) != 0) why = "peer copy: " + std::string(sk_last_error());
                else if (nenc->import_state(b, 1) != 0) why = "import: " + std::string(sk_last_error());
                else carried = true;
            } catch (const std::exception& ex) {
                why = std::string("exception: ") + ex.what();
            }
        }
        if (!carried) {   // a fresh stream: key frame, with the rate control last asked for
            fprintf(stderr, "[capture] move to GPU %d: state not carried (%s), key frame\n", dev, why.c_str());
            nenc->request_keyframe();
            if (last_qp_) nenc->set_qp(last_qp_ & 0xffff, last_qp_ >> 16);
            if (last_rate_) nenc->set_rate((int)((last_rate_ >> 32) & 0xff), (int)(last_rate_ & 0xffffffff));
        }
        *old = std::move(enc_);   // the old encoder (and its GPU memory): released by the caller
        enc_ = std::move(nenc);
        if (registered_device_ >= 0) device_sessions(registered_device_, -1);
        registered_device_ = s_.device = dev;
        device_sessions(dev, +1);
        wm_sent_ = nullptr;       // overlays (watermark, cursor) are re-sent to the new encoder
        wm_on_gpu_ = false;
        cursor_set_ = false;
        return carried ? 0 : 1;
    }

    // Position of the watermark for frame t (location modes of set_watermark); tiled
    // placement returns the period in tdx/tdy (0 otherwise).
    void watermark_place(const Watermark& wmk, unsigned t, int* x, int* y, int* tdx, int* tdy) const {
        const int W = s_.capture_width, H = s_.capture_height, w = wmk.w, h = wmk.h, m = 16;
        *tdx = *tdy = 0;
        switch (wmk.loc) {
            case 0: *x = m; *y = m; break;
            case 1: *x = W - w - m; *y = m; break;
            case 2: *x = m; *y = H - h - m; break;
            case 3: *x = W - w - m; *y = H - h - m; break;
            case 4: *x = (W - w) / 2; *y = (H - h) / 2; break;
            case 5: {
                const int rx = std::max(1, W - w), ry = std::max(1, H - h);
                const int px_ = (int)((2 * t) % (2 * rx)), py_ = (int)((2 * t) % (2 * ry));
                *x = px_ < rx ? px_ : 2 * rx - px_;
                *y = py_ < ry ? py_ : 2 * ry - py_;
                break;
            }
            case 6:    // tiled from (m, m) with a 2m gap
                *x = m; *y = m; *tdx = w + 2 * m; *tdy = h + 2 * m;
                break;
            default:   // unknown location: off screen
                *x = W; *y = H;
                break;
        }
    }

    void composite_watermark(uint8_t* px, int stride, unsigned t, const Watermark& wmk) {
        const int W = s_.capture_width, H = s_.capture_height, w = wmk.w, h = wmk.h;
        auto blit = [&](int x0, int y0) {
            for (int j = 0; j < h; j++) {
                const int y = y0 + j;
                if (y < 0 || y >= H) continue;
                for (int i = 0; i < w; i++) {
                    const int x = x0 + i;
                    if (x < 0 || x >= W) continue;
                    const uint8_t* s = &wmk.px[((size_t)j * w + i) * 4];
                    const uint32_t a = s[3];
                    if (!a) continue;
                    uint8_t* d = px + (size_t)y * stride + 4 * x;
                    for (int c = 0; c < 3; c++) d[c] = (uint8_t)(s[c] + (d[c] * (255 - a) + 127) / 255);
                }
            }
        };
        const int m = 16;  // margin
        switch (wmk.loc) {
            case 0: blit(m, m); break;
            case 1: blit(W - w - m, m); break;
            case 2: blit(m, H - h - m); break;
            case 3: blit(W - w - m, H - h - m); break;
            case 4: blit((W - w) / 2, (H - h) / 2); break;
            case 5: {
                const int rx = std::max(1, W - w), ry = std::max(1, H - h);
                const int px_ = (int)((2 * t) % (2 * rx)), py_ = (int)((2 * t) % (2 * ry));
                blit(px_ < rx ? px_ : 2 * rx - px_, py_ < ry ? py_ : 2 * ry - py_);
                break;
            }
            case 6:
                for (int y = 0; y < H; y += h + 2 * m)
                    for (int x = 0; x < W; x += w + 2 * m) blit(x + m, y + m);
                break;
            default: break;
        }
    }

    std::shared_ptr<Watermark> wm_;
    const Watermark* wm_sent_ = nullptr;   // image last handed to the encoder overlay
    bool wm_on_gpu_ = false;
    bool cursor_via_enc_ = false, cursor_set_ = false;   // K13 through encoder overlay slot 1
    unsigned long cursor_serial_ = 0;
    std::vector<uint8_t> cursor_px_;
    int registered_device_ = -1;
    const uint8_t* pool_ = nullptr;
    std::vector<int> dmg_rows_;
    sk_frame_cb frame_cb_ = nullptr;
    void* frame_user_ = nullptr;
    std::mutex step_mu_;
    std::condition_variable step_cv_;
    int64_t budget_ = 0, target_ = 0, delivered_ = 0;
    static constexpr int kLatRing = 8192;
    float lat_[kLatRing] = {};
    uint64_t lat_count_ = 0;
    sk_capture_settings s_{};
    std::string display_;
    int inflight_max_ = 0;
    sk_stripe_cb cb_ = nullptr;
    void* user_ = nullptr;
    std::unique_ptr<FrameSource> src_;
    std::unique_ptr<EncoderBackend> enc_;
    std::thread th_;
    std::atomic<bool> running_{false}, key_req_{false}, move_pending_{false};
    std::atomic<int> qp_req_{0};
    std::atomic<int64_t> rate_req_{0};
    int last_qp_ = 0;
    int64_t last_rate_ = 0;
    int backend_ = 0;               // 0 CPU reference, 1 HIP
    h264::EncoderConfig ecfg_{};    // the configuration a moved encoder is created with
    jpeg::JpegConfig jcfg_{};
    std::mutex move_mu_;
    std::condition_variable move_cv_;
    uint64_t move_ticket_ = 0, move_done_ = 0, move_serving_ = 0;
    int move_dev_ = -1, move_rc_ = -1;
    std::string move_err_;
    std::unique_ptr<EncoderBackend> move_enc_;   // target encoder built by move_to's caller
    std::unique_ptr<EncoderBackend> move_old_;   // replaced encoder, released by move_to's caller
    std::shared_ptr<void> move_a_, move_b_;      // state staging on the old / new GPU
    int move_a_dev_ = -1;
    double move_stall_ms_ = 0.0;
    uint64_t hist_[kHist] = {};
    double src_kind_ = -1.0;  // 1 x11, 0 synthetic, -1 none (kept after stop for stats)
    std::mutex mu_;
    uint64_t frames_ = 0, bytes_ = 0, packets_ = 0;
    double enc_ms_sum_ = 0, last_enc_ms_ = 0;
};

}  // namespace sk

using sk::CaptureSession;

extern "C" {
void* sk_capture_create(void) { return new CaptureSession(); }
void sk_capture_destroy(void* c) { delete static_cast<CaptureSession*>(c); }
int sk_capture_start(void* c, const sk_capture_settings* s, sk_stripe_cb cb, void* user) {
    static_cast<CaptureSession*>(c)->set_frame_callback(nullptr, nullptr);
    return static_cast<CaptureSession*>(c)->start(*s, cb, user);
}
int sk_capture_start_frames(void* c, const sk_capture_settings* s, sk_frame_cb cb, void* user) {
    static_cast<CaptureSession*>(c)->set_frame_callback(cb, user);
    return static_cast<CaptureSession*>(c)->start(*s, nullptr, nullptr);
}
void sk_capture_run(void* c, int64_t frames) { static_cast<CaptureSession*>(c)->run(frames); }
int sk_capture_wait(void* c, int timeout_ms) { return static_cast<CaptureSession*>(c)->wait(timeout_ms); }
int sk_capture_latencies(void* c, float* out, int cap, int reset) {
    return static_cast<CaptureSession*>(c)->latencies(out, cap, reset);
}
void sk_capture_stop(void* c) { static_cast<CaptureSession*>(c)->stop(); }
void sk_capture_request_keyframe(void* c) { static_cast<CaptureSession*>(c)->request_keyframe(); }
void sk_capture_set_qp(void* c, int qp, int paint_qp) { static_cast<CaptureSession*>(c)->set_qp(qp, paint_qp); }
void sk_capture_set_rate(void* c, int mode, int kbps) { static_cast<CaptureSession*>(c)->set_rate(mode, kbps); }
void sk_capture_stats(void* c, double* out, int n) { static_cast<CaptureSession*>(c)->stats(out, n); }
int sk_capture_move(void* c, int device, int timeout_ms) {
    return static_cast<CaptureSession*>(c)->move_to(device, timeout_ms);
}
int sk_capture_device(void* c) { return static_cast<CaptureSession*>(c)->device(); }
void sk_capture_set_watermark(void* c, const uint8_t* bgra, int w, int h, int location) {
    static_cast<CaptureSession*>(c)->set_watermark(bgra, w, h, location);
}
}
