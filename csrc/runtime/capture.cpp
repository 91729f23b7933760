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
#include <chrono>
#include <mutex>
#include <string.h>
#include <string>
#include <thread>
#include <algorithm>
#include <vector>


namespace sk {

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
        if (!src_) src_ = make_synthetic_source(w, h, s.source >= 1 ? s.source - 1 : 0, 0x1234567u);
        src_kind_ = strcmp(src_->name(), "x11-shm") == 0 ? 1.0 : 0.0;
        // encoder
        try {
            int backend = s.use_cpu ? 0 : (sk_hip_device_count() > 0 ? 1 : 0);
            int sh = s.stripe_height > 0 ? s.stripe_height : 64;
            if (s.output_mode == 0) {
                jpeg::JpegConfig j;
                j.width = w; j.height = h; j.stripe_height = sh;
                j.quality = s.jpeg_quality; j.paint_quality = s.paint_over_jpeg_quality;
                j.use_paint_over = s.use_paint_over_quality; j.paint_over_trigger = s.paint_over_trigger_frames;
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
                enc_.reset(backend ? create_hip_backend(e, s.device) : create_cpu_backend(e));
            }
        } catch (const std::exception& ex) {
            set_last_error(std::string("encoder init failed: ") + ex.what());
            src_.reset();
            return -1;
        }
        if (!enc_) {
            src_.reset();
            return -1;
        }
        running_ = true;
        th_ = std::thread([this] { loop(); });
        return 0;
    }

    void stop() {
        running_ = false;
        if (th_.joinable()) th_.join();
        enc_.reset();
        src_.reset();
    }

    void request_keyframe() { key_req_ = true; }
    void set_qp(int qp, int paint_qp) { qp_req_ = (qp & 0xffff) | (paint_qp & 0xffff) << 16; }

    // Premultiplied BGRA watermark, composited onto every captured frame before
    // encoding. location: 0 top-left, 1 top-right, 2 bottom-left, 3 bottom-right,
    // 4 centre, 5 bouncing (moves 2 px per frame), 6 tiled; < 0 disables.
    // (pixelflux's own enum is not part of the reference tree; this mapping is ours.)
    void set_watermark(const uint8_t* bgra, int w, int h, int location) {
        std::lock_guard<std::mutex> g(mu_);
        wm_.assign(bgra, bgra + (size_t)w * h * 4);
        wm_w_ = w;
        wm_h_ = h;
        wm_loc_ = location;
    }

    // out: frames, mean encode ms, bytes, packets, source kind, last encode ms, then
    // the per-frame encode-time histogram: counts for le = kHistLe[i] ms and +Inf.
    static constexpr int kHist = 9;
    static constexpr double kHistLe[kHist - 1] = {0.25, 0.5, 1, 2, 4, 8, 16, 33};
    void stats(double* out, int n) {
        std::lock_guard<std::mutex> g(mu_);
        double v[6 + kHist] = {(double)frames_, frames_ ? enc_ms_sum_ / frames_ : 0.0, (double)bytes_,
                               (double)packets_, src_kind_, last_enc_ms_};
        for (int i = 0; i < kHist; i++) v[6 + i] = (double)hist_[i];
        for (int i = 0; i < n && i < 6 + kHist; i++) out[i] = v[i];
    }

   private:
    void loop() {
        using clk = std::chrono::steady_clock;
        const double fps = s_.target_fps > 0 ? s_.target_fps : 60.0;
        const auto period = std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(1.0 / fps));
        auto next = clk::now();
        uint16_t frame_id = 0;
        while (running_) {
            if (key_req_.exchange(false)) enc_->request_keyframe();
            if (int q = qp_req_.exchange(0)) enc_->set_qp(q & 0xffff, q >> 16);
            int stride = 0;
            const uint8_t* px = nullptr;
            {
                trace::Range r("capture.grab");
                px = src_->grab(&stride);
            }
            if (px && wm_loc_ >= 0 && !wm_.empty()) composite_watermark(const_cast<uint8_t*>(px), stride, frame_id);
            if (px) {
                auto t0 = clk::now();
                int n = -1;
                try {
                    n = enc_->encode(px, stride, frame_id);
                } catch (const std::exception& ex) {
                    set_last_error(ex.what());
                    n = -1;
                }
                double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
                size_t bytes = 0;
                for (int i = 0; i < n; i++) {
                    h264::EncodedPacket& p = enc_->packets_[i];
                    sk_stripe_result r;
                    r.type = s_.output_mode == 0 ? 0 : 1;
                    r.stripe_y_start = p.y;
                    r.stripe_height = p.h;
                    r.size = (int32_t)p.data.size();
                    r.data = p.data.data();
                    r.frame_id = frame_id;
                    bytes += p.data.size();
                    if (cb_) cb_(&r, user_);
                }
                {
                    std::lock_guard<std::mutex> g(mu_);
                    frames_++;
                    int b = 0;
                    while (b < kHist - 1 && ms > kHistLe[b]) b++;
                    hist_[b]++;
                    enc_ms_sum_ += ms;
                    last_enc_ms_ = ms;
                    bytes_ += bytes;
                    packets_ += n > 0 ? n : 0;
                }
                frame_id++;
            }
            next += period;
            auto now = clk::now();
            if (next < now) next = now;  // behind schedule: do not burst
            else std::this_thread::sleep_until(next);
        }
    }

    void composite_watermark(uint8_t* px, int stride, unsigned t) {
        std::lock_guard<std::mutex> g(mu_);
        const int W = s_.capture_width, H = s_.capture_height, w = wm_w_, h = wm_h_;
        auto blit = [&](int x0, int y0) {
            for (int j = 0; j < h; j++) {
                const int y = y0 + j;
                if (y < 0 || y >= H) continue;
                for (int i = 0; i < w; i++) {
                    const int x = x0 + i;
                    if (x < 0 || x >= W) continue;
                    const uint8_t* s = &wm_[((size_t)j * w + i) * 4];
                    const uint32_t a = s[3];
                    if (!a) continue;
                    uint8_t* d = px + (size_t)y * stride + 4 * x;
                    for (int c = 0; c < 3; c++) d[c] = (uint8_t)(s[c] + (d[c] * (255 - a) + 127) / 255);
                }
            }
        };
        const int m = 16;  // margin
        switch (wm_loc_) {
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

    std::vector<uint8_t> wm_;
    int wm_w_ = 0, wm_h_ = 0, wm_loc_ = -1;
    sk_capture_settings s_{};
    std::string display_;
    sk_stripe_cb cb_ = nullptr;
    void* user_ = nullptr;
    std::unique_ptr<FrameSource> src_;
    std::unique_ptr<EncoderBackend> enc_;
    std::thread th_;
    std::atomic<bool> running_{false}, key_req_{false};
    std::atomic<int> qp_req_{0};
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
    return static_cast<CaptureSession*>(c)->start(*s, cb, user);
}
void sk_capture_stop(void* c) { static_cast<CaptureSession*>(c)->stop(); }
void sk_capture_request_keyframe(void* c) { static_cast<CaptureSession*>(c)->request_keyframe(); }
void sk_capture_set_qp(void* c, int qp, int paint_qp) { static_cast<CaptureSession*>(c)->set_qp(qp, paint_qp); }
void sk_capture_stats(void* c, double* out, int n) { static_cast<CaptureSession*>(c)->stats(out, n); }
void sk_capture_set_watermark(void* c, const uint8_t* bgra, int w, int h, int location) {
    static_cast<CaptureSession*>(c)->set_watermark(bgra, w, h, location);
}
}
