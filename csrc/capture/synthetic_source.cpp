// Synthetic X11-like framebuffer for headless hosts and benchmarks. Mirrors the
// content classes of selkies_gstreamer_amd/utils/synthetic.py:
//   kind 0 "motion"  - the page scrolls every frame, windows move, video region
//   kind 1 "desktop" - mostly static, one moving window and a scrolling band
//   kind 2 "noise"   - uniform random pixels
// Rendered into page-locked memory so the H2D upload is a direct DMA.
#include "frame_source.h"
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <string.h>
#include <vector>

namespace sk {
namespace {

class SyntheticSource : public FrameSource {
   public:
    SyntheticSource(int w, int h, int kind, uint32_t seed) : w_(w), h_(h), kind_(kind), rng_(seed | 1) {
        ph_ = 3 * h;
        page_.resize((size_t)w * ph_ * 4);
        for (int y = 0; y < ph_; y++)
            for (int x = 0; x < w; x++) {
                uint8_t* p = &page_[((size_t)y * w + x) * 4];
                p[0] = (uint8_t)fminf(255.f, fmaxf(0.f, 200 + 40 * sinf(x / 97.f) + 10 * cosf(y / 53.f)));
                p[1] = (uint8_t)fminf(255.f, fmaxf(0.f, 210 + 30 * cosf(y / 71.f)));
                p[2] = (uint8_t)fminf(255.f, fmaxf(0.f, 220 + 25 * sinf((x + y) / 131.f)));
                p[3] = 255;
            }
        for (int ty = 8; ty + 9 < ph_; ty += 18)  // glyph rows
            for (int gx = 0; gx + 8 <= w; gx += 8) {
                if (next() % 10 < 3) continue;
                for (int j = 0; j < 9; j++)
                    for (int i = 0; i < 7; i++)
                        if (next() % 100 < 35) {
                            uint8_t* p = &page_[((size_t)(ty + j) * w + gx + i) * 4];
                            p[0] = 30; p[1] = 30; p[2] = 40;
                        }
            }
        // kRing page-locked frames rendered round robin (FrameSource::ring())
        size_t bytes = (size_t)w * h * 4;
        if (hipHostMalloc((void**)&ring_base_, bytes * kRing, hipHostMallocDefault) != hipSuccess) {
            own_.resize(bytes * kRing);
            ring_base_ = own_.data();
        } else {
            pinned_ = true;
        }
        frame_bytes_ = bytes;
        vh_ = h / 6 > 16 ? h / 6 : 16;
        vw_ = w / 6 > 16 ? w / 6 : 16;
    }
    ~SyntheticSource() override {
        if (pinned_) hipHostFree(ring_base_);
    }
    int ring() const override { return kRing; }
    const uint8_t* grab(int* stride) override {
        *stride = w_ * 4;
        frame_ = ring_base_ + (size_t)(t_ % kRing) * frame_bytes_;
        const size_t row = (size_t)w_ * 4;
        if (kind_ == 2) {
            uint32_t* p = (uint32_t*)frame_;
            for (size_t i = 0; i < (size_t)w_ * h_; i++) p[i] = next();
            t_++;
            return frame_;
        }
        int scroll = kind_ == 0 ? (3 * t_) % (ph_ - h_) : 0;
        memcpy(frame_, &page_[(size_t)scroll * row], (size_t)h_ * row);
        if (kind_ == 1) {
            int s2 = (2 * t_) % (ph_ - h_);
            int y0 = h_ / 5, n = h_ / 8;
            memcpy(frame_ + (size_t)y0 * row, &page_[(size_t)(s2 + y0) * row], (size_t)n * row);
        }
        for (int k = 0; k < (kind_ == 1 ? 1 : 2); k++) {
            int ww = k ? w_ / 4 : w_ / 3, hh = k ? h_ / 4 : h_ / 3, sp = k ? 7 : 4;
            int x0 = (sp * t_ + k * w_ / 2) % (w_ - ww > 1 ? w_ - ww : 1);
            int y0 = (h_ / 3 + k * h_ / 5 + (t_ * (k + 1)) % 40) % (h_ - hh > 1 ? h_ - hh : 1);
            for (int y = y0; y < y0 + hh; y++) {
                uint32_t* p = (uint32_t*)(frame_ + (size_t)y * row) + x0;
                uint32_t c = (y - y0 < 18) ? 0xFF286EB4u : 0xFFECECECu;
                for (int x = 0; x < ww; x++) p[x] = c;
            }
        }
        if (kind_ == 0) {
            int vy = h_ - vh_ - 20, vx = w_ - vw_ - 20;
            if (vy > 0 && vx > 0)
                for (int y = 0; y < vh_; y++) {
                    uint32_t* p = (uint32_t*)(frame_ + (size_t)(vy + y) * row) + vx;
                    for (int x = 0; x < vw_; x++) p[x] = next() | 0xFF000000u;
                }
        }
        t_++;
        return frame_;
    }
    const char* name() const override { return "synthetic"; }

   private:
    uint32_t next() {  // xorshift32
        rng_ ^= rng_ << 13;
        rng_ ^= rng_ >> 17;
        rng_ ^= rng_ << 5;
        return rng_;
    }
    int w_, h_, kind_, ph_, vw_, vh_;
    int t_ = 0;
    uint32_t rng_;
    std::vector<uint8_t> page_, own_;
    static constexpr int kRing = 2;
    uint8_t* ring_base_ = nullptr;
    uint8_t* frame_ = nullptr;
    size_t frame_bytes_ = 0;
    bool pinned_ = false;
};

// Caller-owned pool of pre-rendered frames (benchmarks, replay): grab() cycles
// through them; the pool must outlive the session.
class PoolSource : public FrameSource {
   public:
    PoolSource(const uint8_t* base, int frames, int stride, int h, int phase)
        : base_(base), frames_(frames), stride_(stride), h_(h), t_(phase) {
        // What XDamage reports for a display: the 16-row bands of pool frame j that differ
        // from frame j - 1 (the frame grabbed before it). The pool is immutable while the
        // session runs, so this is computed once, here, outside any timed frame.
        dmg_.resize(frames_);
        for (int j = 0; j < frames_; j++) {
            const uint8_t* a = frame(j);
            const uint8_t* b = frame((j + frames_ - 1) % frames_);
            std::vector<int>& d = dmg_[j];
            for (int y0 = 0; y0 < h_; y0 += 16) {
                const int y1 = y0 + 16 < h_ ? y0 + 16 : h_;
                if (memcmp(a + (size_t)y0 * stride_, b + (size_t)y0 * stride_, (size_t)(y1 - y0) * stride_) == 0) continue;
                if (!d.empty() && d.back() == y0) d.back() = y1;   // extend the previous range
                else { d.push_back(y0); d.push_back(y1); }
            }
        }
    }
    const uint8_t* grab(int* stride) override {
        *stride = stride_;
        cur_ = t_++ % frames_;
        return frame(cur_);
    }
    int ring() const override { return frames_; }
    const char* name() const override { return "pool"; }
    bool damage(std::vector<int>* rows) override {
        if (cur_ < 0) return false;
        *rows = dmg_[cur_];
        return true;
    }

   private:
    const uint8_t* frame(int j) const { return base_ + (size_t)j * stride_ * h_; }
    const uint8_t* base_;
    int frames_, stride_, h_, t_;
    int cur_ = -1;
    std::vector<std::vector<int>> dmg_;
};

}  // namespace

std::unique_ptr<FrameSource> make_synthetic_source(int w, int h, int kind, uint32_t seed) {
    return std::unique_ptr<FrameSource>(new SyntheticSource(w, h, kind, seed));
}

std::unique_ptr<FrameSource> make_pool_source(const uint8_t* base, int frames, int stride, int h, int phase) {
    return std::unique_ptr<FrameSource>(new PoolSource(base, frames, stride, h, phase));
}

}  // namespace sk

extern "C" {
// Frame t (0-based) of the capture sessions' synthetic source (kind 0 motion, 1 desktop,
// 2 noise; the session seed), BGRx into out[h][w]: tests compare decoded frames against
// exactly what a session encoded as frame t.
int sk_synthetic_render(int w, int h, int kind, int t, uint8_t* out) {
    if (w <= 0 || h <= 0 || t < 0 || !out) return -1;
    auto src = sk::make_synthetic_source(w, h, kind, 0x1234567u);
    int stride = 0;
    const uint8_t* f = nullptr;
    for (int i = 0; i <= t; i++) f = src->grab(&stride);
    for (int y = 0; y < h; y++) memcpy(out + (size_t)y * w * 4, f + (size_t)y * stride, (size_t)w * 4);
    return 0;
}
}

