// Native audio capture engine behind the pcmflux-compatible Python module
// (pcmflux/__init__.py): PulseAudio monitor source -> Opus packets on a native
// thread, one callback per packet.
//
// Reference contract: selkies.py:64-70 imports pcmflux's AudioCapture /
// AudioCaptureSettings / AudioChunkCallback; selkies.py:939-1070 starts it with
// device, sample rate, channels, opus bitrate, frame duration, VBR and the
// silence gate, and broadcasts every packet as 0x01 0x00 + opus. pcmflux itself
// is a C++ library; this is its MI355X-build counterpart (audio needs no GPU:
// ~320 kbit/s of Opus is a few percent of one core).
//
// libpulse-simple and libopus are resolved with dlopen at start time, so the
// library links and loads on machines without them (this build image, the GPU
// boxes). Two extra back ends exist for those machines and for tests:
//   source "synthetic[:hz]"  a paced sine tone (real-time, frame_duration_ms cadence)
//   codec  SK_AUDIO_PCM      raw s16le frames instead of Opus packets
// so the whole native loop (pacing, silence gate, callback, stop) is exercised
// without audio hardware.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <dlfcn.h>
#include <string>
#include <thread>
#include <vector>

#include "sk_api.h"

namespace {

// --- libpulse-simple / libopus entry points (subset), resolved at run time ---
struct PaSampleSpec { int format; uint32_t rate; uint8_t channels; };
struct PaBufferAttr { uint32_t maxlength, tlength, prebuf, minreq, fragsize; };
constexpr int kPaSampleS16le = 3;
constexpr int kPaStreamRecord = 2;
constexpr int kOpusApplicationAudio = 2049;
constexpr int kOpusSetBitrate = 4002;
constexpr int kOpusSetVbr = 4006;

struct PulseApi {
    void* h = nullptr;
    void* (*simple_new)(const char*, const char*, int, const char*, const char*, const PaSampleSpec*,
                        const void*, const PaBufferAttr*, int*) = nullptr;
    int (*simple_read)(void*, void*, size_t, int*) = nullptr;
    void (*simple_free)(void*) = nullptr;
    bool load() {
        if (h) return true;
        for (const char* n : {"libpulse-simple.so.0", "libpulse-simple.so"}) {
            if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        }
        if (!h) return false;
        simple_new = reinterpret_cast<decltype(simple_new)>(dlsym(h, "pa_simple_new"));
        simple_read = reinterpret_cast<decltype(simple_read)>(dlsym(h, "pa_simple_read"));
        simple_free = reinterpret_cast<decltype(simple_free)>(dlsym(h, "pa_simple_free"));
        return simple_new && simple_read && simple_free;
    }
};

struct OpusApi {
    void* h = nullptr;
    void* (*create)(int32_t, int, int, int*) = nullptr;
    int32_t (*encode)(void*, const int16_t*, int, unsigned char*, int32_t) = nullptr;
    int (*ctl)(void*, int, ...) = nullptr;
    void (*destroy)(void*) = nullptr;
    bool load() {
        if (h) return true;
        for (const char* n : {"libopus.so.0", "libopus.so"}) {
            if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        }
        if (!h) return false;
        create = reinterpret_cast<decltype(create)>(dlsym(h, "opus_encoder_create"));
        encode = reinterpret_cast<decltype(encode)>(dlsym(h, "opus_encode"));
        ctl = reinterpret_cast<decltype(ctl)>(dlsym(h, "opus_encoder_ctl"));
        destroy = reinterpret_cast<decltype(destroy)>(dlsym(h, "opus_encoder_destroy"));
        return create && encode && ctl && destroy;
    }
};

PulseApi g_pa;
OpusApi g_opus;

class AudioSession {
public:
    ~AudioSession() { stop(); }

    int start(const sk_audio_settings& s, sk_audio_cb cb, void* user) {
        if (th_.joinable()) return -1;
        rate_ = s.sample_rate > 0 ? s.sample_rate : 48000;
        ch_ = s.channels == 1 ? 1 : 2;
        const int dur = s.frame_duration_ms > 0 ? s.frame_duration_ms : 20;
        frame_ = rate_ * dur / 1000;
        gate_ = s.use_silence_gate != 0;
        codec_ = s.codec;
        cb_ = cb;
        user_ = user;
        const std::string dev = s.device_name ? s.device_name : "";
        synthetic_ = dev.rfind("synthetic", 0) == 0;
        if (synthetic_) {
            tone_hz_ = 440.0;
            if (dev.size() > 10 && dev[9] == ':') tone_hz_ = std::atof(dev.c_str() + 10);
            // a tone that is silent for the first `silence_frames` frames exercises the gate
            silence_frames_ = s.synthetic_silence_frames;
        } else {
            if (!g_pa.load()) { err_ = "libpulse-simple not available"; return -2; }
            PaSampleSpec spec{kPaSampleS16le, (uint32_t)rate_, (uint8_t)ch_};
            PaBufferAttr attr{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, (uint32_t)(frame_ * ch_ * 2)};
            int e = 0;
            pa_ = g_pa.simple_new(nullptr, "selkies", kPaStreamRecord, dev.empty() ? nullptr : dev.c_str(),
                                  "desktop-audio", &spec, nullptr, &attr, &e);
            if (!pa_) { err_ = "pa_simple_new failed (" + std::to_string(e) + ")"; return -3; }
        }
        if (codec_ == SK_AUDIO_OPUS) {
            if (!g_opus.load()) { err_ = "libopus not available"; close_source(); return -4; }
            int e = 0;
            enc_ = g_opus.create(rate_, ch_, kOpusApplicationAudio, &e);
            if (!enc_) { err_ = "opus_encoder_create failed (" + std::to_string(e) + ")"; close_source(); return -5; }
            g_opus.ctl(enc_, kOpusSetBitrate, (int32_t)(s.opus_bitrate > 0 ? s.opus_bitrate : 320000));
            g_opus.ctl(enc_, kOpusSetVbr, (int32_t)(s.use_vbr ? 1 : 0));
        }
        stop_ = false;
        th_ = std::thread([this] { loop(); });
        return 0;
    }

    void stop() {
        stop_ = true;
        if (th_.joinable()) th_.join();
        if (enc_) { g_opus.destroy(enc_); enc_ = nullptr; }
        close_source();
    }

    void stats(double* out, int n) const {
        const double v[4] = {(double)frames_.load(), (double)packets_.load(), (double)bytes_.load(),
                             (double)gated_.load()};
        for (int i = 0; i < n && i < 4; i++) out[i] = v[i];
    }

    const std::string& error() const { return err_; }

private:
    void close_source() {
        if (pa_) { g_pa.simple_free(pa_); pa_ = nullptr; }
    }

    bool read_frame(int16_t* pcm, std::chrono::steady_clock::time_point& next) {
        if (!synthetic_) {
            int e = 0;
            if (g_pa.simple_read(pa_, pcm, (size_t)frame_ * ch_ * 2, &e) < 0) {
                err_ = "pa_simple_read failed (" + std::to_string(e) + ")";
                return false;
            }
            return true;
        }
        // paced like a capture device: one frame per frame duration
        std::this_thread::sleep_until(next);
        next += std::chrono::microseconds((int64_t)frame_ * 1000000 / rate_);
        const bool silent = frames_.load() < (uint64_t)silence_frames_;
        for (int i = 0; i < frame_; i++) {
            const double t = (double)(phase_ + i) / rate_;
            const int16_t v = silent ? 0 : (int16_t)std::lrint(8000.0 * std::sin(2.0 * M_PI * tone_hz_ * t));
            for (int c = 0; c < ch_; c++) pcm[i * ch_ + c] = v;
        }
        phase_ += frame_;
        return true;
    }

    void loop() {
        std::vector<int16_t> pcm((size_t)frame_ * ch_);
        std::vector<unsigned char> out(codec_ == SK_AUDIO_OPUS ? 4000 : pcm.size() * 2);
        auto next = std::chrono::steady_clock::now();
        while (!stop_) {
            if (!read_frame(pcm.data(), next)) break;
            frames_++;
            if (gate_) {
                bool any = false;
                for (int16_t v : pcm) { if (v) { any = true; break; } }
                if (!any) { gated_++; continue; }
            }
            int n;
            if (codec_ == SK_AUDIO_OPUS) {
                n = g_opus.encode(enc_, pcm.data(), frame_, out.data(), (int32_t)out.size());
            } else {
                n = (int)(pcm.size() * 2);
                std::memcpy(out.data(), pcm.data(), (size_t)n);
            }
            if (n <= 0) continue;
            sk_audio_chunk chunk{n, out.data()};
            packets_++;
            bytes_ += (uint64_t)n;
            cb_(&chunk, user_);
        }
    }

    int rate_ = 48000, ch_ = 2, frame_ = 960, codec_ = SK_AUDIO_OPUS, silence_frames_ = 0;
    bool gate_ = false, synthetic_ = false;
    double tone_hz_ = 440.0;
    int64_t phase_ = 0;
    void* pa_ = nullptr;
    void* enc_ = nullptr;
    sk_audio_cb cb_ = nullptr;
    void* user_ = nullptr;
    std::thread th_;
    std::atomic<bool> stop_{false};
    std::atomic<uint64_t> frames_{0}, packets_{0}, bytes_{0}, gated_{0};
    std::string err_;
};

}  // namespace

extern "C" {

int sk_audio_available(void) {
    return (g_pa.load() ? 1 : 0) | (g_opus.load() ? 2 : 0);
}

void* sk_audio_create(void) { return new AudioSession(); }

void sk_audio_destroy(void* a) { delete static_cast<AudioSession*>(a); }

int sk_audio_start(void* a, const sk_audio_settings* s, sk_audio_cb cb, void* user) {
    if (!a || !s || !cb) return -1;
    return static_cast<AudioSession*>(a)->start(*s, cb, user);
}

void sk_audio_stop(void* a) {
    if (a) static_cast<AudioSession*>(a)->stop();
}

void sk_audio_stats(void* a, double* out, int n) {
    if (a) static_cast<AudioSession*>(a)->stats(out, n);
}

const char* sk_audio_error(void* a) {
    return a ? static_cast<AudioSession*>(a)->error().c_str() : "";
}

}  // extern "C"
