// HIP backend of the JPEG stripe encoder. Frame flow:
//   H2D(BGRx into the ping-pong frame buffer)
//   -> [k_damage, k_blocks(+stripe plan), k_scan, k_write, k_ffcount, k_stuff]
//      (one hipGraph per frame-buffer parity; stripe plan state lives on the GPU,
//      double-buffered by parity)
//   -> one sync -> packets = [frame_id][y] + cached JFIF header + entropy
//      segment read straight out of host-mapped memory.
#include "encoder_iface.h"
#include "trace.h"
#include "../kernels/jpeg_gpu.h"
#include <hip/hip_runtime.h>
#include <stdexcept>
#include <string.h>
#include <string>

namespace sk {
namespace {

#define HIPCHECK(x)                                                                     \
    do {                                                                                \
        hipError_t e__ = (x);                                                           \
        if (e__ != hipSuccess)                                                          \
            throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e__)); \
    } while (0)

using namespace jpeg;

class HipJpegBackend : public EncoderBackend {
   public:
    HipJpegBackend(const JpegConfig& c, int device) : cfg_(c), device_(device) {
        if (cfg_.stripe_height <= 0 || cfg_.stripe_height % 16)
            throw std::runtime_error("JPEG stripe height must be a positive multiple of 16");
        L_.init(cfg_);
        build_tables(cfg_.quality, tab_[0]);
        build_tables(cfg_.paint_quality, tab_[1]);
        st_.assign(L_.num_stripes, JpegStripeState());
        for (int q = 0; q < 2; q++) {
            build_jpeg_header(L_.W, L_.stripe_pix_h(0), tab_[q], hdr_[q][0]);
            build_jpeg_header(L_.W, L_.stripe_pix_h(L_.num_stripes - 1), tab_[q], hdr_[q][1]);
        }
        HIPCHECK(hipSetDevice(device_));
        warm_copy_engines(device_);
        HIPCHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
        alloc();
    }
    ~HipJpegBackend() override {
        hipSetDevice(device_);
        for (auto& g : graph_)
            if (g) hipGraphExecDestroy(g);
        for (void* p : dev_) hipFree(p);
        for (void* p : host_) hipHostFree(p);
        for (auto* f : frame_)
            if (f) hipFree(f);
        hipStreamDestroy(stream_);
    }

    void request_keyframe() override {
        // consumed by the next frame's stripe plan (host-mapped counter)
        __atomic_add_fetch(h_key_seq_, 1, __ATOMIC_SEQ_CST);
    }

    int encode(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        trace::Range frame_range("jpeg.frame");
        HIPCHECK(hipSetDevice(device_));
        packets_.clear();
        const size_t bytes = (size_t)stride * L_.H;
        if (bytes > frame_cap_ || stride != a_.stride) {
            for (auto*& f : frame_) {
                if (f) hipFree(f);
                HIPCHECK(hipMalloc(&f, bytes));
            }
            frame_cap_ = bytes;
            a_.stride = stride;
            first_ = true;
            for (auto& g : graph_)
                if (g) { hipGraphExecDestroy(g); g = nullptr; }
        }
        if (first_) {  // (re)start: every stripe is sent on the first frame
            for (auto* st : state_)
                HIPCHECK(hipMemcpyAsync(st, st_.data(), sizeof(JpegStripeState) * st_.size(), hipMemcpyHostToDevice,
                                        stream_));
            for (auto* d : dirty_) HIPCHECK(hipMemsetAsync(d, 0, sizeof(int) * L_.num_stripes, stream_));
            HIPCHECK(hipStreamSynchronize(stream_));
            first_ = false;
        }
        a_.cur = frame_[parity_];
        a_.prev = frame_[parity_ ^ 1];
        a_.state_in = state_[parity_];
        a_.state_out = state_[parity_ ^ 1];
        a_.dirty_in = dirty_[parity_];
        a_.dirty_out = dirty_[parity_ ^ 1];
        HIPCHECK(hipMemcpyAsync(frame_[parity_], bgrx, bytes, hipMemcpyHostToDevice, stream_));
        run_graph();
        HIPCHECK(hipStreamSynchronize(stream_));
        for (int s = 0; s < L_.num_stripes; s++) {
            const int act = h_action_[s];
            if (act < 0) continue;
            const int n = h_size_[s];
            if (n <= 0 || n > a_.out_slot) throw std::runtime_error("JPEG stripe size out of range");
            const std::vector<uint8_t>& hdr = hdr_[act][s == L_.num_stripes - 1 ? 1 : 0];
            h264::EncodedPacket pk;
            pk.y = L_.stripe_y(s);
            pk.w = L_.W;
            pk.h = L_.stripe_pix_h(s);
            pk.key = 1;
            pk.data.reserve(4 + hdr.size() + (size_t)n);
            const uint8_t pre[4] = {(uint8_t)(frame_id >> 8), (uint8_t)frame_id, (uint8_t)(pk.y >> 8),
                                    (uint8_t)pk.y};
            pk.data.insert(pk.data.end(), pre, pre + 4);
            pk.data.insert(pk.data.end(), hdr.begin(), hdr.end());
            const uint8_t* seg = h_out_ + (size_t)s * a_.out_slot;
            pk.data.insert(pk.data.end(), seg, seg + n);
            packets_.push_back(std::move(pk));
        }
        parity_ ^= 1;
        return (int)packets_.size();
    }

    int64_t debug_buffer(const char* name, void* dst, int64_t cap) override {
        HIPCHECK(hipSetDevice(device_));
        HIPCHECK(hipStreamSynchronize(stream_));
        std::string s(name);
        const void* p = nullptr;
        int64_t n = 0;
        const int64_t nb = (int64_t)L_.num_stripes * a_.blocks_per_stripe;
        if (s == "coef") { p = a_.coef; n = nb * 64 * 2; }
        else if (s == "dc") { p = a_.dc; n = nb * 2; }
        else if (s == "blk_off") { p = a_.blk_off; n = nb * 4; }
        else if (s == "stripe_bits") { p = a_.stripe_bits; n = L_.num_stripes * 4; }
        else if (s == "state") { p = state_[parity_]; n = L_.num_stripes * (int64_t)sizeof(JpegStripeState); }
        else return -1;
        if (dst && cap >= n) HIPCHECK(hipMemcpyAsync(dst, p, (size_t)n, hipMemcpyDeviceToHost, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
        return n;
    }

   private:
    template <class T>
    T* dmalloc(size_t count) {
        void* p = nullptr;
        HIPCHECK(hipMalloc(&p, count * sizeof(T)));
        HIPCHECK(hipMemsetAsync(p, 0, count * sizeof(T), stream_));
        dev_.push_back(p);
        return (T*)p;
    }
    template <class T>
    T* hmalloc(size_t count, unsigned flags) {
        void* p = nullptr;
        HIPCHECK(hipHostMalloc(&p, count * sizeof(T), flags));
        memset(p, 0, count * sizeof(T));
        host_.push_back(p);
        return (T*)p;
    }

    void alloc() {
        const int ns = L_.num_stripes;
        const int bps = (cfg_.stripe_height / 16) * L_.mcu_w * 6;
        const size_t nb = (size_t)ns * bps;
        a_ = gpu::JpegArgs{};
        a_.W = L_.W;
        a_.H = L_.H;
        a_.stripe_h = cfg_.stripe_height;
        a_.num_stripes = ns;
        a_.mcu_w = L_.mcu_w;
        a_.blocks_per_stripe = bps;
        a_.stride = -1;
        for (int i = 0; i < 2; i++) {
            dirty_[i] = dmalloc<int>(ns);
            state_[i] = dmalloc<JpegStripeState>(ns);
        }
        a_.action = dmalloc<int>(ns);
        a_.key_now = dmalloc<int>(1);
        a_.use_paint_over = cfg_.use_paint_over;
        a_.paint_over_trigger = cfg_.paint_over_trigger;
        JpegTables* dt = dmalloc<JpegTables>(2);
        HIPCHECK(hipMemcpyAsync(dt, tab_, sizeof(tab_), hipMemcpyHostToDevice, stream_));
        HIPCHECK(hipStreamSynchronize(stream_));
        a_.tabs = dt;
        a_.coef = dmalloc<int16_t>(nb * 64);
        a_.dc = dmalloc<int16_t>(nb);
        a_.dcdiff = dmalloc<int16_t>(nb);
        a_.ac_bits = dmalloc<int>(nb);
        a_.blk_off = dmalloc<int>(nb);
        a_.stripe_bits = dmalloc<int>(ns);
        const size_t slot_bytes = ((size_t)bps * gpu::kMaxBlockBytes + 64 + 15) & ~(size_t)15;
        a_.bits_slot_words = (int)(slot_bytes / 4);
        a_.bits = dmalloc<uint32_t>((size_t)ns * a_.bits_slot_words);
        a_.out_slot = (int)slot_bytes;
        a_.max_tiles = (int)(((size_t)bps * 208 + gpu::kTileBytes - 1) / gpu::kTileBytes);
        a_.tile_ff = dmalloc<int>((size_t)ns * a_.max_tiles);
        h_out_ = hmalloc<uint8_t>((size_t)ns * slot_bytes, hipHostMallocMapped);
        h_size_ = hmalloc<int>(ns, hipHostMallocMapped);
        h_action_ = hmalloc<int>(ns, hipHostMallocMapped);
        h_key_seq_ = hmalloc<int>(1, hipHostMallocMapped);
        a_.host_out = dev_ptr(h_out_);
        a_.host_size = dev_ptr(h_size_);
        a_.host_action = dev_ptr(h_action_);
        a_.key_seq = dev_ptr(h_key_seq_);
    }

    template <class T>
    T* dev_ptr(T* host) {
        void* dp = nullptr;
        HIPCHECK(hipHostGetDevicePointer(&dp, host, 0));
        return (T*)dp;
    }

    void run_graph() {
        hipGraphExec_t& g = graph_[parity_];
        if (!g) {
            hipGraph_t graph;
            HIPCHECK(hipStreamBeginCapture(stream_, hipStreamCaptureModeRelaxed));
            gpu::launch_frame(a_, stream_);
            HIPCHECK(hipStreamEndCapture(stream_, &graph));
            HIPCHECK(hipGraphInstantiate(&g, graph, nullptr, nullptr, 0));
            hipGraphDestroy(graph);
        }
        HIPCHECK(hipGraphLaunch(g, stream_));
    }

    JpegConfig cfg_;
    int device_;
    JpegLayout L_;
    JpegTables tab_[2];
    std::vector<uint8_t> hdr_[2][2];
    std::vector<JpegStripeState> st_;
    hipStream_t stream_ = nullptr;
    gpu::JpegArgs a_{};
    uint8_t* frame_[2] = {nullptr, nullptr};
    size_t frame_cap_ = 0;
    int parity_ = 0;
    bool first_ = true;
    int* h_action_ = nullptr;
    int* h_key_seq_ = nullptr;
    int* dirty_[2] = {nullptr, nullptr};
    JpegStripeState* state_[2] = {nullptr, nullptr};
    int* h_size_ = nullptr;
    uint8_t* h_out_ = nullptr;
    std::vector<void*> dev_, host_;
    hipGraphExec_t graph_[2] = {nullptr, nullptr};
};

}  // namespace

EncoderBackend* create_hip_jpeg_backend(const jpeg::JpegConfig& c, int device) {
    return new HipJpegBackend(c, device);
}

}  // namespace sk
