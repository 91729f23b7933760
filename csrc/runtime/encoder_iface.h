// Backend interface behind the C ABI.
#pragma once
#include <deque>
#include <string>
#include <vector>
#include "../codec/h264_frame.h"
#include "../codec/jpeg_encoder.h"

namespace sk {

void set_last_error(const std::string& e);

class EncoderBackend {
   public:
    virtual ~EncoderBackend() = default;
    virtual void request_keyframe() = 0;
    virtual int encode(const uint8_t* bgrx, int stride, uint16_t frame_id) = 0;
    // Split form of encode(): submit() queues the frame (the caller keeps `bgrx`
    // alive until finish()), finish() waits and returns the packet count. Several
    // encoders can be submitted before any is finished (bands of one frame, or
    // sessions driven from one thread). Default: synchronous; the packets of each
    // submitted frame are queued, so two frames may be submitted before finish().
    virtual int submit(const uint8_t* bgrx, int stride, uint16_t frame_id) {
        if (encode(bgrx, stride, frame_id) < 0) return -1;
        done_.push_back(std::move(packets_));
        packets_.clear();
        return 0;
    }
    virtual int finish() {
        if (done_.empty()) {
            set_last_error("finish() without a submitted frame");
            return -1;
        }
        packets_ = std::move(done_.front());
        done_.pop_front();
        return (int)packets_.size();
    }
    // submit() in two steps, so the next frame's upload can overlap this frame's
    // kernels: upload(n+1) ... finish(n) ... launch(n+1), or with two frames in
    // flight upload(n+1) launch(n+1) ... finish(n). Default: upload encodes.
    virtual int upload(const uint8_t* bgrx, int stride, uint16_t frame_id) { return submit(bgrx, stride, frame_id); }
    // Damage of the next upload(): `n` row ranges [r[2i], r[2i+1]) that differ from the
    // previously uploaded frame (n < 0: unknown, everything). A backend that keeps the
    // frame on the device may then copy only those rows (HIP: rows changed since the
    // frame its upload buffer last held).
    virtual void set_upload_rows(const int* r, int n) { (void)r; (void)n; }
    // Fraction of frame rows uploaded so far (1.0 without damage-driven uploads).
    virtual double upload_fraction() const { return 1.0; }
    // The next upload() waits (on the device) for the work queued so far on a foreign
    // HIP stream of this device, e.g. the torch stream an RCCL scatter wrote the frame on.
    virtual int wait_stream(void* stream) { (void)stream; return 0; }
    virtual int launch() { return 0; }
    // Planar 4:2:0 input (h264::YuvInput: fmt YUV_I420 / YUV_NV12, planes and strides)
    // instead of BGRx; on_device: the planes are device memory of this encoder's GPU.
    // Encodes the frame like encode() and returns the packet count.
    virtual int encode_yuv(const h264::YuvInput& in, int on_device, uint16_t frame_id) {
        (void)in; (void)on_device; (void)frame_id;
        set_last_error("this encoder takes BGRx input only");
        return -1;
    }
    // Session state transfer (h264::StateHeader layout). `on_device`: the buffer is
    // device memory of this encoder's GPU (HIP backend) instead of host memory.
    virtual int64_t state_bytes() { return -1; }
    virtual int export_state(void* dst, int on_device) { (void)dst; (void)on_device; return -1; }
    virtual int import_state(const void* src, int on_device) { (void)src; (void)on_device; return -1; }
    virtual int64_t debug_buffer(const char* name, void* dst, int64_t cap) = 0;
    virtual int stage_times(float* dst, int n) { (void)dst; (void)n; return 0; }
    // H.264 rate control hook (QP <= 0 keeps the current value); JPEG ignores it.
    virtual void set_qp(int qp, int paint_qp) { (void)qp; (void)paint_qp; }
    // K10 rate control (ratecontrol.h): mode RC_CQP / RC_CRF / RC_CBR, CBR bitrate.
    virtual void set_rate(int mode, int kbps) { (void)mode; (void)kbps; }
    // RcState words (ratecontrol.h) into out; returns the count (< 0: no controller).
    virtual int64_t rc_stats(int32_t* out, int n) { (void)out; (void)n; return -1; }
    // K12/K13 overlays (overlay.h), applied inside the colour conversion of the frames
    // uploaded after the call: slot 0 watermark, 1 cursor; premultiplied BGRA images.
    virtual int set_overlay_image(int slot, const uint8_t* bgra, int w, int h) {
        (void)slot; (void)bgra; (void)w; (void)h;
        return -1;
    }
    virtual int set_overlay_pos(int slot, int on, int x, int y, int tdx, int tdy) {
        (void)slot; (void)on; (void)x; (void)y; (void)tdx; (void)tdy;
        return -1;
    }
    std::vector<h264::EncodedPacket> packets_;

   protected:
    std::deque<std::vector<h264::EncodedPacket>> done_;
};

// Damage-driven upload: the union of row-range lists (pairs [y0, y1), any order, from
// the public API) on 16-row bands, as maximal row ranges clamped to [0, rows). Empty,
// inverted and out-of-frame pairs contribute nothing.
inline std::vector<std::pair<int, int>> upload_ranges(const std::vector<const std::vector<int>*>& lists, int rows) {
    std::vector<std::pair<int, int>> out;
    if (rows <= 0) return out;
    std::vector<uint8_t> band((size_t)(rows + 15) / 16, 0);
    for (const auto* v : lists)
        for (size_t i = 0; i + 1 < v->size(); i += 2) {
            const int y0 = (*v)[i] < 0 ? 0 : (*v)[i], y1 = (*v)[i + 1] > rows ? rows : (*v)[i + 1];
            if (y0 >= y1) continue;
            for (int y = y0 / 16; y * 16 < y1; y++) band[y] = 1;
        }
    for (int b = 0; b < (int)band.size();) {
        if (!band[b]) { b++; continue; }
        int e = b;
        while (e < (int)band.size() && band[e]) e++;
        out.emplace_back(b * 16, e * 16 < rows ? e * 16 : rows);
        b = e;
    }
    return out;
}

EncoderBackend* create_cpu_backend(const h264::EncoderConfig& c);
EncoderBackend* create_hip_backend(const h264::EncoderConfig& c, int device);
EncoderBackend* create_cpu_jpeg_backend(const jpeg::JpegConfig& c);
EncoderBackend* create_hip_jpeg_backend(const jpeg::JpegConfig& c, int device);
// Once per process and device, before the first session's frames: brings up the
// runtime's host->device copy engines (see h264_hip.cpp). SK_COPY_WARMUP=0 skips it.
void warm_copy_engines(int device);

}  // namespace sk
