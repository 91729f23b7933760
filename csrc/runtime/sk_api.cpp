// C ABI implementation: encoder factory (CPU reference / HIP backend), packet
// access and debug hooks used by the Python layer and the tests.
#include "sk_api.h"
#include "encoder_iface.h"
#include "../codec/hevc_encoder.h"
#include "../codec/av1_encoder.h"
#include <hip/hip_runtime_api.h>
#include <string.h>
#include <string>
#include <mutex>
#include <stdlib.h>

namespace sk {

static thread_local std::string g_last_error;
void set_last_error(const std::string& e) { g_last_error = e; }

namespace {

// Planar input for a CPU encoder: device planes are copied to host memory first.
struct HostYuv {
    std::vector<uint8_t> buf[3];
    h264::YuvInput in;
    int load(const h264::YuvInput& src, int on_device, int W, int H) {
        in = src;
        if (!on_device) return 0;
        const int cw = (W + 1) / 2, ch = (H + 1) / 2;
        const int nplanes = src.fmt == h264::YUV_NV12 ? 2 : 3;
        for (int p = 0; p < nplanes; p++) {
            const int w = p == 0 ? W : (src.fmt == h264::YUV_NV12 ? 2 * cw : cw), h = p == 0 ? H : ch;
            buf[p].resize((size_t)w * h);
            if (hipMemcpy2D(buf[p].data(), w, src.p[p], src.stride[p], w, h, hipMemcpyDeviceToHost) != hipSuccess) {
                set_last_error("device planes: copy to the host failed");
                return -1;
            }
            in.p[p] = buf[p].data();
            in.stride[p] = w;
        }
        return 0;
    }
};

// Session state of a CPU encoder (h264_encoder.h StateHeader layout); HEVC / AV1 keep
// all their inter-frame state in the shared front end (references, controller, K10).
int cpu_export_state(h264::CpuH264Encoder& e, void* dst, int on_device) {
    if (on_device) return -1;
    uint8_t* o = static_cast<uint8_t*>(dst);
    h264::StateHeader h;
    h264::state_header(e.cfg, e.g, e.first_frame ? 0 : 1, e.ctl_.qp(), e.ctl_.paint_qp(), h);
    memcpy(o, &h, sizeof(h));
    o += sizeof(h);
    e.ctl_.export_states(reinterpret_cast<h264::StripeState*>(o));
    o += sizeof(h264::StripeState) * (e.g.num_slices + 1);
    memcpy(o, &e.ctl_.rc(), sizeof(h264::RcState));
    o += sizeof(h264::RcState);
    for (auto* planes : {e.ref, e.ref1, e.prev})
        for (int p = 0; p < 3; p++) {
            memcpy(o, planes[p].data(), planes[p].size());
            o += planes[p].size();
        }
    memcpy(o, e.mvfield.data(), e.mvfield.size() * sizeof(int16_t));
    return 0;
}

int cpu_import_state(h264::CpuH264Encoder& e, const void* src, int on_device) {
    if (on_device) return -1;
    const uint8_t* i = static_cast<const uint8_t*>(src);
    h264::StateHeader h;
    memcpy(&h, i, sizeof(h));
    if (!h264::state_header_matches(e.cfg, e.g, h)) {
        set_last_error("encoder state does not match this encoder's geometry / codec");
        return -1;
    }
    i += sizeof(h);
    e.ctl_.import_states(reinterpret_cast<const h264::StripeState*>(i));
    i += sizeof(h264::StripeState) * (e.g.num_slices + 1);
    memcpy(&e.ctl_.rc(), i, sizeof(h264::RcState));
    i += sizeof(h264::RcState);
    for (auto* planes : {e.ref, e.ref1, e.prev})
        for (int p = 0; p < 3; p++) {
            memcpy(planes[p].data(), i, planes[p].size());
            i += planes[p].size();
        }
    memcpy(e.mvfield.data(), i, e.mvfield.size() * sizeof(int16_t));
    e.first_frame = !h.started;
    e.set_qp(h.qp, h.paint_qp);
    return 0;
}

class CpuBackend : public EncoderBackend {
   public:
    explicit CpuBackend(const h264::EncoderConfig& c) : enc_(c) {}
    void request_keyframe() override { enc_.request_keyframe(); }
    void set_qp(int qp, int paint_qp) override { enc_.set_qp(qp, paint_qp); }
    void set_rate(int mode, int kbps) override { enc_.ctl_.set_rate(mode, kbps); }
    int64_t rc_stats(int32_t* out, int n) override {
        const int k = n < (int)(sizeof(h264::RcState) / 4) ? n : (int)(sizeof(h264::RcState) / 4);
        memcpy(out, &enc_.ctl_.rc(), (size_t)k * 4);
        return k;
    }
    int set_overlay_image(int slot, const uint8_t* bgra, int w, int h) override {
        enc_.set_overlay_image(slot, bgra, w, h);
        return 0;
    }
    int set_overlay_pos(int slot, int on, int x, int y, int tdx, int tdy) override {
        enc_.set_overlay_pos(slot, on, x, y, tdx, tdy);
        return 0;
    }
    int encode(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        packets_.clear();
        enc_.encode(bgrx, stride, frame_id, packets_);
        return (int)packets_.size();
    }
    int encode_yuv(const h264::YuvInput& in, int on_device, uint16_t frame_id) override {
        if (enc_.scaled_) { set_last_error("planar input cannot be resampled"); return -1; }
        HostYuv h;
        if (h.load(in, on_device, enc_.g.W, enc_.g.H) < 0) return -1;
        enc_.yuv_in = h.in;
        return encode(nullptr, 0, frame_id);
    }
    int64_t debug_buffer(const char* name, void* dst, int64_t cap) override {
        const void* p = nullptr;
        int64_t n = 0;
        std::string s(name);
        auto plane = [&](const std::vector<uint8_t>& v) { p = v.data(); n = (int64_t)v.size(); };
        if (s == "src_y") plane(enc_.prev[0]);  // after finish_frame the source lives in prev
        else if (s == "src_u") plane(enc_.prev[1]);
        else if (s == "src_v") plane(enc_.prev[2]);
        else if (s == "ref_y") plane(enc_.ref[0]);
        else if (s == "ref_u") plane(enc_.ref[1]);
        else if (s == "ref_v") plane(enc_.ref[2]);
        else if (s == "ref1_y") plane(enc_.ref1[0]);
        else if (s == "mbs") { p = enc_.mbs.data(); n = (int64_t)(enc_.mbs.size() * sizeof(h264::MbInfo)); }
        else if (s == "coefs") { p = enc_.coefs.data(); n = (int64_t)(enc_.coefs.size() * 2); }
        else if (s == "me") { p = enc_.me.data(); n = (int64_t)(enc_.me.size() * sizeof(h264::MeResult)); }
        else if (s == "tasks") { p = enc_.tasks.data(); n = (int64_t)(enc_.tasks.size() * sizeof(h264::SliceTask)); }
        else if (s == "mb_dirty") plane(enc_.mb_dirty);
        else if (s == "aq") { p = enc_.aq.data(); n = (int64_t)enc_.aq.size(); }
        else if (s == "fs_mv") { p = enc_.fs_mv.data(); n = (int64_t)(enc_.fs_mv.size() * 2); }
        else return -1;
        if (dst && cap >= n) memcpy(dst, p, (size_t)n);
        return n;
    }

    int64_t state_bytes() override { return (int64_t)h264::state_bytes(enc_.g); }
    int export_state(void* dst, int on_device) override { return cpu_export_state(enc_, dst, on_device); }
    int import_state(const void* src, int on_device) override { return cpu_import_state(enc_, src, on_device); }

   private:
    h264::CpuH264Encoder enc_;
};

class CpuHevcBackend : public EncoderBackend {
   public:
    explicit CpuHevcBackend(const h264::EncoderConfig& c) : enc_(c) {}
    void request_keyframe() override { enc_.request_keyframe(); }
    void set_qp(int qp, int paint_qp) override { enc_.set_qp(qp, paint_qp); }
    void set_rate(int mode, int kbps) override { enc_.fe.ctl_.set_rate(mode, kbps); }
    int64_t rc_stats(int32_t* out, int n) override {
        const int k = n < (int)(sizeof(h264::RcState) / 4) ? n : (int)(sizeof(h264::RcState) / 4);
        memcpy(out, &enc_.fe.ctl_.rc(), (size_t)k * 4);
        return k;
    }
    int set_overlay_image(int slot, const uint8_t* bgra, int w, int h) override {
        enc_.fe.set_overlay_image(slot, bgra, w, h);
        return 0;
    }
    int set_overlay_pos(int slot, int on, int x, int y, int tdx, int tdy) override {
        enc_.fe.set_overlay_pos(slot, on, x, y, tdx, tdy);
        return 0;
    }
    int encode(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        packets_.clear();
        enc_.encode(bgrx, stride, frame_id, packets_);
        return (int)packets_.size();
    }
    int encode_yuv(const h264::YuvInput& in, int on_device, uint16_t frame_id) override {
        if (enc_.fe.scaled_) { set_last_error("planar input cannot be resampled"); return -1; }
        HostYuv h;
        if (h.load(in, on_device, enc_.fe.g.W, enc_.fe.g.H) < 0) return -1;
        enc_.fe.yuv_in = h.in;
        return encode(nullptr, 0, frame_id);
    }
    int64_t debug_buffer(const char* name, void* dst, int64_t cap) override {
        const void* p = nullptr;
        int64_t n = 0;
        std::string s(name);
        auto plane = [&](const std::vector<uint8_t>& v) { p = v.data(); n = (int64_t)v.size(); };
        if (s == "src_y") plane(enc_.fe.prev[0]);
        else if (s == "src_u") plane(enc_.fe.prev[1]);
        else if (s == "src_v") plane(enc_.fe.prev[2]);
        else if (s == "ref_y") plane(enc_.fe.ref[0]);
        else if (s == "ref_u") plane(enc_.fe.ref[1]);
        else if (s == "ref_v") plane(enc_.fe.ref[2]);
        else if (s == "cus") { p = enc_.cus.data(); n = (int64_t)(enc_.cus.size() * sizeof(hevc::CuInfo)); }
        else if (s == "sao") { p = enc_.sao.data(); n = (int64_t)(enc_.sao.size() * sizeof(hevc::SaoParams)); }
        else if (s == "coefs") { p = enc_.coefs.data(); n = (int64_t)(enc_.coefs.size() * 2); }
        else if (s == "bin_n") { p = enc_.bin_n.data(); n = (int64_t)(enc_.bin_n.size() * 4); }
        else if (s == "pc_dbg") { p = enc_.pc_dbg_.data(); n = (int64_t)(enc_.pc_dbg_.size() * 4); }
        else if (s == "me") { p = enc_.fe.me.data(); n = (int64_t)(enc_.fe.me.size() * sizeof(h264::MeResult)); }
        else if (s == "tasks") { p = enc_.fe.tasks.data(); n = (int64_t)(enc_.fe.tasks.size() * sizeof(h264::SliceTask)); }
        else return -1;
        if (dst && cap >= n) memcpy(dst, p, (size_t)n);
        return n;
    }

    int64_t state_bytes() override { return (int64_t)h264::state_bytes(enc_.fe.g); }
    int export_state(void* dst, int on_device) override { return cpu_export_state(enc_.fe, dst, on_device); }
    int import_state(const void* src, int on_device) override {
        if (cpu_import_state(enc_.fe, src, on_device) < 0) return -1;
        // the next POC: the picture state's frame_num (the GPU back end codes POC from it)
        std::vector<h264::StripeState> st(enc_.fe.g.num_slices + 1);
        enc_.fe.ctl_.export_states(st.data());
        enc_.poc = st.back().frame_num;
        return 0;
    }

   private:
    hevc::CpuHevcEncoder enc_;
};

class CpuAv1Backend : public EncoderBackend {
   public:
    explicit CpuAv1Backend(const h264::EncoderConfig& c) : enc_(c, c.tile_cols_log2, c.tile_rows_log2) {}
    void request_keyframe() override { enc_.request_keyframe(); }
    void set_qp(int qp, int paint_qp) override { enc_.set_qp(qp, paint_qp); }
    void set_rate(int mode, int kbps) override { enc_.fe.ctl_.set_rate(mode, kbps); }
    int64_t rc_stats(int32_t* out, int n) override {
        const int k = n < (int)(sizeof(h264::RcState) / 4) ? n : (int)(sizeof(h264::RcState) / 4);
        memcpy(out, &enc_.fe.ctl_.rc(), (size_t)k * 4);
        return k;
    }
    int set_overlay_image(int slot, const uint8_t* bgra, int w, int h) override {
        enc_.fe.set_overlay_image(slot, bgra, w, h);
        return 0;
    }
    int set_overlay_pos(int slot, int on, int x, int y, int tdx, int tdy) override {
        enc_.fe.set_overlay_pos(slot, on, x, y, tdx, tdy);
        return 0;
    }
    int encode(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        packets_.clear();
        enc_.encode(bgrx, stride, frame_id, packets_);
        return (int)packets_.size();
    }
    int encode_yuv(const h264::YuvInput& in, int on_device, uint16_t frame_id) override {
        if (enc_.fe.scaled_) { set_last_error("planar input cannot be resampled"); return -1; }
        HostYuv h;
        if (h.load(in, on_device, enc_.fe.g.W, enc_.fe.g.H) < 0) return -1;
        enc_.fe.yuv_in = h.in;
        return encode(nullptr, 0, frame_id);
    }
    int64_t debug_buffer(const char* name, void* dst, int64_t cap) override {
        const void* p = nullptr;
        int64_t n = 0;
        std::string s(name);
        auto plane = [&](const std::vector<uint8_t>& v) { p = v.data(); n = (int64_t)v.size(); };
        if (s == "src_y") plane(enc_.fe.prev[0]);
        else if (s == "src_u") plane(enc_.fe.prev[1]);
        else if (s == "src_v") plane(enc_.fe.prev[2]);
        else if (s == "ref_y") plane(enc_.fe.ref[0]);
        else if (s == "ref_u") plane(enc_.fe.ref[1]);
        else if (s == "ref_v") plane(enc_.fe.ref[2]);
        else if (s == "blk") { p = enc_.blk.data(); n = (int64_t)(enc_.blk.size() * sizeof(av1::BlkInfo)); }
        else if (s == "levels") { p = enc_.lev.data(); n = (int64_t)(enc_.lev.size() * 2); }
        else if (s == "me") { p = enc_.fe.me.data(); n = (int64_t)(enc_.fe.me.size() * sizeof(h264::MeResult)); }
        else if (s == "tasks") { p = enc_.fe.tasks.data(); n = (int64_t)(enc_.fe.tasks.size() * sizeof(h264::SliceTask)); }
        else if (s == "av1_geo") { p = &enc_.geo; n = (int64_t)sizeof(av1::Av1Geo); }
        else if (s == "av1_qidx") { p = &enc_.fp.qidx; n = 4; }
        else return -1;
        if (dst && cap >= n) memcpy(dst, p, (size_t)n);
        return n;
    }

    int64_t state_bytes() override { return (int64_t)h264::state_bytes(enc_.fe.g); }
    int export_state(void* dst, int on_device) override { return cpu_export_state(enc_.fe, dst, on_device); }
    int import_state(const void* src, int on_device) override { return cpu_import_state(enc_.fe, src, on_device); }

   private:
    av1::CpuAv1Encoder enc_;
};

class CpuJpegBackend : public EncoderBackend {
   public:
    explicit CpuJpegBackend(const jpeg::JpegConfig& c) : enc_(c) {}
    void request_keyframe() override { enc_.request_keyframe(); }
    int encode(const uint8_t* bgrx, int stride, uint16_t frame_id) override {
        packets_.clear();
        enc_.encode(bgrx, stride, frame_id, packets_);
        return (int)packets_.size();
    }
    int64_t debug_buffer(const char*, void*, int64_t) override { return -1; }

   private:
    jpeg::CpuJpegEncoder enc_;
};

}  // namespace

EncoderBackend* create_cpu_jpeg_backend(const jpeg::JpegConfig& c) { return new CpuJpegBackend(c); }

EncoderBackend* create_cpu_backend(const h264::EncoderConfig& c) {
    if (c.codec == 1) return new CpuHevcBackend(c);
    if (c.codec == 2) return new CpuAv1Backend(c);
    return new CpuBackend(c);
}

h264::EncoderConfig to_config(const sk_h264_config* c) {
    h264::EncoderConfig e;
    e.width = c->width;
    e.height = c->height;
    e.stripe_height = c->stripe_height > 0 ? c->stripe_height : 64;
    e.fullframe = c->fullframe;
    e.full_range = c->full_range;
    e.qp = c->qp;
    e.paint_qp = c->paint_qp;
    e.use_paint_over = c->use_paint_over;
    e.paint_over_trigger = c->paint_over_trigger;
    e.paint_over_burst = c->paint_over_burst;
    e.streaming_mode = c->streaming_mode;
    e.damage_threshold = c->damage_threshold;
    e.damage_duration = c->damage_duration;
    e.me_range = c->me_range > 0 ? c->me_range : 64;
    e.me_iters = c->me_iters > 0 ? c->me_iters : 24;
    e.scenecut = c->scenecut;
    e.fps = c->fps > 0 ? c->fps : 60.f;
    e.deblock = c->deblock < 0 ? 0 : (c->deblock == 1 ? 1 : 2);   // default automatic (h264_encoder.h slice_deblock)
    e.me_full = c->me_full >= 0 ? 1 : 0;
    e.shared_copy = c->shared_copy > 0 ? 1 : 0;
    e.src_width = c->src_width > 0 ? c->src_width : 0;
    e.src_height = c->src_height > 0 ? c->src_height : 0;
    e.num_refs = c->num_refs > 1 ? 2 : 1;
    e.codec = (c->codec == 1 || c->codec == 2) ? c->codec : 0;
    e.tile_cols_log2 = c->tile_cols_log2;
    e.tile_rows_log2 = c->tile_rows_log2;
    e.rc_mode = c->rc_mode >= 0 && c->rc_mode <= 2 ? c->rc_mode : 0;
    e.bitrate_kbps = c->bitrate_kbps > 0 ? c->bitrate_kbps : 0;
    if (e.rc_mode == h264::RC_CBR && e.bitrate_kbps <= 0) e.rc_mode = h264::RC_CRF;
    e.aq_strength = c->aq_strength > 0 ? (c->aq_strength > 64 ? 64 : c->aq_strength) : 0;
    e.subpel = c->subpel >= 0 ? 1 : 0;
    e.intra4x4 = c->intra4x4 > 0 ? 1 : 0;
    if (e.codec >= 1) {   // HEVC / AV1: full-frame pictures, slices of whole CTB rows, one reference
        e.aq_strength = 0;   // no cu_qp_delta in this HEVC profile setup
        e.fullframe = 1;
        e.num_refs = 1;
        e.deblock = 0;
    }
    return e;
}

}  // namespace sk

using namespace sk;

extern "C" {

const char* sk_version(void) { return "selkies-mi355x native 0.1 (gfx950)"; }

int sk_hip_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int sk_hip_pci_bus_id(int device, char* buf, int len) {
    if (hipDeviceGetPCIBusId(buf, len, device) != hipSuccess) return -1;
    return 0;
}

const char* sk_last_error(void) { return g_last_error.c_str(); }

void* sk_host_alloc(int64_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, (size_t)bytes, hipHostMallocDefault) != hipSuccess) {
        p = aligned_alloc(4096, ((size_t)bytes + 4095) & ~(size_t)4095);  // no GPU: plain memory
    }
    return p;
}

void sk_host_free(void* p) {
    if (!p) return;
    if (hipHostFree(p) != hipSuccess) free(p);
}

void* sk_h264_create(const sk_h264_config* c) {
    if (!c || c->width < 16 || c->height < 16 || (c->width & 1) || (c->height & 1)) {
        set_last_error("invalid encoder geometry (width/height must be even and >= 16)");
        return nullptr;
    }
    if (c->stripe_height > 0 && (c->stripe_height % 16) != 0) {
        set_last_error("stripe_height must be a multiple of 16");
        return nullptr;
    }
    // the HIP intra/deblock wavefronts run one wave per MB row of a stripe (+1 producer wave)
    // in one workgroup: at most 15 rows (1024 threads). Same limit on the CPU reference so
    // both backends accept the same configurations.
    if (c->stripe_height > 240) {
        set_last_error("stripe_height must be <= 240 (15 macroblock rows per stripe)");
        return nullptr;
    }
    if (c->qp < 0 || c->qp > 51 || c->paint_qp < 0 || c->paint_qp > 51) {
        set_last_error("qp out of range");
        return nullptr;
    }
    h264::EncoderConfig e = to_config(c);
    try {
        if (c->backend == 1) return create_hip_backend(e, c->device);
        return create_cpu_backend(e);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return nullptr;
    }
}

void* sk_jpeg_create(const sk_jpeg_config* c) {
    if (!c || c->width < 16 || c->height < 16 || (c->stripe_height % 16) != 0 || c->stripe_height <= 0) {
        set_last_error("invalid JPEG encoder geometry");
        return nullptr;
    }
    jpeg::JpegConfig j;
    j.width = c->width;
    j.height = c->height;
    j.stripe_height = c->stripe_height;
    j.quality = c->quality;
    j.paint_quality = c->paint_quality;
    j.use_paint_over = c->use_paint_over;
    j.paint_over_trigger = c->paint_over_trigger;
    try {
        if (c->backend == 1) return create_hip_jpeg_backend(j, c->device);
        return create_cpu_jpeg_backend(j);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return nullptr;
    }
}

void sk_h264_destroy(void* enc) { delete static_cast<EncoderBackend*>(enc); }
void sk_h264_request_keyframe(void* enc) { static_cast<EncoderBackend*>(enc)->request_keyframe(); }
void sk_h264_set_qp(void* enc, int qp, int paint_qp) { static_cast<EncoderBackend*>(enc)->set_qp(qp, paint_qp); }
void sk_h264_set_rate(void* enc, int mode, int kbps) { static_cast<EncoderBackend*>(enc)->set_rate(mode, kbps); }
int sk_h264_rc_stats(void* enc, int32_t* out, int n) {
    return (int)static_cast<EncoderBackend*>(enc)->rc_stats(out, n);
}
int sk_h264_set_overlay_image(void* enc, int slot, const uint8_t* bgra, int w, int h) {
    return static_cast<EncoderBackend*>(enc)->set_overlay_image(slot, bgra, w, h);
}
int sk_h264_set_overlay_pos(void* enc, int slot, int on, int x, int y, int tdx, int tdy) {
    return static_cast<EncoderBackend*>(enc)->set_overlay_pos(slot, on, x, y, tdx, tdy);
}

int sk_h264_encode(void* enc, const uint8_t* bgrx, int32_t stride, int32_t frame_id) {
    try {
        return static_cast<EncoderBackend*>(enc)->encode(bgrx, stride, (uint16_t)frame_id);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_submit(void* enc, const uint8_t* bgrx, int32_t stride, int32_t frame_id) {
    try {
        return static_cast<EncoderBackend*>(enc)->submit(bgrx, stride, (uint16_t)frame_id);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_wait_stream(void* enc, void* stream) {
    try {
        return static_cast<EncoderBackend*>(enc)->wait_stream(stream);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_upload(void* enc, const uint8_t* bgrx, int32_t stride, int32_t frame_id) {
    try {
        return static_cast<EncoderBackend*>(enc)->upload(bgrx, stride, (uint16_t)frame_id);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_set_upload_rows(void* enc, const int32_t* rows, int32_t n) {
    static_cast<EncoderBackend*>(enc)->set_upload_rows(rows, n);
    return 0;
}

int sk_upload_ranges(const int32_t* pairs, int32_t n, int32_t rows, int32_t* out, int32_t cap) {
    std::vector<int> v(pairs && n > 0 ? pairs : nullptr, pairs && n > 0 ? pairs + 2 * n : nullptr);
    const auto r = upload_ranges({&v}, rows);
    for (int i = 0; i < (int)r.size() && i < cap; i++) {
        out[2 * i] = r[i].first;
        out[2 * i + 1] = r[i].second;
    }
    return (int)r.size();
}

int sk_h264_encode_yuv(void* enc, int32_t fmt, const uint8_t* y, int32_t ys, const uint8_t* u, int32_t us,
                       const uint8_t* v, int32_t vs, int32_t on_device, int32_t frame_id) {
    if (fmt != h264::YUV_I420 && fmt != h264::YUV_NV12) {
        set_last_error("planar format must be 1 (I420) or 2 (NV12)");
        return -1;
    }
    h264::YuvInput in;
    in.fmt = fmt;
    in.p[0] = y; in.p[1] = u; in.p[2] = fmt == h264::YUV_NV12 ? u : v;
    in.stride[0] = ys; in.stride[1] = us; in.stride[2] = fmt == h264::YUV_NV12 ? us : vs;
    try {
        return static_cast<EncoderBackend*>(enc)->encode_yuv(in, on_device, (uint16_t)frame_id);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_launch(void* enc) {
    try {
        return static_cast<EncoderBackend*>(enc)->launch();
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_finish(void* enc) {
    try {
        return static_cast<EncoderBackend*>(enc)->finish();
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int64_t sk_h264_state_bytes(void* enc) { return static_cast<EncoderBackend*>(enc)->state_bytes(); }

int sk_h264_export_state(void* enc, void* dst, int32_t on_device) {
    try {
        return static_cast<EncoderBackend*>(enc)->export_state(dst, on_device);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_import_state(void* enc, const void* src, int32_t on_device) {
    try {
        return static_cast<EncoderBackend*>(enc)->import_state(src, on_device);
    } catch (const std::exception& ex) {
        set_last_error(ex.what());
        return -1;
    }
}

int sk_h264_get_packet(void* enc, int32_t i, sk_packet* out) {
    auto* e = static_cast<EncoderBackend*>(enc);
    if (i < 0 || i >= (int)e->packets_.size()) return -1;
    const h264::EncodedPacket& p = e->packets_[i];
    out->data = p.data.data();
    out->size = (int32_t)p.data.size();
    out->y = p.y;
    out->w = p.w;
    out->h = p.h;
    out->key = p.key;
    return 0;
}

int64_t sk_h264_debug_buffer(void* enc, const char* name, void* dst, int64_t cap) {
    return static_cast<EncoderBackend*>(enc)->debug_buffer(name, dst, cap);
}

int sk_h264_stage_times(void* enc, float* dst, int32_t n) {
    return static_cast<EncoderBackend*>(enc)->stage_times(dst, n);
}

}  // extern "C"
