// C ABI of libselkies_native.so (loaded from Python with ctypes, exactly like
// the reference loads pixelflux/pcmflux; see selkies.py:64-92, 2846-2964).
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sk_h264_config {
    int32_t width, height, stripe_height, fullframe, full_range;
    int32_t qp, paint_qp, use_paint_over, paint_over_trigger, paint_over_burst;
    int32_t streaming_mode, damage_threshold, damage_duration;
    int32_t me_range, me_iters, scenecut;
    float fps;
    int32_t device;   // HIP device ordinal for the GPU backend
    int32_t backend;  // 0 = CPU reference, 1 = HIP (gfx950)
    int32_t deblock;  // in-loop deblocking: 0 = default (automatic: slices at QP >= 34), 1 on, 2 automatic, < 0 off
    int32_t me_full;  // MFMA +-16 exhaustive search candidate: 0 = default (on), > 0 on, < 0 off
    int32_t shared_copy;  // > 0: H2D on the device's shared copy stream (bands of one frame)
    int32_t src_width, src_height;  // capture size if it differs (K2 resample in K1); 0 = width/height
    int32_t num_refs;               // reference pictures (sliding-window DPB): 0/1 = one, 2 = two
    int32_t codec;                  // 0 = H.264 (stripes or full frame), 1 = HEVC Main (full frame, WPP),
                                    // 2 = AV1 Main (full frame, tiles)
    int32_t aq_strength;            // H.264 MB-level adaptive QP, Q4 (16 = 1.0); 0 = off
    int32_t subpel;                 // H.264 quarter-pel motion refinement: 0 = default (on), < 0 off
    int32_t intra4x4;               // H.264 Intra4x4 (I_NxN) macroblocks in I slices: > 0 on, else off
    int32_t tile_cols_log2;         // AV1 tile columns / rows (log2); -1 = automatic
    int32_t tile_rows_log2;
    int32_t rc_mode;                // K10 rate control: 0 = constant QP, 1 = CRF (qp = CRF), 2 = CBR
    int32_t bitrate_kbps;           // CBR target (VBV = 1.5 frame intervals)
} sk_h264_config;

typedef struct sk_packet {
    const uint8_t* data;  // 0x04 stripe packet (10-byte header + Annex-B)
    int32_t size;
    int32_t y, w, h, key;
} sk_packet;

const char* sk_version(void);
int sk_hip_device_count(void);
// PCI address ("0000:c1:00.0") of a HIP device, for NUMA placement of host buffers.
int sk_hip_pci_bus_id(int device, char* buf, int len);

void* sk_h264_create(const sk_h264_config* cfg);
void sk_h264_destroy(void* enc);
void sk_h264_request_keyframe(void* enc);
// Rate control: QP of changed stripes / paint-over from the next frame (<= 0 keeps the value).
void sk_h264_set_qp(void* enc, int qp, int paint_qp);
// K10 rate control from the next frame: mode 0 constant QP, 1 CRF, 2 CBR at kbps.
void sk_h264_set_rate(void* enc, int mode, int kbps);
// Rate-control state words (codec/ratecontrol.h RcState); returns the count or -1.
int sk_h264_rc_stats(void* enc, int32_t* out, int n);
// K12/K13 overlays blended during colour conversion (csrc/codec/overlay.h): slot 0 =
// watermark, 1 = cursor; premultiplied BGRA, at most 512x512. Positions apply to frames
// uploaded after the call; tdx/tdy > 0 tile the image with that period. 0 = ok, < 0 =
// not supported by this encoder (JPEG).
int sk_h264_set_overlay_image(void* enc, int slot, const uint8_t* bgra, int w, int h);
int sk_h264_set_overlay_pos(void* enc, int slot, int on, int x, int y, int tdx, int tdy);
// Encodes one BGRx frame; returns the number of packets (or < 0 on error).
int sk_h264_encode(void* enc, const uint8_t* bgrx, int32_t stride_bytes, int32_t frame_id);
// Planar 4:2:0 input instead of BGRx (GStreamer NV12 / I420): fmt 1 = I420 (y, u, v planes),
// 2 = NV12 (y plane, interleaved uv in u / us); on_device: the planes are HIP device memory
// (of the encoder's GPU for the HIP backend). Returns the packet count like sk_h264_encode.
int sk_h264_encode_yuv(void* enc, int32_t fmt, const uint8_t* y, int32_t ys, const uint8_t* u, int32_t us,
                       const uint8_t* v, int32_t vs, int32_t on_device, int32_t frame_id);
// Split encode: submit queues the frame (bgrx must stay valid until finish), finish
// waits and returns the packet count (then sk_h264_get_packet as after sk_h264_encode).
int sk_h264_submit(void* enc, const uint8_t* bgrx, int32_t stride, int32_t frame_id);
int sk_h264_finish(void* enc);
// submit = upload + launch. upload(n+1) may run while frame n encodes (its copy
// overlaps n's kernels); call launch() for it after sk_h264_finish of frame n.
int sk_h264_upload(void* enc, const uint8_t* bgrx, int32_t stride, int32_t frame_id);
// The next sk_h264_upload waits on the device for the work queued on `stream` (a HIP
// stream of the encoder's device), instead of a host synchronisation.
int sk_h264_wait_stream(void* enc, void* stream);
// Damage of the next sk_h264_upload: n [y0, y1) row ranges changed since the previous
// upload (n < 0: unknown -> full copy). The HIP backend then copies only those rows.
int sk_h264_set_upload_rows(void* enc, const int32_t* rows, int32_t n);
// The row ranges a damage-driven upload copies for `n` pairs (clamped to [0, rows),
// 16-row bands); returns the range count, the first `cap` go to out as pairs.
int sk_upload_ranges(const int32_t* pairs, int32_t n, int32_t rows, int32_t* out, int32_t cap);
int sk_h264_launch(void* enc);
// Session state snapshot (codec/h264_encoder.h StateHeader layout, identical for the
// CPU and HIP backends): move a session between GPUs / processes without an IDR.
// on_device = 1: `dst`/`src` is device memory on the encoder's GPU (HIP backend).
int64_t sk_h264_state_bytes(void* enc);
int sk_h264_export_state(void* enc, void* dst, int32_t on_device);
int sk_h264_import_state(void* enc, const void* src, int32_t on_device);
int sk_h264_get_packet(void* enc, int32_t i, sk_packet* out);
// Debug / test access to internal buffers ("src_y", "rec_y", "ref_y", "mbs", "coefs", "me", ...).
int64_t sk_h264_debug_buffer(void* enc, const char* name, void* dst, int64_t cap);
// Per-stage timings of the last frame in microseconds (GPU backend), n entries.
int sk_h264_stage_times(void* enc, float* dst, int32_t n);

const char* sk_last_error(void);

// Standalone BGRx / BGRA -> I420 converter (BT.709; the encoders' K1 arithmetic), backend
// 0 = CPU, 1 = HIP on `device`; run returns 0 on success. Odd sizes repeat the last
// column / row into the chroma average; chroma planes are (w+1)/2 x (h+1)/2.
void* sk_convert_create(int w, int h, int full_range, int backend, int device);
int sk_convert_run(void* conv, const uint8_t* bgrx, int32_t stride, uint8_t* y, int32_t ys, uint8_t* u, int32_t us,
                   uint8_t* v, int32_t vs);
// General form: BGRx source in host or device memory; fmt 1 = I420, 2 = NV12 (u = the
// interleaved UV plane, v unused); destination planes in host or device memory.
int sk_convert_run_ex(void* conv, const uint8_t* bgrx, int32_t stride, int32_t src_on_device, int32_t fmt,
                      uint8_t* y, int32_t ys, uint8_t* u, int32_t us, uint8_t* v, int32_t vs,
                      int32_t dst_on_device);
void sk_convert_destroy(void* conv);

// Frame sources for hipximagesrc (csrc/runtime/source_api.cpp): kind 0 = X11 MIT-SHM
// region (x, y, w, h of `display`, XFixes cursor when show_pointer), 1 / 2 / 3 =
// synthetic motion / desktop / noise frames (headless hosts; seed). grab() returns BGRx
// rows valid until the next grab, the stride, and the changed row ranges (pairs, at
// most cap; *nrows = -1 when the source cannot tell).
void* sk_source_open(int32_t kind, const char* display, int32_t x, int32_t y, int32_t w, int32_t h,
                     int32_t show_pointer, uint32_t seed);
const uint8_t* sk_source_grab(void* src, int32_t* stride, int32_t* rows, int32_t cap, int32_t* nrows);
const char* sk_source_name(void* src);
void sk_source_close(void* src);
// Device memory of the GStreamer HIPMemory allocator. kind: 0 host->device,
// 1 device->host, 2 device->device, 3 either (unified addressing). 0 on success.
void* sk_dev_alloc(int32_t device, int64_t bytes);
void sk_dev_free(int32_t device, void* p);
int sk_dev_copy(int32_t device, void* dst, const void* src, int64_t bytes, int32_t kind);
int sk_dev_copy2d(int32_t device, void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width,
                  int64_t height, int32_t kind);

typedef struct sk_jpeg_config {
    int32_t width, height, stripe_height;
    int32_t quality, paint_quality, use_paint_over, paint_over_trigger;
    int32_t device;
    int32_t backend;  // 0 = CPU reference, 1 = HIP
} sk_jpeg_config;

// JPEG stripe encoder; shares sk_h264_encode / get_packet / destroy (generic encoder handle).
void* sk_jpeg_create(const sk_jpeg_config* cfg);

// ---- capture session (pixelflux-compatible ScreenCapture) ----
typedef struct sk_capture_settings {
    // pixelflux CaptureSettings fields (selkies.py:2925-2962)
    int32_t capture_width, capture_height, capture_x, capture_y;
    double target_fps;
    int32_t capture_cursor, debug_logging, output_mode;
    int32_t jpeg_quality, paint_over_jpeg_quality, use_paint_over_quality;
    int32_t paint_over_trigger_frames, damage_block_threshold, damage_block_duration;
    int32_t h264_crf, h264_paintover_crf, h264_paintover_burst_frames;
    int32_t h264_fullcolor, h264_streaming_mode, h264_fullframe;
    int32_t use_cpu, vaapi_render_node_index;
    const char* watermark_path;
    int32_t watermark_location_enum;
    // extensions
    int32_t device;          // HIP device ordinal
    int32_t stripe_height;   // 0 -> 64
    int32_t source;          // -1 auto (X11 if reachable), 0 X11 only, 1/2/3 synthetic motion/desktop/noise
    const char* display;     // X display name (nullptr -> $DISPLAY)
    int32_t output_width, output_height;  // H.264 stream size if it differs from the capture (K2); 0 = same
    int32_t step_mode;       // 1: encode only frames granted by sk_capture_run, unpaced (benchmarks)
    const uint8_t* pool;     // source 4: caller-owned BGRx frames (pool_frames x capture_height rows)
    int32_t pool_frames, pool_stride, pool_phase;
    // H.264 quality tools (0 = defaults: AQ off, quarter-pel on, Intra4x4 off)
    int32_t h264_aq_strength;  // MB-level adaptive QP, Q4 (16 = x264 aq-strength 1.0)
    int32_t h264_subpel;       // < 0: integer-pel motion only
    int32_t h264_intra4x4;     // > 0: I_NxN macroblocks in keyframes
    // K10 rate control (codec/ratecontrol.h): 0 = constant QP (h264_crf as QP),
    // 1 = CRF (complexity-adaptive QP around h264_crf), 2 = CBR at h264_bitrate_kbps
    int32_t h264_rc_mode;
    int32_t h264_bitrate_kbps;
    // < 0: no exhaustive +-16 search candidate, diamond search only (x264 "ultrafast"-like
    // CPU plumbing; with h264_subpel < 0 the CPU encoder runs 640x480 at ~55 fps on one core)
    int32_t h264_me_full;
} sk_capture_settings;

typedef struct sk_stripe_result {
    int32_t type;            // 0 = JPEG stripe, 1 = H.264 stripe/frame, 2 = HEVC stripe/frame
    int32_t stripe_y_start;
    int32_t stripe_height;
    int32_t size;
    uint8_t* data;
    int32_t frame_id;
    int64_t grab_ns;         // extension: CLOCK_MONOTONIC time the frame was grabbed (latency tracing)
} sk_stripe_result;

typedef void (*sk_stripe_cb)(sk_stripe_result*, void*);
// One call per encoded frame with all of its stripe packets (n may be 0).
typedef void (*sk_frame_cb)(const sk_stripe_result*, int32_t n, void*);

void* sk_capture_create(void);
void sk_capture_destroy(void* c);
// Starts the capture thread; cb runs on that thread once per stripe packet.
int sk_capture_start(void* c, const sk_capture_settings* s, sk_stripe_cb cb, void* user);
// Same session, one callback per frame instead of one per stripe.
int sk_capture_start_frames(void* c, const sk_capture_settings* s, sk_frame_cb cb, void* user);
// Step mode: grant `frames` more frames; wait blocks until every granted frame is
// delivered (0), times out (1, timeout_ms >= 0) or the session stopped (-1).
void sk_capture_run(void* c, int64_t frames);
int sk_capture_wait(void* c, int timeout_ms);
// Capture-to-packets latency in ms of the most recent frames (oldest first).
int sk_capture_latencies(void* c, float* out, int cap, int reset);
void sk_capture_stop(void* c);
void sk_capture_request_keyframe(void* c);
void sk_capture_set_qp(void* c, int qp, int paint_qp);
void sk_capture_set_rate(void* c, int mode, int kbps);   // K10: 0 CQP, 1 CRF, 2 CBR at kbps
// Moves a running HIP session's encoder to GPU `device` between two frames, carrying the
// inter-frame state GPU-to-GPU: 0 stream continued (P frames), 1 moved with a key frame,
// -1 not moved (sk_last_error). Blocks up to timeout_ms (<= 0: 10 s).
int sk_capture_move(void* c, int device, int timeout_ms);
int sk_capture_device(void* c);   // GPU the session encodes on (-1: CPU)
// frames, mean encode ms, bytes, packets, source (1 = X11, 0 = synthetic), last encode ms
void sk_capture_stats(void* c, double* out, int n);
// Premultiplied BGRA watermark composited before encoding (location enum in capture.cpp).
void sk_capture_set_watermark(void* c, const uint8_t* bgra, int w, int h, int location);

// ---- X11 input injection (XTest) and cursor watching (XFixes) ----
// cursor_only=1 opens a connection that only watches cursor changes.
void* sk_x11_input_open(const char* display, int cursor_only);
void sk_x11_input_close(void* h);
int sk_x11_key(void* h, uint32_t keysym, int down, int shift_held);
int sk_x11_motion(void* h, int x, int y);
int sk_x11_motion_rel(void* h, int dx, int dy);
int sk_x11_button(void* h, int button, int down);
void sk_x11_screen_size(void* h, int* w, int* hh);
int sk_x11_cursor_wait(void* h, int timeout_ms);
int sk_x11_cursor_image(void* h, uint64_t* serial, int* w, int* hh, int* xhot, int* yhot, uint32_t* argb, int cap);

// ---- Audio capture (pcmflux engine, audio_capture.cpp) ----
enum { SK_AUDIO_OPUS = 0, SK_AUDIO_PCM = 1 };
typedef struct sk_audio_settings {
    const char* device_name;        // PulseAudio source; "synthetic[:hz]" = paced sine tone
    int32_t sample_rate, channels, opus_bitrate, frame_duration_ms;
    int32_t use_vbr, use_silence_gate;
    int32_t codec;                  // SK_AUDIO_OPUS (libopus) or SK_AUDIO_PCM (raw s16le)
    int32_t synthetic_silence_frames;  // synthetic source: leading all-zero frames
} sk_audio_settings;
typedef struct sk_audio_chunk { int32_t size; const uint8_t* data; } sk_audio_chunk;
typedef void (*sk_audio_cb)(sk_audio_chunk*, void*);
// bit 0: libpulse-simple loadable, bit 1: libopus loadable
int sk_audio_available(void);
void* sk_audio_create(void);
void sk_audio_destroy(void* a);
// 0 = capture thread running; < 0 = error (sk_audio_error)
int sk_audio_start(void* a, const sk_audio_settings* s, sk_audio_cb cb, void* user);
void sk_audio_stop(void* a);
// frames read, packets delivered, bytes delivered, frames dropped by the silence gate
void sk_audio_stats(void* a, double* out, int n);
const char* sk_audio_error(void* a);

// ---- AV1 multi-symbol entropy coder (codec/av1_ec.h), test entry ----
int sk_av1_ec_encode(const int32_t* kind, const int32_t* ctx, const int32_t* sym, int n, uint16_t* cdfs,
                     const int32_t* nsym, int adapt, uint8_t* out, int cap);

// Page-locked host memory (capture buffers / frame pools): DMA-able by HIP.
void* sk_host_alloc(int64_t bytes);
void sk_host_free(void* p);

// Telephony audio codecs (codec/telephony.cpp): G.711 u-law (alaw = 0) / A-law,
// G.722 64 kbit/s (16 kHz PCM, 2 samples per byte).
int sk_g711_encode(int alaw, const int16_t* pcm, int n, uint8_t* out);
int sk_g711_decode(int alaw, const uint8_t* in, int n, int16_t* pcm);
void* sk_g722_create(void);
void sk_g722_destroy(void* h);
int sk_g722_encode(void* h, const int16_t* pcm, int n, uint8_t* out);
int sk_g722_decode(void* h, const uint8_t* in, int n, int16_t* pcm);

#ifdef __cplusplus
}
#endif
