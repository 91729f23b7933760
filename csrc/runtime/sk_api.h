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
} sk_h264_config;

typedef struct sk_packet {
    const uint8_t* data;  // 0x04 stripe packet (10-byte header + Annex-B)
    int32_t size;
    int32_t y, w, h, key;
} sk_packet;

const char* sk_version(void);
int sk_hip_device_count(void);

void* sk_h264_create(const sk_h264_config* cfg);
void sk_h264_destroy(void* enc);
void sk_h264_request_keyframe(void* enc);
// Encodes one BGRx frame; returns the number of packets (or < 0 on error).
int sk_h264_encode(void* enc, const uint8_t* bgrx, int32_t stride_bytes, int32_t frame_id);
int sk_h264_get_packet(void* enc, int32_t i, sk_packet* out);
// Debug / test access to internal buffers ("src_y", "rec_y", "ref_y", "mbs", "coefs", "me", ...).
int64_t sk_h264_debug_buffer(void* enc, const char* name, void* dst, int64_t cap);
// Per-stage timings of the last frame in microseconds (GPU backend), n entries.
int sk_h264_stage_times(void* enc, float* dst, int32_t n);

const char* sk_last_error(void);

// Page-locked host memory (capture buffers / frame pools): DMA-able by HIP.
void* sk_host_alloc(int64_t bytes);
void sk_host_free(void* p);

#ifdef __cplusplus
}
#endif
