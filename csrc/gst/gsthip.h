/* Shared declarations of the libgsthip elements (csrc/gst/*.c).
 *
 * Device memory: frames that live on the GPU travel between the elements as
 * GstMemory of type "HIPMemory" (caps feature memory:HIPMemory), the analogue of the
 * reference's CUDAMemory caps between cudaupload / cudaconvert / nvh264enc
 * (legacy/gstwebrtc_app.py:261-284). One memory holds a whole frame laid out like its
 * GstVideoInfo (GstVideoMeta attached), in hipMalloc'd memory of the allocator's
 * device; mapping it from the host stages a copy (read: device -> host, write: host ->
 * device on unmap), so any element can still look at it.
 */
#pragma once
#include <gst/gst.h>
#include <gst/base/gstbasetransform.h>
#include <gst/base/gstpushsrc.h>
#include <gst/video/video.h>
#include <gst/video/gstvideoencoder.h>

#include "../runtime/sk_api.h"

G_BEGIN_DECLS

GST_DEBUG_CATEGORY_EXTERN(gst_hip_debug);

#define GST_HIP_MEMORY_TYPE "HIPMemory"
#define GST_CAPS_FEATURE_MEMORY_HIP "memory:HIPMemory"
/* the raw formats every element of the plugin moves around */
#define GST_HIP_RAW_FORMATS "{ BGRx, BGRA, I420, NV12 }"

typedef enum { HIP_BACKEND_AUTO = 0, HIP_BACKEND_CPU = 1, HIP_BACKEND_HIP = 2 } GstHipBackend;
GType gst_hip_backend_get_type(void);
/* 1: HIP kernels, 0: the CPU reference (auto: HIP when a device is present) */
int gst_hip_resolve_backend(int backend);

/* ---- HIPMemory ---- */
typedef struct {
    GstMemory mem;
    void* dev;          /* device pointer (maxsize bytes) */
    gint device;
    guint8* host;       /* staging copy for host maps (lazily allocated) */
} GstHipMemory;

GstAllocator* gst_hip_allocator_get(gint device); /* one per device, owned by the plugin */
gboolean gst_is_hip_memory(GstMemory* mem);
/* A buffer whose single memory is HIPMemory: its device pointer (memory offset
 * applied) and device, else NULL. */
guint8* gst_hip_buffer_device_ptr(GstBuffer* buf, gint* device);
/* A frame buffer of `info` in HIPMemory of `device`, with a GstVideoMeta. */
GstBuffer* gst_hip_buffer_new_video(const GstVideoInfo* info, gint device);
/* Plane offsets / strides of a frame buffer (its GstVideoMeta, else `info`). */
void gst_hip_buffer_planes(GstBuffer* buf, const GstVideoInfo* info, gsize* offsets, gint* strides);
/* Does any structure of `caps` carry the memory:HIPMemory feature? */
gboolean gst_hip_caps_have_memory(GstCaps* caps);

GType gst_hip_upload_get_type(void);
GType gst_hip_download_get_type(void);
GType gst_hip_convert_get_type(void);
GType gst_hip_ximage_src_get_type(void);
GType gst_hip_enc_register(int codec);

G_END_DECLS
