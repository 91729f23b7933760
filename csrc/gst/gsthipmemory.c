/* HIPMemory: a GstAllocator over hipMalloc (through libselkies_native's sk_dev_* ABI),
 * and the hipupload / hipdownload elements that move raw frames between system
 * memory and memory:HIPMemory caps (cudaupload / cudadownload in the reference's
 * nvh264enc graph, legacy/gstwebrtc_app.py:261-284).
 *
 * Freed device blocks are kept on a small per-allocator list and reused for the next
 * frame of the same size: a hipMalloc / hipFree pair per frame would cost more than
 * the copy it serves. */
#include "gsthip.h"

#include <string.h>

/* ------------------------------------------------------------------ allocator */
typedef struct {
    GstAllocator parent;
    gint device;
    GMutex lock;
    GSList* cache; /* GstHipBlock* of freed memories */
} GstHipAllocator;
typedef struct {
    GstAllocatorClass parent_class;
} GstHipAllocatorClass;

typedef struct {
    void* dev;
    gsize size;
} GstHipBlock;

#define HIP_CACHE_MAX 8

static GType gst_hip_allocator_get_type(void);

static void* hip_block_take(GstHipAllocator* a, gsize size) {
    void* p = NULL;
    g_mutex_lock(&a->lock);
    for (GSList* l = a->cache; l; l = l->next) {
        GstHipBlock* b = (GstHipBlock*)l->data;
        if (b->size == size) {
            p = b->dev;
            a->cache = g_slist_delete_link(a->cache, l);
            g_free(b);
            break;
        }
    }
    g_mutex_unlock(&a->lock);
    return p ? p : sk_dev_alloc(a->device, (int64_t)size);
}

static void hip_block_give(GstHipAllocator* a, void* dev, gsize size) {
    g_mutex_lock(&a->lock);
    if (g_slist_length(a->cache) < HIP_CACHE_MAX) {
        GstHipBlock* b = g_new(GstHipBlock, 1);
        b->dev = dev;
        b->size = size;
        a->cache = g_slist_prepend(a->cache, b);
        dev = NULL;
    }
    g_mutex_unlock(&a->lock);
    if (dev) sk_dev_free(a->device, dev);
}

static GstMemory* hip_mem_new(GstHipAllocator* a, GstMemory* parent, void* dev, gsize maxsize, gsize offset,
                              gsize size) {
    GstHipMemory* m = g_slice_new0(GstHipMemory);
    gst_memory_init(GST_MEMORY_CAST(m), GST_MEMORY_FLAG_NO_SHARE, GST_ALLOCATOR_CAST(a), parent, maxsize, 0, offset,
                    size);
    m->dev = dev;
    m->device = a->device;
    m->host = NULL;
    return GST_MEMORY_CAST(m);
}

static GstMemory* hip_alloc(GstAllocator* alloc, gsize size, GstAllocationParams* params) {
    (void)params;
    GstHipAllocator* a = (GstHipAllocator*)alloc;
    void* dev = hip_block_take(a, size);
    if (!dev) {
        GST_ERROR("HIPMemory: allocation of %" G_GSIZE_FORMAT " bytes failed: %s", size, sk_last_error());
        return NULL;
    }
    return hip_mem_new(a, NULL, dev, size, 0, size);
}

static void hip_free(GstAllocator* alloc, GstMemory* mem) {
    GstHipMemory* m = (GstHipMemory*)mem;
    hip_block_give((GstHipAllocator*)alloc, m->dev, mem->maxsize);
    g_free(m->host);
    g_slice_free(GstHipMemory, m);
}

/* host view: read maps download the device bytes, write maps upload at unmap */
static gpointer hip_mem_map_full(GstMemory* mem, GstMapInfo* info, gsize maxsize) {
    GstHipMemory* m = (GstHipMemory*)mem;
    if (!m->host) m->host = g_malloc(mem->maxsize);
    if ((info->flags & GST_MAP_READ) && sk_dev_copy(m->device, m->host, m->dev, (int64_t)maxsize, 1) != 0) {
        GST_ERROR("HIPMemory: download for a host map failed: %s", sk_last_error());
        return NULL;
    }
    return m->host;
}

static void hip_mem_unmap_full(GstMemory* mem, GstMapInfo* info) {
    GstHipMemory* m = (GstHipMemory*)mem;
    if ((info->flags & GST_MAP_WRITE) && sk_dev_copy(m->device, m->dev, m->host, (int64_t)mem->maxsize, 0) != 0)
        GST_ERROR("HIPMemory: upload after a host write map failed: %s", sk_last_error());
}

static GstMemory* hip_mem_copy(GstMemory* mem, gssize offset, gssize size) {
    GstHipMemory* m = (GstHipMemory*)mem;
    GstHipAllocator* a = (GstHipAllocator*)mem->allocator;
    if (size == -1) size = (gssize)mem->size - offset;
    void* dev = hip_block_take(a, (gsize)size);
    if (!dev) return NULL;
    if (sk_dev_copy(m->device, dev, (guint8*)m->dev + mem->offset + offset, size, 2) != 0) {
        hip_block_give(a, dev, (gsize)size);
        return NULL;
    }
    return hip_mem_new(a, NULL, dev, (gsize)size, 0, (gsize)size);
}

static GstMemory* hip_mem_share(GstMemory* mem, gssize offset, gssize size) {
    (void)mem;
    (void)offset;
    (void)size;
    return NULL; /* GST_MEMORY_FLAG_NO_SHARE: whole frames only */
}

static void gst_hip_allocator_finalize(GObject* obj) {
    GstHipAllocator* a = (GstHipAllocator*)obj;
    for (GSList* l = a->cache; l; l = l->next) {
        GstHipBlock* b = (GstHipBlock*)l->data;
        sk_dev_free(a->device, b->dev);
        g_free(b);
    }
    g_slist_free(a->cache);
    g_mutex_clear(&a->lock);
    G_OBJECT_CLASS(g_type_class_peek_parent(G_OBJECT_GET_CLASS(obj)))->finalize(obj);
}

static void gst_hip_allocator_class_init(gpointer klass, gpointer data) {
    (void)data;
    GstAllocatorClass* ac = GST_ALLOCATOR_CLASS(klass);
    ac->alloc = hip_alloc;
    ac->free = hip_free;
    G_OBJECT_CLASS(klass)->finalize = gst_hip_allocator_finalize;
}

static void gst_hip_allocator_init(GTypeInstance* inst, gpointer klass) {
    (void)klass;
    GstAllocator* alloc = GST_ALLOCATOR_CAST(inst);
    GstHipAllocator* a = (GstHipAllocator*)inst;
    alloc->mem_type = GST_HIP_MEMORY_TYPE;
    alloc->mem_map_full = hip_mem_map_full;
    alloc->mem_unmap_full = hip_mem_unmap_full;
    alloc->mem_copy = hip_mem_copy;
    alloc->mem_share = hip_mem_share;
    alloc->mem_is_span = NULL;
    GST_OBJECT_FLAG_SET(alloc, GST_ALLOCATOR_FLAG_CUSTOM_ALLOC);
    g_mutex_init(&a->lock);
    a->cache = NULL;
    a->device = 0;
}

static GType gst_hip_allocator_get_type(void) {
    static gsize id = 0;
    if (g_once_init_enter(&id)) {
        GTypeInfo info;
        memset(&info, 0, sizeof(info));
        info.class_size = sizeof(GstHipAllocatorClass);
        info.class_init = gst_hip_allocator_class_init;
        info.instance_size = sizeof(GstHipAllocator);
        info.instance_init = gst_hip_allocator_init;
        g_once_init_leave(&id, g_type_register_static(GST_TYPE_ALLOCATOR, "GstHipAllocator", &info, (GTypeFlags)0));
    }
    return (GType)id;
}

#define HIP_MAX_DEVICES 64
static GstAllocator* g_allocators[HIP_MAX_DEVICES];
G_LOCK_DEFINE_STATIC(allocators);

GstAllocator* gst_hip_allocator_get(gint device) {
    if (device < 0 || device >= HIP_MAX_DEVICES) return NULL;
    G_LOCK(allocators);
    if (!g_allocators[device]) {
        GstHipAllocator* a = (GstHipAllocator*)g_object_new(gst_hip_allocator_get_type(), NULL);
        a->device = device;
        gst_object_ref_sink(a);
        GST_OBJECT_FLAG_SET(a, GST_OBJECT_FLAG_MAY_BE_LEAKED);
        g_allocators[device] = GST_ALLOCATOR_CAST(a);
    }
    GstAllocator* r = g_allocators[device];
    G_UNLOCK(allocators);
    return r;
}

gboolean gst_is_hip_memory(GstMemory* mem) {
    return mem && mem->allocator && g_type_is_a(G_OBJECT_TYPE(mem->allocator), gst_hip_allocator_get_type());
}

guint8* gst_hip_buffer_device_ptr(GstBuffer* buf, gint* device) {
    if (!buf || gst_buffer_n_memory(buf) != 1) return NULL;
    GstMemory* mem = gst_buffer_peek_memory(buf, 0);
    if (!gst_is_hip_memory(mem)) return NULL;
    GstHipMemory* m = (GstHipMemory*)mem;
    if (device) *device = m->device;
    return (guint8*)m->dev + mem->offset;
}

GstBuffer* gst_hip_buffer_new_video(const GstVideoInfo* info, gint device) {
    GstAllocator* a = gst_hip_allocator_get(device);
    if (!a) return NULL;
    GstMemory* mem = gst_allocator_alloc(a, GST_VIDEO_INFO_SIZE(info), NULL);
    if (!mem) return NULL;
    GstBuffer* buf = gst_buffer_new();
    gst_buffer_append_memory(buf, mem);
    gsize offsets[GST_VIDEO_MAX_PLANES];
    gint strides[GST_VIDEO_MAX_PLANES];
    for (guint p = 0; p < GST_VIDEO_INFO_N_PLANES(info); p++) {
        offsets[p] = GST_VIDEO_INFO_PLANE_OFFSET(info, p);
        strides[p] = GST_VIDEO_INFO_PLANE_STRIDE(info, p);
    }
    gst_buffer_add_video_meta_full(buf, GST_VIDEO_FRAME_FLAG_NONE, GST_VIDEO_INFO_FORMAT(info),
                                   GST_VIDEO_INFO_WIDTH(info), GST_VIDEO_INFO_HEIGHT(info),
                                   GST_VIDEO_INFO_N_PLANES(info), offsets, strides);
    return buf;
}

void gst_hip_buffer_planes(GstBuffer* buf, const GstVideoInfo* info, gsize* offsets, gint* strides) {
    GstVideoMeta* vm = gst_buffer_get_video_meta(buf);
    for (guint p = 0; p < GST_VIDEO_INFO_N_PLANES(info); p++) {
        offsets[p] = vm ? vm->offset[p] : GST_VIDEO_INFO_PLANE_OFFSET(info, p);
        strides[p] = vm ? vm->stride[p] : GST_VIDEO_INFO_PLANE_STRIDE(info, p);
    }
}

gboolean gst_hip_caps_have_memory(GstCaps* caps) {
    for (guint i = 0; caps && i < gst_caps_get_size(caps); i++) {
        GstCapsFeatures* f = gst_caps_get_features(caps, i);
        if (f && gst_caps_features_contains(f, GST_CAPS_FEATURE_MEMORY_HIP)) return TRUE;
    }
    return FALSE;
}

/* ------------------------------------------------------------------ hipupload / hipdownload */
typedef struct {
    GstBaseTransform parent;
    gint device;
    GstVideoInfo info;
    gboolean to_device; /* class constant: upload (TRUE) or download */
} GstHipXfer;
typedef struct {
    GstBaseTransformClass parent_class;
    gboolean to_device;
} GstHipXferClass;

enum { XPROP_0, XPROP_DEVICE };

static void hipxfer_set_property(GObject* obj, guint id, const GValue* v, GParamSpec* ps) {
    GstHipXfer* s = (GstHipXfer*)obj;
    if (id == XPROP_DEVICE) s->device = g_value_get_int(v);
    else G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps);
}
static void hipxfer_get_property(GObject* obj, guint id, GValue* v, GParamSpec* ps) {
    GstHipXfer* s = (GstHipXfer*)obj;
    if (id == XPROP_DEVICE) g_value_set_int(v, s->device);
    else G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps);
}

/* the same caps with the memory feature added (towards the device side) or removed */
static GstCaps* caps_set_hip(GstCaps* caps, gboolean hip) {
    GstCaps* res = gst_caps_new_empty();
    for (guint i = 0; i < gst_caps_get_size(caps); i++) {
        GstStructure* st = gst_structure_copy(gst_caps_get_structure(caps, i));
        GstCapsFeatures* f = hip ? gst_caps_features_new(GST_CAPS_FEATURE_MEMORY_HIP, NULL)
                                 : gst_caps_features_new_empty();
        gst_caps_append_structure_full(res, st, f);
    }
    return res;
}

static GstCaps* hipxfer_transform_caps(GstBaseTransform* t, GstPadDirection dir, GstCaps* caps, GstCaps* filter) {
    const gboolean up = ((GstHipXferClass*)G_OBJECT_GET_CLASS(t))->to_device;
    /* sink -> src: upload adds the feature, download removes it; src -> sink the reverse.
     * Without a HIP device (CPU-only host) both are passthrough in system memory. */
    const gboolean hip = (dir == GST_PAD_SINK) ? up : !up;
    GstCaps* res = sk_hip_device_count() > 0 ? caps_set_hip(caps, hip) : caps_set_hip(caps, FALSE);
    if (filter) {
        GstCaps* f = gst_caps_intersect_full(filter, res, GST_CAPS_INTERSECT_FIRST);
        gst_caps_unref(res);
        res = f;
    }
    return res;
}

static gboolean hipxfer_set_caps(GstBaseTransform* t, GstCaps* in, GstCaps* out) {
    (void)out;
    GstHipXfer* s = (GstHipXfer*)t;
    return gst_video_info_from_caps(&s->info, in);
}

static GstFlowReturn hipxfer_prepare_output_buffer(GstBaseTransform* t, GstBuffer* in, GstBuffer** out) {
    GstHipXfer* s = (GstHipXfer*)t;
    if (gst_base_transform_is_passthrough(t)) {   /* no HIP device: the input goes on as it is */
        *out = in;
        return GST_FLOW_OK;
    }
    if (s->to_device) {
        *out = gst_hip_buffer_new_video(&s->info, s->device);
        if (!*out) return GST_FLOW_ERROR;
    } else {
        *out = gst_buffer_new_allocate(NULL, GST_VIDEO_INFO_SIZE(&s->info), NULL);
    }
    gst_buffer_copy_into(*out, in, (GstBufferCopyFlags)(GST_BUFFER_COPY_FLAGS | GST_BUFFER_COPY_TIMESTAMPS), 0, -1);
    return GST_FLOW_OK;
}

/* plane by plane 2D copies between the two layouts (device side: GstVideoInfo layout) */
static GstFlowReturn hipxfer_transform(GstBaseTransform* t, GstBuffer* in, GstBuffer* out) {
    GstHipXfer* s = (GstHipXfer*)t;
    const GstVideoInfo* info = &s->info;
    GstBuffer* dbuf = s->to_device ? out : in;
    GstBuffer* hbuf = s->to_device ? in : out;
    gint dev_id = s->device;
    guint8* d = gst_hip_buffer_device_ptr(dbuf, &dev_id);
    if (!d) {
        GST_ELEMENT_ERROR(s, STREAM, FAILED, ("expected a HIPMemory buffer"), (NULL));
        return GST_FLOW_ERROR;
    }
    gsize doff[GST_VIDEO_MAX_PLANES];
    gint dstr[GST_VIDEO_MAX_PLANES];
    gst_hip_buffer_planes(dbuf, info, doff, dstr);
    GstVideoFrame hf;
    if (!gst_video_frame_map(&hf, info, hbuf, s->to_device ? GST_MAP_READ : GST_MAP_WRITE)) return GST_FLOW_ERROR;
    GstFlowReturn ret = GST_FLOW_OK;
    /* both sides in the same layout (strides and plane offsets): one copy of the whole
       frame, row and plane padding included, so a round trip is byte-exact */
    gboolean same = hf.map[0].size >= GST_VIDEO_INFO_SIZE(info);
    for (guint p = 0; p < GST_VIDEO_INFO_N_PLANES(info); p++)
        same = same && GST_VIDEO_FRAME_PLANE_STRIDE(&hf, p) == dstr[p] &&
               (gsize)((guint8*)GST_VIDEO_FRAME_PLANE_DATA(&hf, p) - (guint8*)GST_VIDEO_FRAME_PLANE_DATA(&hf, 0)) ==
                   doff[p] - doff[0];
    if (same) {
        guint8* hp = (guint8*)GST_VIDEO_FRAME_PLANE_DATA(&hf, 0);
        const gint64 n = (gint64)GST_VIDEO_INFO_SIZE(info) - (gint64)GST_VIDEO_INFO_PLANE_OFFSET(info, 0);
        const int rc = s->to_device ? sk_dev_copy(dev_id, d + doff[0], hp, n, 0) : sk_dev_copy(dev_id, hp, d + doff[0], n, 1);
        if (rc != 0) {
            GST_ELEMENT_ERROR(s, RESOURCE, FAILED, ("frame copy failed"), ("%s", sk_last_error()));
            ret = GST_FLOW_ERROR;
        }
        gst_video_frame_unmap(&hf);
        return ret;
    }
    for (guint p = 0; p < GST_VIDEO_INFO_N_PLANES(info); p++) {
        const gint64 hb = GST_VIDEO_FRAME_COMP_HEIGHT(&hf, p);
        guint8* hp = (guint8*)GST_VIDEO_FRAME_PLANE_DATA(&hf, p);
        const gint hs = GST_VIDEO_FRAME_PLANE_STRIDE(&hf, p);
        /* equal strides (both sides in the GstVideoInfo layout): whole rows, padding
           included, so a round trip returns the buffer byte for byte */
        const gint64 wb = hs == dstr[p] ? (gint64)hs
                                        : (gint64)GST_VIDEO_FRAME_COMP_WIDTH(&hf, p) * GST_VIDEO_FRAME_COMP_PSTRIDE(&hf, p);
        const int rc = s->to_device ? sk_dev_copy2d(dev_id, d + doff[p], dstr[p], hp, hs, wb, hb, 0)
                                    : sk_dev_copy2d(dev_id, hp, hs, d + doff[p], dstr[p], wb, hb, 1);
        if (rc != 0) {
            GST_ELEMENT_ERROR(s, RESOURCE, FAILED, ("plane copy failed"), ("%s", sk_last_error()));
            ret = GST_FLOW_ERROR;
            break;
        }
    }
    gst_video_frame_unmap(&hf);
    return ret;
}

static void hipxfer_init(GTypeInstance* inst, gpointer klass) {
    GstHipXfer* s = (GstHipXfer*)inst;
    s->device = 0;
    s->to_device = ((GstHipXferClass*)klass)->to_device;
}

static void hipxfer_class_init(gpointer klass, gpointer data) {
    const gboolean up = GPOINTER_TO_INT(data);
    ((GstHipXferClass*)klass)->to_device = up;
    GObjectClass* oc = G_OBJECT_CLASS(klass);
    GstElementClass* ec = GST_ELEMENT_CLASS(klass);
    GstBaseTransformClass* bc = GST_BASE_TRANSFORM_CLASS(klass);
    oc->set_property = hipxfer_set_property;
    oc->get_property = hipxfer_get_property;
    bc->transform_caps = hipxfer_transform_caps;
    bc->set_caps = hipxfer_set_caps;
    bc->prepare_output_buffer = hipxfer_prepare_output_buffer;
    bc->transform = hipxfer_transform;
    bc->passthrough_on_same_caps = TRUE;   /* no HIP device: system memory in and out */
    g_object_class_install_property(oc, XPROP_DEVICE,
        g_param_spec_int("device", "Device", "HIP device ordinal", 0, 63, 0,
                         (GParamFlags)(G_PARAM_READWRITE | G_PARAM_STATIC_STRINGS)));
    GstCaps* sys = gst_caps_from_string("video/x-raw, format=(string)" GST_HIP_RAW_FORMATS
                                        ", width=(int)[ 1, 16384 ], height=(int)[ 1, 16384 ], "
                                        "framerate=(fraction)[ 0/1, MAX ]");
    GstCaps* hip = gst_caps_from_string("video/x-raw(" GST_CAPS_FEATURE_MEMORY_HIP "), format=(string)"
                                        GST_HIP_RAW_FORMATS ", width=(int)[ 1, 16384 ], height=(int)[ 1, 16384 ], "
                                        "framerate=(fraction)[ 0/1, MAX ]");
    /* the device side also takes system memory (passthrough on hosts without a HIP device) */
    GstCaps* dev = gst_caps_merge(gst_caps_ref(hip), gst_caps_ref(sys));
    gst_element_class_add_pad_template(ec, gst_pad_template_new("sink", GST_PAD_SINK, GST_PAD_ALWAYS, up ? sys : dev));
    gst_element_class_add_pad_template(ec, gst_pad_template_new("src", GST_PAD_SRC, GST_PAD_ALWAYS, up ? dev : sys));
    gst_caps_unref(sys);
    gst_caps_unref(hip);
    gst_caps_unref(dev);
    if (up)
        gst_element_class_set_static_metadata(ec, "Upload to HIP memory", "Filter/Video/Hardware",
                                              "Copies raw frames into MI355X device memory (memory:HIPMemory)",
                                              "selkies-mi355x");
    else
        gst_element_class_set_static_metadata(ec, "Download from HIP memory", "Filter/Video/Hardware",
                                              "Copies raw frames from MI355X device memory to system memory",
                                              "selkies-mi355x");
}

static GType hipxfer_register(gboolean up) {
    GTypeInfo info;
    memset(&info, 0, sizeof(info));
    info.class_size = sizeof(GstHipXferClass);
    info.class_init = hipxfer_class_init;
    info.class_data = GINT_TO_POINTER(up);
    info.instance_size = sizeof(GstHipXfer);
    info.instance_init = hipxfer_init;
    return g_type_register_static(GST_TYPE_BASE_TRANSFORM, up ? "GstHipUpload" : "GstHipDownload", &info,
                                  (GTypeFlags)0);
}

GType gst_hip_upload_get_type(void) {
    static gsize id = 0;
    if (g_once_init_enter(&id)) g_once_init_leave(&id, hipxfer_register(TRUE));
    return (GType)id;
}

GType gst_hip_download_get_type(void) {
    static gsize id = 0;
    if (g_once_init_enter(&id)) g_once_init_leave(&id, hipxfer_register(FALSE));
    return (GType)id;
}
