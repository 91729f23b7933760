/* hipconvert: BGRx / BGRA -> I420 or NV12 with the encoders' K1 arithmetic (BT.709,
 * codec/color.h), on the GPU (k_bgrx_i420) or the CPU reference. Either side may be
 * system memory or memory:HIPMemory; with HIPMemory on both sides the frame never
 * leaves the device (the reference's cudaconvert in front of nvh264enc,
 * legacy/gstwebrtc_app.py:261-284). Output caps prefer HIPMemory, then system memory,
 * so `hipconvert ! hiph264enc` stays on the GPU and `hipconvert ! video/x-raw,
 * format=NV12 ! x264enc` gets system memory. */
#include "gsthip.h"

#include <string.h>

typedef struct {
    GstBaseTransform parent;
    void* conv;
    gint backend, device;
    GstVideoInfo in_info, out_info;
    gboolean out_hip;
} GstHipConvert;
typedef struct {
    GstBaseTransformClass parent_class;
} GstHipConvertClass;

enum { CPROP_0, CPROP_BACKEND, CPROP_DEVICE };

static void hipconv_set_property(GObject* obj, guint id, const GValue* v, GParamSpec* ps) {
    GstHipConvert* s = (GstHipConvert*)obj;
    switch (id) {
        case CPROP_BACKEND: s->backend = g_value_get_enum(v); break;
        case CPROP_DEVICE: s->device = g_value_get_int(v); break;
        default: G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps); break;
    }
}
static void hipconv_get_property(GObject* obj, guint id, GValue* v, GParamSpec* ps) {
    GstHipConvert* s = (GstHipConvert*)obj;
    switch (id) {
        case CPROP_BACKEND: g_value_set_enum(v, s->backend); break;
        case CPROP_DEVICE: g_value_set_int(v, s->device); break;
        default: G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps); break;
    }
}

static void set_format_list(GstStructure* st, const char* a, const char* b) {
    GValue list = G_VALUE_INIT, v = G_VALUE_INIT;
    g_value_init(&list, GST_TYPE_LIST);
    g_value_init(&v, G_TYPE_STRING);
    g_value_set_string(&v, a);
    gst_value_list_append_value(&list, &v);
    g_value_set_string(&v, b);
    gst_value_list_append_value(&list, &v);
    gst_structure_take_value(st, "format", &list);
    g_value_unset(&v);
}

/* sink -> src: {I420, NV12} in HIPMemory first, then in system memory; src -> sink:
 * {BGRx, BGRA} in either memory */
static GstCaps* hipconv_transform_caps(GstBaseTransform* t, GstPadDirection dir, GstCaps* caps, GstCaps* filter) {
    (void)t;
    GstCaps* res = gst_caps_new_empty();
    /* no HIP device (CPU-only host): system memory only */
    const int first = sk_hip_device_count() > 0 ? 0 : 1;
    for (int pass = first; pass < 2; pass++) {
        const gboolean hip = pass == 0;
        for (guint i = 0; i < gst_caps_get_size(caps); i++) {
            GstStructure* st = gst_structure_copy(gst_caps_get_structure(caps, i));
            if (dir == GST_PAD_SINK) set_format_list(st, "I420", "NV12");
            else set_format_list(st, "BGRx", "BGRA");
            gst_structure_remove_fields(st, "colorimetry", "chroma-site", NULL);
            GstCapsFeatures* f = hip ? gst_caps_features_new(GST_CAPS_FEATURE_MEMORY_HIP, NULL)
                                     : gst_caps_features_new_empty();
            res = gst_caps_merge_structure_full(res, st, f);
        }
    }
    if (filter) {
        GstCaps* f = gst_caps_intersect_full(filter, res, GST_CAPS_INTERSECT_FIRST);
        gst_caps_unref(res);
        res = f;
    }
    return res;
}

static gboolean hipconv_set_caps(GstBaseTransform* t, GstCaps* in, GstCaps* out) {
    GstHipConvert* s = (GstHipConvert*)t;
    if (!gst_video_info_from_caps(&s->in_info, in) || !gst_video_info_from_caps(&s->out_info, out)) return FALSE;
    if (GST_VIDEO_INFO_WIDTH(&s->in_info) != GST_VIDEO_INFO_WIDTH(&s->out_info) ||
        GST_VIDEO_INFO_HEIGHT(&s->in_info) != GST_VIDEO_INFO_HEIGHT(&s->out_info))
        return FALSE;
    s->out_hip = gst_hip_caps_have_memory(out);
    if (s->conv) sk_convert_destroy(s->conv);
    s->conv = sk_convert_create(GST_VIDEO_INFO_WIDTH(&s->in_info), GST_VIDEO_INFO_HEIGHT(&s->in_info), 0,
                                gst_hip_resolve_backend(s->backend), s->device);
    if (!s->conv) {
        GST_ELEMENT_ERROR(s, LIBRARY, INIT, ("converter init failed"), ("%s", sk_last_error()));
        return FALSE;
    }
    return TRUE;
}

static GstFlowReturn hipconv_prepare_output_buffer(GstBaseTransform* t, GstBuffer* in, GstBuffer** out) {
    GstHipConvert* s = (GstHipConvert*)t;
    *out = s->out_hip ? gst_hip_buffer_new_video(&s->out_info, s->device)
                      : gst_buffer_new_allocate(NULL, GST_VIDEO_INFO_SIZE(&s->out_info), NULL);
    if (!*out) return GST_FLOW_ERROR;
    gst_buffer_copy_into(*out, in, (GstBufferCopyFlags)(GST_BUFFER_COPY_FLAGS | GST_BUFFER_COPY_TIMESTAMPS), 0, -1);
    return GST_FLOW_OK;
}

static GstFlowReturn hipconv_transform(GstBaseTransform* t, GstBuffer* inbuf, GstBuffer* outbuf) {
    GstHipConvert* s = (GstHipConvert*)t;
    const int fmt = GST_VIDEO_INFO_FORMAT(&s->out_info) == GST_VIDEO_FORMAT_NV12 ? 2 : 1;
    const gboolean hip = gst_hip_resolve_backend(s->backend) == 1;
    /* source: device pointer when the input is HIPMemory and the converter runs on HIP */
    GstVideoFrame fi, fo;
    gboolean mapped_in = FALSE, mapped_out = FALSE;
    const guint8* src = hip ? gst_hip_buffer_device_ptr(inbuf, NULL) : NULL;
    gint src_stride = 0;
    if (src) {
        gsize off[GST_VIDEO_MAX_PLANES];
        gint st[GST_VIDEO_MAX_PLANES];
        gst_hip_buffer_planes(inbuf, &s->in_info, off, st);
        src += off[0];
        src_stride = st[0];
    } else {
        if (!gst_video_frame_map(&fi, &s->in_info, inbuf, GST_MAP_READ)) return GST_FLOW_ERROR;
        mapped_in = TRUE;
        src = (const guint8*)GST_VIDEO_FRAME_PLANE_DATA(&fi, 0);
        src_stride = GST_VIDEO_FRAME_PLANE_STRIDE(&fi, 0);
    }
    guint8* dp[3] = {NULL, NULL, NULL};
    gint ds[3] = {0, 0, 0};
    guint8* dbase = gst_hip_buffer_device_ptr(outbuf, NULL);
    const gboolean dst_dev = dbase != NULL;
    if (dst_dev) {
        gsize off[GST_VIDEO_MAX_PLANES];
        gint st[GST_VIDEO_MAX_PLANES];
        gst_hip_buffer_planes(outbuf, &s->out_info, off, st);
        for (guint p = 0; p < GST_VIDEO_INFO_N_PLANES(&s->out_info); p++) {
            dp[p] = dbase + off[p];
            ds[p] = st[p];
        }
    } else {
        if (!gst_video_frame_map(&fo, &s->out_info, outbuf, GST_MAP_WRITE)) {
            if (mapped_in) gst_video_frame_unmap(&fi);
            return GST_FLOW_ERROR;
        }
        mapped_out = TRUE;
        for (guint p = 0; p < GST_VIDEO_INFO_N_PLANES(&s->out_info); p++) {
            dp[p] = (guint8*)GST_VIDEO_FRAME_PLANE_DATA(&fo, p);
            ds[p] = GST_VIDEO_FRAME_PLANE_STRIDE(&fo, p);
        }
    }
    const int rc = sk_convert_run_ex(s->conv, src, src_stride, mapped_in ? 0 : 1, fmt, dp[0], ds[0], dp[1], ds[1],
                                     dp[2], ds[2], dst_dev ? 1 : 0);
    if (mapped_out) gst_video_frame_unmap(&fo);
    if (mapped_in) gst_video_frame_unmap(&fi);
    if (rc != 0) {
        GST_ELEMENT_ERROR(s, STREAM, FAILED, ("conversion failed"), ("%s", sk_last_error()));
        return GST_FLOW_ERROR;
    }
    return GST_FLOW_OK;
}

static gboolean hipconv_stop(GstBaseTransform* t) {
    GstHipConvert* s = (GstHipConvert*)t;
    if (s->conv) sk_convert_destroy(s->conv);
    s->conv = NULL;
    return TRUE;
}

static void hipconv_init(GTypeInstance* inst, gpointer klass) {
    (void)klass;
    GstHipConvert* s = (GstHipConvert*)inst;
    s->conv = NULL;
    s->backend = HIP_BACKEND_AUTO;
    s->device = 0;
    s->out_hip = FALSE;
}

static void hipconv_class_init(gpointer klass, gpointer data) {
    (void)data;
    GObjectClass* oc = G_OBJECT_CLASS(klass);
    GstElementClass* ec = GST_ELEMENT_CLASS(klass);
    GstBaseTransformClass* bc = GST_BASE_TRANSFORM_CLASS(klass);
    oc->set_property = hipconv_set_property;
    oc->get_property = hipconv_get_property;
    bc->transform_caps = hipconv_transform_caps;
    bc->set_caps = hipconv_set_caps;
    bc->prepare_output_buffer = hipconv_prepare_output_buffer;
    bc->transform = hipconv_transform;
    bc->stop = hipconv_stop;
    bc->passthrough_on_same_caps = FALSE;
    const GParamFlags rw = (GParamFlags)(G_PARAM_READWRITE | G_PARAM_STATIC_STRINGS);
    g_object_class_install_property(oc, CPROP_BACKEND,
        g_param_spec_enum("backend", "Backend", "Conversion back end", gst_hip_backend_get_type(), HIP_BACKEND_AUTO, rw));
    g_object_class_install_property(oc, CPROP_DEVICE, g_param_spec_int("device", "Device", "HIP device ordinal", 0, 63, 0, rw));
    GstCaps* sink = gst_caps_from_string(
        "video/x-raw(" GST_CAPS_FEATURE_MEMORY_HIP "), format=(string){ BGRx, BGRA }, width=(int)[ 2, 8192 ], "
        "height=(int)[ 2, 8192 ], framerate=(fraction)[ 0/1, MAX ]; "
        "video/x-raw, format=(string){ BGRx, BGRA }, width=(int)[ 2, 8192 ], height=(int)[ 2, 8192 ], "
        "framerate=(fraction)[ 0/1, MAX ]");
    GstCaps* src = gst_caps_from_string(
        "video/x-raw(" GST_CAPS_FEATURE_MEMORY_HIP "), format=(string){ I420, NV12 }, width=(int)[ 2, 8192 ], "
        "height=(int)[ 2, 8192 ], framerate=(fraction)[ 0/1, MAX ]; "
        "video/x-raw, format=(string){ I420, NV12 }, width=(int)[ 2, 8192 ], height=(int)[ 2, 8192 ], "
        "framerate=(fraction)[ 0/1, MAX ]");
    gst_element_class_add_pad_template(ec, gst_pad_template_new("sink", GST_PAD_SINK, GST_PAD_ALWAYS, sink));
    gst_element_class_add_pad_template(ec, gst_pad_template_new("src", GST_PAD_SRC, GST_PAD_ALWAYS, src));
    gst_caps_unref(sink);
    gst_caps_unref(src);
    gst_element_class_set_static_metadata(ec, "BGRx to I420 / NV12 converter (gfx950 HIP)",
                                          "Filter/Converter/Video/Hardware",
                                          "BT.709 limited-range colour conversion on the MI355X, system or HIP memory",
                                          "selkies-mi355x");
}

GType gst_hip_convert_get_type(void) {
    static gsize id = 0;
    if (g_once_init_enter(&id)) {
        GTypeInfo info;
        memset(&info, 0, sizeof(info));
        info.class_size = sizeof(GstHipConvertClass);
        info.class_init = hipconv_class_init;
        info.instance_size = sizeof(GstHipConvert);
        info.instance_init = hipconv_init;
        g_once_init_leave(&id, g_type_register_static(GST_TYPE_BASE_TRANSFORM, "GstHipConvert", &info, (GTypeFlags)0));
    }
    return (GType)id;
}
