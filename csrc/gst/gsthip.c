/* libgsthip: GStreamer 1.x elements over the gfx950 media engine (libselkies_native.so).
 *
 *   hiph264enc  H.264 Constrained Baseline (CAVLC), slices of stripe-height rows
 *   hiph265enc  HEVC Main (CABAC, WPP), slices of CTB rows
 *   hipav1enc   AV1 Main 8-bit 4:2:0 (tiles), OBU temporal units
 *   hipconvert  BGRx / BGRA -> I420 (BT.709, the encoders' K1 colour conversion)
 *
 * The encoders are GstVideoEncoder subclasses taking BGRx / BGRA (what ximagesrc and
 * the capture path deliver); conversion to 4:2:0 is fused into the encoder's first
 * kernel, so a pipeline needs no videoconvert in front of them. They replace the
 * reference's encoder elements in its GStreamer graph (legacy/gstwebrtc_app.py:
 * 200-1001, x264enc / nvh264enc / vah264enc at :352-663, x265enc at :667-683,
 * svtav1enc / av1enc / rav1enc at :724-783) with the reference's property names:
 * bitrate (kbit/s), key-int-max (gop-size alias), rate-control, qp, plus
 * backend=auto|cpu|hip and device. Output buffers are byte-stream access units
 * (Annex B for H.264 / H.265, low-overhead OBUs for AV1): the native encoder's packet
 * minus its 10-byte stripe header, byte for byte.
 */
#include <gst/gst.h>
#include <gst/base/gstbasetransform.h>
#include <gst/video/video.h>
#include <gst/video/gstvideoencoder.h>
#include <string.h>

#include "../runtime/sk_api.h"

#define PACKAGE "selkies-mi355x"
#define VERSION "0.1"

GST_DEBUG_CATEGORY_STATIC(gst_hip_debug);
#define GST_CAT_DEFAULT gst_hip_debug

/* ------------------------------------------------------------------ enums */
typedef enum { HIP_BACKEND_AUTO = 0, HIP_BACKEND_CPU = 1, HIP_BACKEND_HIP = 2 } GstHipBackend;
typedef enum { HIP_RC_CQP = 0, HIP_RC_CRF = 1, HIP_RC_CBR = 2 } GstHipRateControl;

static GType gst_hip_backend_get_type(void) {
    static gsize id = 0;
    static const GEnumValue values[] = {
        {HIP_BACKEND_AUTO, "HIP when a device is present, else the CPU reference", "auto"},
        {HIP_BACKEND_CPU, "CPU reference encoder", "cpu"},
        {HIP_BACKEND_HIP, "gfx950 HIP kernels", "hip"},
        {0, NULL, NULL}};
    if (g_once_init_enter(&id)) g_once_init_leave(&id, g_enum_register_static("GstHipBackend", values));
    return (GType)id;
}

static GType gst_hip_rate_control_get_type(void) {
    static gsize id = 0;
    static const GEnumValue values[] = {
        {HIP_RC_CQP, "Constant QP", "cqp"},
        {HIP_RC_CRF, "Constant rate factor (complexity-adaptive QP around qp)", "crf"},
        {HIP_RC_CBR, "Constant bitrate (bitrate kbit/s)", "cbr"},
        {0, NULL, NULL}};
    if (g_once_init_enter(&id)) g_once_init_leave(&id, g_enum_register_static("GstHipRateControl", values));
    return (GType)id;
}

static int resolve_backend(int b) {
    if (b == HIP_BACKEND_CPU) return 0;
    if (b == HIP_BACKEND_HIP) return 1;
    return sk_hip_device_count() > 0 ? 1 : 0;
}

/* ------------------------------------------------------------------ encoders */
enum { CODEC_H264 = 0, CODEC_H265 = 1, CODEC_AV1 = 2 };

typedef struct {
    GstVideoEncoder parent;
    void* enc;
    GstVideoCodecState* in_state;
    /* properties */
    guint bitrate;
    gint rate_control; /* -1: cbr when bitrate > 0, else crf */
    guint qp;
    gint key_int_max;
    gint backend;
    gint device;
    guint stripe_height;
    /* state */
    gint since_key;
    guint16 frame_id;
    gint last_kbps, last_mode;
} GstHipEnc;

typedef struct {
    GstVideoEncoderClass parent_class;
    gint codec;
} GstHipEncClass;

enum {
    PROP_0,
    PROP_BITRATE,
    PROP_RATE_CONTROL,
    PROP_QP,
    PROP_KEY_INT_MAX,
    PROP_GOP_SIZE,
    PROP_BACKEND,
    PROP_DEVICE,
    PROP_STRIPE_HEIGHT,
};

static GstElementClass* hipenc_parent_class = NULL;

#define HIPENC(o) ((GstHipEnc*)(o))
#define HIPENC_CODEC(o) (((GstHipEncClass*)G_OBJECT_GET_CLASS(o))->codec)

static int hipenc_rc_mode(const GstHipEnc* s) {
    if (s->rate_control >= 0) return s->rate_control == HIP_RC_CBR && s->bitrate == 0 ? HIP_RC_CRF : s->rate_control;
    return s->bitrate > 0 ? HIP_RC_CBR : HIP_RC_CRF;
}

static void hipenc_set_property(GObject* obj, guint id, const GValue* v, GParamSpec* ps) {
    GstHipEnc* s = HIPENC(obj);
    GST_OBJECT_LOCK(s);
    switch (id) {
        case PROP_BITRATE: s->bitrate = g_value_get_uint(v); break;
        case PROP_RATE_CONTROL: s->rate_control = g_value_get_enum(v); break;
        case PROP_QP: s->qp = g_value_get_uint(v); break;
        case PROP_KEY_INT_MAX:
        case PROP_GOP_SIZE: s->key_int_max = g_value_get_int(v); break;
        case PROP_BACKEND: s->backend = g_value_get_enum(v); break;
        case PROP_DEVICE: s->device = g_value_get_int(v); break;
        case PROP_STRIPE_HEIGHT: s->stripe_height = g_value_get_uint(v); break;
        default: G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps); break;
    }
    GST_OBJECT_UNLOCK(s);
}

static void hipenc_get_property(GObject* obj, guint id, GValue* v, GParamSpec* ps) {
    GstHipEnc* s = HIPENC(obj);
    GST_OBJECT_LOCK(s);
    switch (id) {
        case PROP_BITRATE: g_value_set_uint(v, s->bitrate); break;
        case PROP_RATE_CONTROL: g_value_set_enum(v, hipenc_rc_mode(s)); break;
        case PROP_QP: g_value_set_uint(v, s->qp); break;
        case PROP_KEY_INT_MAX:
        case PROP_GOP_SIZE: g_value_set_int(v, s->key_int_max); break;
        case PROP_BACKEND: g_value_set_enum(v, s->backend); break;
        case PROP_DEVICE: g_value_set_int(v, s->device); break;
        case PROP_STRIPE_HEIGHT: g_value_set_uint(v, s->stripe_height); break;
        default: G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps); break;
    }
    GST_OBJECT_UNLOCK(s);
}

static void hipenc_close_encoder(GstHipEnc* s) {
    if (s->enc) sk_h264_destroy(s->enc);
    s->enc = NULL;
}

static gboolean hipenc_stop(GstVideoEncoder* e) {
    GstHipEnc* s = HIPENC(e);
    hipenc_close_encoder(s);
    if (s->in_state) gst_video_codec_state_unref(s->in_state);
    s->in_state = NULL;
    return TRUE;
}

static GstCaps* hipenc_src_caps(int codec) {
    switch (codec) {
        case CODEC_H264:
            return gst_caps_from_string(
                "video/x-h264, stream-format=(string)byte-stream, alignment=(string)au, "
                "profile=(string)constrained-baseline");
        case CODEC_H265:
            return gst_caps_from_string(
                "video/x-h265, stream-format=(string)byte-stream, alignment=(string)au, profile=(string)main");
        default:
            return gst_caps_from_string("video/x-av1, stream-format=(string)obu-stream, alignment=(string)tu");
    }
}

static gboolean hipenc_set_format(GstVideoEncoder* e, GstVideoCodecState* state) {
    GstHipEnc* s = HIPENC(e);
    const int codec = HIPENC_CODEC(e);
    const GstVideoInfo* info = &state->info;
    hipenc_close_encoder(s);
    if (s->in_state) gst_video_codec_state_unref(s->in_state);
    s->in_state = gst_video_codec_state_ref(state);

    sk_h264_config c;
    memset(&c, 0, sizeof(c));
    c.width = GST_VIDEO_INFO_WIDTH(info) & ~1;
    c.height = GST_VIDEO_INFO_HEIGHT(info) & ~1;
    c.stripe_height = (int32_t)(s->stripe_height ? s->stripe_height : 64);
    c.fullframe = 1; /* one picture per buffer: stripes are its slices */
    c.qp = (int32_t)s->qp;
    c.paint_qp = (int32_t)s->qp;
    c.use_paint_over = 0;
    c.paint_over_trigger = 15;
    c.paint_over_burst = 5;
    c.damage_threshold = 10;
    c.damage_duration = 20;
    c.me_range = 64;
    c.me_iters = 24;
    c.scenecut = 1;
    c.fps = GST_VIDEO_INFO_FPS_N(info) > 0 && GST_VIDEO_INFO_FPS_D(info) > 0
                ? (float)GST_VIDEO_INFO_FPS_N(info) / (float)GST_VIDEO_INFO_FPS_D(info)
                : 60.f;
    c.device = s->device;
    c.backend = resolve_backend(s->backend);
    c.codec = codec;
    c.tile_cols_log2 = c.tile_rows_log2 = -1;
    c.rc_mode = hipenc_rc_mode(s);
    c.bitrate_kbps = (int32_t)s->bitrate;
    if (s->backend == HIP_BACKEND_HIP && sk_hip_device_count() <= 0) {
        GST_ELEMENT_ERROR(s, RESOURCE, NOT_FOUND, ("backend=hip but no HIP device"), (NULL));
        return FALSE;
    }
    s->enc = sk_h264_create(&c);
    if (!s->enc) {
        GST_ELEMENT_ERROR(s, LIBRARY, INIT, ("encoder init failed"), ("%s", sk_last_error()));
        return FALSE;
    }
    s->last_mode = c.rc_mode;
    s->last_kbps = c.bitrate_kbps;
    s->since_key = 0;
    GST_INFO_OBJECT(s, "%dx%d @ %.2f fps, codec %d, backend %s, rc %d, %u kbit/s", c.width, c.height, c.fps,
                    codec, c.backend ? "hip" : "cpu", c.rc_mode, s->bitrate);

    GstCaps* caps = hipenc_src_caps(codec);
    GstVideoCodecState* out = gst_video_encoder_set_output_state(e, caps, state);
    gst_video_codec_state_unref(out);
    /* one frame in, one access unit out: no reordering; latency of one frame interval */
    GstClockTime lat = gst_util_uint64_scale_int(GST_SECOND, GST_VIDEO_INFO_FPS_D(info) > 0 ? GST_VIDEO_INFO_FPS_D(info) : 1,
                                                 GST_VIDEO_INFO_FPS_N(info) > 0 ? GST_VIDEO_INFO_FPS_N(info) : 60);
    gst_video_encoder_set_latency(e, lat, lat);
    return gst_video_encoder_negotiate(e);
}

static GstFlowReturn hipenc_handle_frame(GstVideoEncoder* e, GstVideoCodecFrame* frame) {
    GstHipEnc* s = HIPENC(e);
    if (!s->enc || !s->in_state) {
        gst_video_encoder_finish_frame(e, frame);
        return GST_FLOW_NOT_NEGOTIATED;
    }
    /* rate / bitrate changes (e.g. a congestion controller writing bitrate) */
    GST_OBJECT_LOCK(s);
    const int mode = hipenc_rc_mode(s), kbps = (int)s->bitrate, kim = s->key_int_max;
    GST_OBJECT_UNLOCK(s);
    if (mode != s->last_mode || (mode == HIP_RC_CBR && kbps != s->last_kbps)) {
        sk_h264_set_rate(s->enc, mode, kbps);
        s->last_mode = mode;
        s->last_kbps = kbps;
    }
    if (GST_VIDEO_CODEC_FRAME_IS_FORCE_KEYFRAME(frame) || (kim > 0 && s->since_key >= kim))
        sk_h264_request_keyframe(s->enc);

    GstVideoFrame vf;
    if (!gst_video_frame_map(&vf, &s->in_state->info, frame->input_buffer, GST_MAP_READ)) {
        gst_video_encoder_finish_frame(e, frame);
        return GST_FLOW_ERROR;
    }
    const int n = sk_h264_encode(s->enc, (const uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&vf, 0),
                                 GST_VIDEO_FRAME_PLANE_STRIDE(&vf, 0), s->frame_id++);
    gst_video_frame_unmap(&vf);
    if (n < 0) {
        GST_ELEMENT_ERROR(s, STREAM, ENCODE, ("encode failed"), ("%s", sk_last_error()));
        gst_video_encoder_finish_frame(e, frame);
        return GST_FLOW_ERROR;
    }
    gsize total = 0;
    gboolean key = FALSE;
    for (int i = 0; i < n; i++) {
        sk_packet p;
        if (sk_h264_get_packet(s->enc, i, &p) == 0 && p.size > 10) {
            total += (gsize)(p.size - 10);
            key |= p.key != 0;
        }
    }
    if (total == 0) { /* nothing coded (no change in a striped picture): drop */
        return gst_video_encoder_finish_frame(e, frame);
    }
    GstBuffer* out = gst_buffer_new_allocate(NULL, total, NULL);
    GstMapInfo m;
    gst_buffer_map(out, &m, GST_MAP_WRITE);
    gsize o = 0;
    for (int i = 0; i < n; i++) {
        sk_packet p;
        if (sk_h264_get_packet(s->enc, i, &p) == 0 && p.size > 10) {
            memcpy(m.data + o, p.data + 10, (size_t)(p.size - 10));
            o += (gsize)(p.size - 10);
        }
    }
    gst_buffer_unmap(out, &m);
    frame->output_buffer = out;
    if (key) {
        GST_VIDEO_CODEC_FRAME_SET_SYNC_POINT(frame);
        s->since_key = 1;
    } else {
        GST_VIDEO_CODEC_FRAME_UNSET_SYNC_POINT(frame);
        s->since_key++;
    }
    return gst_video_encoder_finish_frame(e, frame);
}

static void hipenc_finalize(GObject* obj) {
    hipenc_stop(GST_VIDEO_ENCODER(obj));
    G_OBJECT_CLASS(hipenc_parent_class)->finalize(obj);
}

static void hipenc_init(GTypeInstance* inst, gpointer klass) {
    (void)klass;
    GstHipEnc* s = HIPENC(inst);
    s->enc = NULL;
    s->in_state = NULL;
    s->bitrate = 0;
    s->rate_control = -1;
    s->qp = 25;
    s->key_int_max = -1;
    s->backend = HIP_BACKEND_AUTO;
    s->device = 0;
    s->stripe_height = 64;
    s->since_key = 0;
    s->frame_id = 0;
}

static const char* kEncNames[3] = {"hiph264enc", "hiph265enc", "hipav1enc"};
static const char* kEncLong[3] = {"H.264 encoder (gfx950 HIP)", "H.265 encoder (gfx950 HIP)",
                                  "AV1 encoder (gfx950 HIP)"};

static void hipenc_class_init(gpointer klass, gpointer data) {
    GObjectClass* oc = G_OBJECT_CLASS(klass);
    GstElementClass* ec = GST_ELEMENT_CLASS(klass);
    GstVideoEncoderClass* vc = GST_VIDEO_ENCODER_CLASS(klass);
    const int codec = GPOINTER_TO_INT(data);
    ((GstHipEncClass*)klass)->codec = codec;
    hipenc_parent_class = (GstElementClass*)g_type_class_peek_parent(klass);
    oc->set_property = hipenc_set_property;
    oc->get_property = hipenc_get_property;
    oc->finalize = hipenc_finalize;
    vc->stop = hipenc_stop;
    vc->set_format = hipenc_set_format;
    vc->handle_frame = hipenc_handle_frame;

    const GParamFlags rw = (GParamFlags)(G_PARAM_READWRITE | G_PARAM_STATIC_STRINGS);
    g_object_class_install_property(oc, PROP_BITRATE,
        g_param_spec_uint("bitrate", "Bitrate", "Target bitrate in kbit/s (CBR; 0 = quality mode)", 0, 2000000, 0, rw));
    g_object_class_install_property(oc, PROP_RATE_CONTROL,
        g_param_spec_enum("rate-control", "Rate control", "Rate control mode (default: cbr when bitrate > 0, else crf)",
                          gst_hip_rate_control_get_type(), HIP_RC_CRF, rw));
    g_object_class_install_property(oc, PROP_QP,
        g_param_spec_uint("qp", "QP", "Constant QP / CRF value (H.264 scale; AV1 maps it to a qindex)", 0, 51, 25, rw));
    g_object_class_install_property(oc, PROP_KEY_INT_MAX,
        g_param_spec_int("key-int-max", "Key-frame interval", "Maximum frames between key frames (-1 / 0 = only on request)",
                         -1, G_MAXINT, -1, rw));
    g_object_class_install_property(oc, PROP_GOP_SIZE,
        g_param_spec_int("gop-size", "GOP size", "Alias of key-int-max (nvh264enc / vah264enc name)", -1, G_MAXINT, -1, rw));
    g_object_class_install_property(oc, PROP_BACKEND,
        g_param_spec_enum("backend", "Backend", "Encoder back end", gst_hip_backend_get_type(), HIP_BACKEND_AUTO, rw));
    g_object_class_install_property(oc, PROP_DEVICE,
        g_param_spec_int("device", "Device", "HIP device ordinal", 0, 63, 0, rw));
    g_object_class_install_property(oc, PROP_STRIPE_HEIGHT,
        g_param_spec_uint("stripe-height", "Stripe height", "Rows per slice (multiple of 16)", 16, 4096, 64, rw));

    GstCaps* sink = gst_caps_from_string(
        "video/x-raw, format=(string){ BGRx, BGRA }, width=(int)[ 16, 8192 ], height=(int)[ 16, 8192 ], "
        "framerate=(fraction)[ 0/1, MAX ]");
    gst_element_class_add_pad_template(ec, gst_pad_template_new("sink", GST_PAD_SINK, GST_PAD_ALWAYS, sink));
    gst_caps_unref(sink);
    GstCaps* src = hipenc_src_caps(codec);
    gst_element_class_add_pad_template(ec, gst_pad_template_new("src", GST_PAD_SRC, GST_PAD_ALWAYS, src));
    gst_caps_unref(src);
    gst_element_class_set_static_metadata(ec, kEncLong[codec], "Codec/Encoder/Video/Hardware",
                                          "Encodes BGRx frames on the MI355X (gfx950) media kernels",
                                          "selkies-mi355x");
}

static GType hipenc_register(int codec) {
    GTypeInfo info;
    memset(&info, 0, sizeof(info));
    info.class_size = sizeof(GstHipEncClass);
    info.class_init = hipenc_class_init;
    info.class_data = GINT_TO_POINTER(codec);
    info.instance_size = sizeof(GstHipEnc);
    info.instance_init = hipenc_init;
    static const char* tnames[3] = {"GstHipH264Enc", "GstHipH265Enc", "GstHipAv1Enc"};
    return g_type_register_static(GST_TYPE_VIDEO_ENCODER, tnames[codec], &info, (GTypeFlags)0);
}

/* ------------------------------------------------------------------ hipconvert */
typedef struct {
    GstBaseTransform parent;
    void* conv;
    gint backend, device;
    GstVideoInfo in_info, out_info;
} GstHipConvert;
typedef struct {
    GstBaseTransformClass parent_class;
} GstHipConvertClass;

enum { CPROP_0, CPROP_BACKEND, CPROP_DEVICE };
static GstBaseTransformClass* hipconv_parent_class = NULL;

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

static GstCaps* hipconv_transform_caps(GstBaseTransform* t, GstPadDirection dir, GstCaps* caps, GstCaps* filter) {
    (void)t;
    GstCaps* res = gst_caps_new_empty();
    for (guint i = 0; i < gst_caps_get_size(caps); i++) {
        GstStructure* st = gst_structure_copy(gst_caps_get_structure(caps, i));
        if (dir == GST_PAD_SINK) {
            gst_structure_set(st, "format", G_TYPE_STRING, "I420", NULL);
        } else {
            GValue list = G_VALUE_INIT, v = G_VALUE_INIT;
            g_value_init(&list, GST_TYPE_LIST);
            g_value_init(&v, G_TYPE_STRING);
            g_value_set_string(&v, "BGRx");
            gst_value_list_append_value(&list, &v);
            g_value_set_string(&v, "BGRA");
            gst_value_list_append_value(&list, &v);
            gst_structure_take_value(st, "format", &list);
            g_value_unset(&v);
        }
        gst_structure_remove_fields(st, "colorimetry", "chroma-site", NULL);
        res = gst_caps_merge_structure(res, st);
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
    if (s->conv) sk_convert_destroy(s->conv);
    s->conv = sk_convert_create(GST_VIDEO_INFO_WIDTH(&s->in_info), GST_VIDEO_INFO_HEIGHT(&s->in_info), 0,
                                resolve_backend(s->backend), s->device);
    if (!s->conv) {
        GST_ELEMENT_ERROR(s, LIBRARY, INIT, ("converter init failed"), ("%s", sk_last_error()));
        return FALSE;
    }
    return TRUE;
}

static GstFlowReturn hipconv_transform(GstBaseTransform* t, GstBuffer* inbuf, GstBuffer* outbuf) {
    GstHipConvert* s = (GstHipConvert*)t;
    GstVideoFrame fi, fo;
    if (!gst_video_frame_map(&fi, &s->in_info, inbuf, GST_MAP_READ)) return GST_FLOW_ERROR;
    if (!gst_video_frame_map(&fo, &s->out_info, outbuf, GST_MAP_WRITE)) {
        gst_video_frame_unmap(&fi);
        return GST_FLOW_ERROR;
    }
    const int rc = sk_convert_run(s->conv, (const uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&fi, 0),
                                  GST_VIDEO_FRAME_PLANE_STRIDE(&fi, 0), (uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&fo, 0),
                                  GST_VIDEO_FRAME_PLANE_STRIDE(&fo, 0), (uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&fo, 1),
                                  GST_VIDEO_FRAME_PLANE_STRIDE(&fo, 1), (uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&fo, 2),
                                  GST_VIDEO_FRAME_PLANE_STRIDE(&fo, 2));
    gst_video_frame_unmap(&fo);
    gst_video_frame_unmap(&fi);
    return rc == 0 ? GST_FLOW_OK : GST_FLOW_ERROR;
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
}

static void hipconv_class_init(gpointer klass, gpointer data) {
    (void)data;
    GObjectClass* oc = G_OBJECT_CLASS(klass);
    GstElementClass* ec = GST_ELEMENT_CLASS(klass);
    GstBaseTransformClass* bc = GST_BASE_TRANSFORM_CLASS(klass);
    hipconv_parent_class = (GstBaseTransformClass*)g_type_class_peek_parent(klass);
    oc->set_property = hipconv_set_property;
    oc->get_property = hipconv_get_property;
    bc->transform_caps = hipconv_transform_caps;
    bc->set_caps = hipconv_set_caps;
    bc->transform = hipconv_transform;
    bc->stop = hipconv_stop;
    bc->passthrough_on_same_caps = FALSE;
    const GParamFlags rw = (GParamFlags)(G_PARAM_READWRITE | G_PARAM_STATIC_STRINGS);
    g_object_class_install_property(oc, CPROP_BACKEND,
        g_param_spec_enum("backend", "Backend", "Conversion back end", gst_hip_backend_get_type(), HIP_BACKEND_AUTO, rw));
    g_object_class_install_property(oc, CPROP_DEVICE, g_param_spec_int("device", "Device", "HIP device ordinal", 0, 63, 0, rw));
    GstCaps* sink = gst_caps_from_string(
        "video/x-raw, format=(string){ BGRx, BGRA }, width=(int)[ 2, 8192 ], height=(int)[ 2, 8192 ], "
        "framerate=(fraction)[ 0/1, MAX ]");
    GstCaps* src = gst_caps_from_string(
        "video/x-raw, format=(string)I420, width=(int)[ 2, 8192 ], height=(int)[ 2, 8192 ], "
        "framerate=(fraction)[ 0/1, MAX ]");
    gst_element_class_add_pad_template(ec, gst_pad_template_new("sink", GST_PAD_SINK, GST_PAD_ALWAYS, sink));
    gst_element_class_add_pad_template(ec, gst_pad_template_new("src", GST_PAD_SRC, GST_PAD_ALWAYS, src));
    gst_caps_unref(sink);
    gst_caps_unref(src);
    gst_element_class_set_static_metadata(ec, "BGRx to I420 converter (gfx950 HIP)", "Filter/Converter/Video/Hardware",
                                          "BT.709 limited-range colour conversion on the MI355X", "selkies-mi355x");
}

static GType hipconv_register(void) {
    GTypeInfo info;
    memset(&info, 0, sizeof(info));
    info.class_size = sizeof(GstHipConvertClass);
    info.class_init = hipconv_class_init;
    info.instance_size = sizeof(GstHipConvert);
    info.instance_init = hipconv_init;
    return g_type_register_static(GST_TYPE_BASE_TRANSFORM, "GstHipConvert", &info, (GTypeFlags)0);
}

/* ------------------------------------------------------------------ plugin */
static gboolean plugin_init(GstPlugin* plugin) {
    GST_DEBUG_CATEGORY_INIT(gst_hip_debug, "hip", 0, "gfx950 media elements");
    for (int c = 0; c < 3; c++)
        if (!gst_element_register(plugin, kEncNames[c], GST_RANK_PRIMARY + 1, hipenc_register(c))) return FALSE;
    return gst_element_register(plugin, "hipconvert", GST_RANK_NONE, hipconv_register());
}

GST_PLUGIN_DEFINE(GST_VERSION_MAJOR, GST_VERSION_MINOR, hip, "gfx950 (MI355X) media elements: H.264 / H.265 / AV1 encoders, BGRx->I420",
                  plugin_init, VERSION, "LGPL", PACKAGE, "selkies-mi355x")
