/* libgsthip: GStreamer 1.x elements over the gfx950 media engine (libselkies_native.so).
 *
 *   hiph264enc     H.264 Constrained Baseline (CAVLC), slices of stripe-height rows
 *   hiph265enc     HEVC Main (CABAC, WPP), slices of CTB rows
 *   hipav1enc      AV1 Main 8-bit 4:2:0 (tiles), OBU temporal units
 *   hipconvert     BGRx / BGRA -> I420 / NV12 (BT.709, the encoders' K1 colour conversion)
 *   hipupload      system memory -> memory:HIPMemory      (gsthipmemory.c)
 *   hipdownload    memory:HIPMemory -> system memory
 *   hipximagesrc   X11 MIT-SHM screen source              (gsthipximagesrc.c)
 *
 * The encoders are GstVideoEncoder subclasses taking BGRx / BGRA (what ximagesrc and the
 * capture path deliver; conversion to 4:2:0 is fused into the encoder's first kernel)
 * or I420 / NV12 (what `videoconvert ! video/x-raw,format=NV12` hands x264enc in the
 * reference, legacy/gstwebrtc_app.py:611-617), each in system memory or in
 * memory:HIPMemory (`hipupload ! hipconvert ! video/x-raw(memory:HIPMemory),format=NV12
 * ! hiph264enc`, the reference's cudaupload / cudaconvert / nvh264enc chain at :261-284:
 * the frame crosses PCIe once). They replace the reference's encoder elements in its
 * GStreamer graph (legacy/gstwebrtc_app.py:200-1001, x264enc / nvh264enc / vah264enc at
 * :352-663, x265enc at :667-683, svtav1enc / av1enc / rav1enc at :724-783) with the
 * reference's property names: bitrate (kbit/s), key-int-max (gop-size alias),
 * rate-control, qp, plus backend=auto|cpu|hip and device. Output buffers are
 * byte-stream access units (Annex B for H.264 / H.265, low-overhead OBUs for AV1): the
 * native encoder's packet minus its 10-byte stripe header, byte for byte.
 */
#include "gsthip.h"

#include <string.h>

#define PACKAGE "selkies-mi355x"
#define VERSION "0.1"

GST_DEBUG_CATEGORY(gst_hip_debug);
#define GST_CAT_DEFAULT gst_hip_debug

/* ------------------------------------------------------------------ enums */
typedef enum { HIP_RC_CQP = 0, HIP_RC_CRF = 1, HIP_RC_CBR = 2 } GstHipRateControl;

GType gst_hip_backend_get_type(void) {
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

int gst_hip_resolve_backend(int b) {
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
    c.backend = gst_hip_resolve_backend(s->backend);
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
    /* the coded size (odd input sizes lose their last column / row) */
    out->info.width = c.width;
    out->info.height = c.height;
    gst_video_codec_state_unref(out);
    /* one frame in, one access unit out: no reordering; latency of one frame interval */
    GstClockTime lat = gst_util_uint64_scale_int(GST_SECOND, GST_VIDEO_INFO_FPS_D(info) > 0 ? GST_VIDEO_INFO_FPS_D(info) : 1,
                                                 GST_VIDEO_INFO_FPS_N(info) > 0 ? GST_VIDEO_INFO_FPS_N(info) : 60);
    gst_video_encoder_set_latency(e, lat, lat);
    return gst_video_encoder_negotiate(e);
}

/* One frame through the native encoder: BGRx / BGRA or I420 / NV12 planes, from
 * device pointers when the buffer is HIPMemory and the encoder runs on HIP (no host
 * copy), else from a host map (HIPMemory maps stage a copy). Returns the packet count. */
static int hipenc_encode_buffer(GstHipEnc* s, GstBuffer* buf) {
    const GstVideoInfo* info = &s->in_state->info;
    const GstVideoFormat fmt = GST_VIDEO_INFO_FORMAT(info);
    const gboolean planar = fmt == GST_VIDEO_FORMAT_I420 || fmt == GST_VIDEO_FORMAT_NV12;
    const int yfmt = fmt == GST_VIDEO_FORMAT_NV12 ? 2 : 1;
    gint dev = -1;
    guint8* d = gst_hip_resolve_backend(s->backend) == 1 ? gst_hip_buffer_device_ptr(buf, &dev) : NULL;
    if (d && dev == s->device) {
        gsize off[GST_VIDEO_MAX_PLANES];
        gint st[GST_VIDEO_MAX_PLANES];
        gst_hip_buffer_planes(buf, info, off, st);
        if (!planar) return sk_h264_encode(s->enc, d + off[0], st[0], s->frame_id++);
        return sk_h264_encode_yuv(s->enc, yfmt, d + off[0], st[0], d + off[1], st[1],
                                  yfmt == 1 ? d + off[2] : NULL, yfmt == 1 ? st[2] : 0, 1, s->frame_id++);
    }
    GstVideoFrame vf;
    if (!gst_video_frame_map(&vf, info, buf, GST_MAP_READ)) return -2;   /* -2: not mappable */
    int n;
    if (!planar) {
        n = sk_h264_encode(s->enc, (const uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&vf, 0),
                           GST_VIDEO_FRAME_PLANE_STRIDE(&vf, 0), s->frame_id++);
    } else {
        n = sk_h264_encode_yuv(s->enc, yfmt, (const uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&vf, 0),
                               GST_VIDEO_FRAME_PLANE_STRIDE(&vf, 0), (const uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&vf, 1),
                               GST_VIDEO_FRAME_PLANE_STRIDE(&vf, 1),
                               yfmt == 1 ? (const uint8_t*)GST_VIDEO_FRAME_PLANE_DATA(&vf, 2) : NULL,
                               yfmt == 1 ? GST_VIDEO_FRAME_PLANE_STRIDE(&vf, 2) : 0, 0, s->frame_id++);
    }
    gst_video_frame_unmap(&vf);
    return n;
}

static GstFlowReturn hipenc_handle_frame(GstVideoEncoder* e, GstVideoCodecFrame* frame) {
    GstHipEnc* s = HIPENC(e);
    if (!s->enc || !s->in_state) {
        /* finish_frame without an output buffer is how 1.14 drops a frame (and releases
         * it); the error stops the stream */
        GST_ELEMENT_ERROR(s, CORE, NEGOTIATION, ("no encoder: caps were never set"), (NULL));
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

    const int n = hipenc_encode_buffer(s, frame->input_buffer);
    if (n == -2) {
        GST_ELEMENT_ERROR(s, STREAM, ENCODE, ("cannot map the input frame"), (NULL));
        gst_video_encoder_finish_frame(e, frame);
        return GST_FLOW_ERROR;
    }
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
        "video/x-raw(" GST_CAPS_FEATURE_MEMORY_HIP "), format=(string)" GST_HIP_RAW_FORMATS ", "
        "width=(int)[ 16, 8192 ], height=(int)[ 16, 8192 ], framerate=(fraction)[ 0/1, MAX ]; "
        "video/x-raw, format=(string)" GST_HIP_RAW_FORMATS ", width=(int)[ 16, 8192 ], height=(int)[ 16, 8192 ], "
        "framerate=(fraction)[ 0/1, MAX ]");
    gst_element_class_add_pad_template(ec, gst_pad_template_new("sink", GST_PAD_SINK, GST_PAD_ALWAYS, sink));
    gst_caps_unref(sink);
    GstCaps* src = hipenc_src_caps(codec);
    gst_element_class_add_pad_template(ec, gst_pad_template_new("src", GST_PAD_SRC, GST_PAD_ALWAYS, src));
    gst_caps_unref(src);
    gst_element_class_set_static_metadata(ec, kEncLong[codec], "Codec/Encoder/Video/Hardware",
                                          "Encodes BGRx / I420 / NV12 frames (system or HIP memory) on the MI355X "
                                          "(gfx950) media kernels",
                                          "selkies-mi355x");
}

GType gst_hip_enc_register(int codec) {
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

/* ------------------------------------------------------------------ plugin */
static gboolean plugin_init(GstPlugin* plugin) {
    GST_DEBUG_CATEGORY_INIT(gst_hip_debug, "hip", 0, "gfx950 media elements");
    for (int c = 0; c < 3; c++)
        if (!gst_element_register(plugin, kEncNames[c], GST_RANK_PRIMARY + 1, gst_hip_enc_register(c))) return FALSE;
    return gst_element_register(plugin, "hipconvert", GST_RANK_NONE, gst_hip_convert_get_type()) &&
           gst_element_register(plugin, "hipupload", GST_RANK_NONE, gst_hip_upload_get_type()) &&
           gst_element_register(plugin, "hipdownload", GST_RANK_NONE, gst_hip_download_get_type()) &&
           gst_element_register(plugin, "hipximagesrc", GST_RANK_NONE, gst_hip_ximage_src_get_type());
}

GST_PLUGIN_DEFINE(GST_VERSION_MAJOR, GST_VERSION_MINOR, hip,
                  "gfx950 (MI355X) media elements: H.264 / H.265 / AV1 encoders, conversion, HIP memory, X11 source",
                  plugin_init, VERSION, "LGPL", PACKAGE, "selkies-mi355x")
