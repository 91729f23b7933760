/* hipximagesrc: live BGRx source over the native X11 MIT-SHM grabber
 * (csrc/capture/x11_source.cpp: XShmGetImage of a root-window region, XFixes cursor,
 * XDamage rows), the element the reference's graphs start from (ximagesrc,
 * legacy/gstwebrtc_app.py:210-255) with its property names: display-name, show-pointer,
 * use-damage, startx / starty / endx / endy, remote. source= selects the synthetic
 * desktop instead of X (headless hosts and tests, like the server's
 * --capture-source synthetic).
 *
 * use-damage: when the grabber reports that no row changed since the previous grab,
 * the previous buffer is pushed again (no copy of the frame). Frames are paced on the
 * pipeline clock at the negotiated framerate (default 60/1). */
#include "gsthip.h"

#include <string.h>

typedef enum { HIP_SRC_X11 = 0, HIP_SRC_MOTION = 1, HIP_SRC_DESKTOP = 2, HIP_SRC_NOISE = 3 } GstHipSourceKind;

static GType gst_hip_source_kind_get_type(void) {
    static gsize id = 0;
    static const GEnumValue values[] = {
        {HIP_SRC_X11, "X11 screen (MIT-SHM)", "x11"},
        {HIP_SRC_MOTION, "Synthetic desktop, scrolling and moving windows", "synthetic-motion"},
        {HIP_SRC_DESKTOP, "Synthetic desktop, mostly static", "synthetic-desktop"},
        {HIP_SRC_NOISE, "Uniform noise", "noise"},
        {0, NULL, NULL}};
    if (g_once_init_enter(&id)) g_once_init_leave(&id, g_enum_register_static("GstHipSourceKind", values));
    return (GType)id;
}

typedef struct {
    GstPushSrc parent;
    /* properties */
    gchar* display;
    gboolean show_pointer, use_damage, remote;
    guint startx, starty, endx, endy;
    gint kind;
    guint seed;
    /* state */
    void* src;
    gint width, height, fps_n, fps_d;
    GstClockTime next_rt; /* running time of the next frame */
    guint64 frames;
    GstClockID clock_id;
    gboolean flushing;
    GstBuffer* last;
} GstHipXImageSrc;
typedef struct {
    GstPushSrcClass parent_class;
} GstHipXImageSrcClass;

enum {
    SPROP_0,
    SPROP_DISPLAY,
    SPROP_SHOW_POINTER,
    SPROP_USE_DAMAGE,
    SPROP_STARTX,
    SPROP_STARTY,
    SPROP_ENDX,
    SPROP_ENDY,
    SPROP_REMOTE,
    SPROP_SOURCE,
    SPROP_SEED,
};

static GstPushSrcClass* ximg_parent_class = NULL;
#define XIMG(o) ((GstHipXImageSrc*)(o))

static void ximg_set_property(GObject* obj, guint id, const GValue* v, GParamSpec* ps) {
    GstHipXImageSrc* s = XIMG(obj);
    switch (id) {
        case SPROP_DISPLAY: g_free(s->display); s->display = g_value_dup_string(v); break;
        case SPROP_SHOW_POINTER: s->show_pointer = g_value_get_boolean(v); break;
        case SPROP_USE_DAMAGE: s->use_damage = g_value_get_boolean(v); break;
        case SPROP_STARTX: s->startx = g_value_get_uint(v); break;
        case SPROP_STARTY: s->starty = g_value_get_uint(v); break;
        case SPROP_ENDX: s->endx = g_value_get_uint(v); break;
        case SPROP_ENDY: s->endy = g_value_get_uint(v); break;
        case SPROP_REMOTE: s->remote = g_value_get_boolean(v); break;
        case SPROP_SOURCE: s->kind = g_value_get_enum(v); break;
        case SPROP_SEED: s->seed = g_value_get_uint(v); break;
        default: G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps); break;
    }
}

static void ximg_get_property(GObject* obj, guint id, GValue* v, GParamSpec* ps) {
    GstHipXImageSrc* s = XIMG(obj);
    switch (id) {
        case SPROP_DISPLAY: g_value_set_string(v, s->display); break;
        case SPROP_SHOW_POINTER: g_value_set_boolean(v, s->show_pointer); break;
        case SPROP_USE_DAMAGE: g_value_set_boolean(v, s->use_damage); break;
        case SPROP_STARTX: g_value_set_uint(v, s->startx); break;
        case SPROP_STARTY: g_value_set_uint(v, s->starty); break;
        case SPROP_ENDX: g_value_set_uint(v, s->endx); break;
        case SPROP_ENDY: g_value_set_uint(v, s->endy); break;
        case SPROP_REMOTE: g_value_set_boolean(v, s->remote); break;
        case SPROP_SOURCE: g_value_set_enum(v, s->kind); break;
        case SPROP_SEED: g_value_set_uint(v, s->seed); break;
        default: G_OBJECT_WARN_INVALID_PROPERTY_ID(obj, id, ps); break;
    }
}

/* Region size: endx / endy inclusive like ximagesrc; 0 = to the screen edge (X11) or
 * 1920x1080 (synthetic). */
static gboolean ximg_open(GstHipXImageSrc* s) {
    if (s->src) return TRUE;
    gint sw = 1920, sh = 1080;
    const char* disp = s->display && *s->display ? s->display : g_getenv("DISPLAY");
    if (s->kind == HIP_SRC_X11 && (!s->endx || !s->endy)) {
        void* x = sk_x11_input_open(disp, 1);
        if (!x) {
            GST_ELEMENT_ERROR(s, RESOURCE, OPEN_READ, ("cannot open X display %s", disp ? disp : "(unset)"),
                              ("%s", sk_last_error()));
            return FALSE;
        }
        sk_x11_screen_size(x, &sw, &sh);
        sk_x11_input_close(x);
    }
    const gint x1 = s->endx ? (gint)s->endx : sw - 1, y1 = s->endy ? (gint)s->endy : sh - 1;
    s->width = (x1 - (gint)s->startx + 1) & ~1;
    s->height = (y1 - (gint)s->starty + 1) & ~1;
    if (s->width < 16 || s->height < 16) {
        GST_ELEMENT_ERROR(s, RESOURCE, SETTINGS, ("capture region below 16x16"), (NULL));
        return FALSE;
    }
    s->src = sk_source_open(s->kind, disp, (int32_t)s->startx, (int32_t)s->starty, s->width, s->height,
                            s->show_pointer ? 1 : 0, s->seed);
    if (!s->src) {
        GST_ELEMENT_ERROR(s, RESOURCE, OPEN_READ, ("cannot open the frame source"), ("%s", sk_last_error()));
        return FALSE;
    }
    GST_INFO_OBJECT(s, "%s source %dx%d at %u,%u", sk_source_name(s->src), s->width, s->height, s->startx, s->starty);
    return TRUE;
}

static gboolean ximg_start(GstBaseSrc* b) {
    GstHipXImageSrc* s = XIMG(b);
    s->frames = 0;
    s->next_rt = GST_CLOCK_TIME_NONE;
    s->flushing = FALSE;
    return ximg_open(s);
}

static gboolean ximg_stop(GstBaseSrc* b) {
    GstHipXImageSrc* s = XIMG(b);
    if (s->src) sk_source_close(s->src);
    s->src = NULL;
    if (s->last) gst_buffer_unref(s->last);
    s->last = NULL;
    return TRUE;
}

static GstCaps* ximg_get_caps(GstBaseSrc* b, GstCaps* filter) {
    GstHipXImageSrc* s = XIMG(b);
    GstCaps* caps;
    if (!s->src) {
        caps = gst_pad_get_pad_template_caps(GST_BASE_SRC_PAD(b));
    } else {
        caps = gst_caps_new_simple("video/x-raw", "format", G_TYPE_STRING, "BGRx", "width", G_TYPE_INT, s->width,
                                   "height", G_TYPE_INT, s->height, "framerate", GST_TYPE_FRACTION_RANGE, 1, 1,
                                   G_MAXINT, 1, "pixel-aspect-ratio", GST_TYPE_FRACTION, 1, 1, NULL);
    }
    if (filter) {
        GstCaps* f = gst_caps_intersect_full(filter, caps, GST_CAPS_INTERSECT_FIRST);
        gst_caps_unref(caps);
        caps = f;
    }
    return caps;
}

static GstCaps* ximg_fixate(GstBaseSrc* b, GstCaps* caps) {
    caps = gst_caps_make_writable(caps);
    GstStructure* st = gst_caps_get_structure(caps, 0);
    gst_structure_fixate_field_nearest_fraction(st, "framerate", 60, 1);
    return GST_BASE_SRC_CLASS(ximg_parent_class)->fixate(b, caps);
}

static gboolean ximg_set_caps(GstBaseSrc* b, GstCaps* caps) {
    GstHipXImageSrc* s = XIMG(b);
    GstStructure* st = gst_caps_get_structure(caps, 0);
    if (!gst_structure_get_fraction(st, "framerate", &s->fps_n, &s->fps_d) || s->fps_n <= 0) {
        s->fps_n = 60;
        s->fps_d = 1;
    }
    return TRUE;
}

static gboolean ximg_unlock(GstBaseSrc* b) {
    GstHipXImageSrc* s = XIMG(b);
    GST_OBJECT_LOCK(s);
    s->flushing = TRUE;
    if (s->clock_id) gst_clock_id_unschedule(s->clock_id);
    GST_OBJECT_UNLOCK(s);
    return TRUE;
}

static gboolean ximg_unlock_stop(GstBaseSrc* b) {
    GstHipXImageSrc* s = XIMG(b);
    GST_OBJECT_LOCK(s);
    s->flushing = FALSE;
    GST_OBJECT_UNLOCK(s);
    return TRUE;
}

static GstFlowReturn ximg_create(GstPushSrc* ps, GstBuffer** out) {
    GstHipXImageSrc* s = XIMG(ps);
    const GstClockTime dur = gst_util_uint64_scale_int(GST_SECOND, s->fps_d, s->fps_n);
    GstClockTime pts = s->frames * dur;
    GstClock* clock = gst_element_get_clock(GST_ELEMENT(s));
    if (clock) {   /* live pacing: wait for the next frame slot on the pipeline clock */
        const GstClockTime base = gst_element_get_base_time(GST_ELEMENT(s));
        GstClockTime now = gst_clock_get_time(clock) - base;
        if (!GST_CLOCK_TIME_IS_VALID(s->next_rt) || s->next_rt + dur < now) s->next_rt = now;   /* (re)start or late */
        if (s->next_rt > now) {
            GST_OBJECT_LOCK(s);
            if (s->flushing) {
                GST_OBJECT_UNLOCK(s);
                gst_object_unref(clock);
                return GST_FLOW_FLUSHING;
            }
            s->clock_id = gst_clock_new_single_shot_id(clock, base + s->next_rt);
            GST_OBJECT_UNLOCK(s);
            const GstClockReturn r = gst_clock_id_wait(s->clock_id, NULL);
            GST_OBJECT_LOCK(s);
            gst_clock_id_unref(s->clock_id);
            s->clock_id = NULL;
            GST_OBJECT_UNLOCK(s);
            if (r == GST_CLOCK_UNSCHEDULED) {
                gst_object_unref(clock);
                return GST_FLOW_FLUSHING;
            }
        }
        pts = s->next_rt;
        s->next_rt += dur;
        gst_object_unref(clock);
    }
    int32_t stride = 0, nrows = -1;
    int32_t rows[64];
    const uint8_t* px = sk_source_grab(s->src, &stride, rows, 32, &nrows);
    if (!px) {
        GST_ELEMENT_ERROR(s, RESOURCE, READ, ("grab failed"), ("%s", sk_last_error()));
        return GST_FLOW_ERROR;
    }
    GstBuffer* buf;
    if (s->use_damage && nrows == 0 && s->last) {   /* nothing changed: the last frame again */
        buf = gst_buffer_copy(s->last);               /* shares the memory, fresh metadata */
    } else {
        const gsize row = (gsize)s->width * 4, size = row * (gsize)s->height;
        buf = gst_buffer_new_allocate(NULL, size, NULL);
        GstMapInfo m;
        gst_buffer_map(buf, &m, GST_MAP_WRITE);
        if ((gsize)stride == row) {
            memcpy(m.data, px, size);
        } else {
            for (gint y = 0; y < s->height; y++) memcpy(m.data + (gsize)y * row, px + (gsize)y * stride, row);
        }
        gst_buffer_unmap(buf, &m);
        if (s->last) gst_buffer_unref(s->last);
        s->last = gst_buffer_ref(buf);
    }
    GST_BUFFER_PTS(buf) = pts;
    GST_BUFFER_DTS(buf) = GST_CLOCK_TIME_NONE;
    GST_BUFFER_DURATION(buf) = dur;
    GST_BUFFER_OFFSET(buf) = s->frames;
    GST_BUFFER_OFFSET_END(buf) = s->frames + 1;
    s->frames++;
    *out = buf;
    return GST_FLOW_OK;
}

static void ximg_finalize(GObject* obj) {
    GstHipXImageSrc* s = XIMG(obj);
    g_free(s->display);
    if (s->src) sk_source_close(s->src);
    if (s->last) gst_buffer_unref(s->last);
    G_OBJECT_CLASS(ximg_parent_class)->finalize(obj);
}

static void ximg_init(GTypeInstance* inst, gpointer klass) {
    (void)klass;
    GstHipXImageSrc* s = XIMG(inst);
    s->display = NULL;
    s->show_pointer = TRUE;
    s->use_damage = TRUE;
    s->remote = FALSE;
    s->startx = s->starty = s->endx = s->endy = 0;
    s->kind = HIP_SRC_X11;
    s->seed = 0x1234567u;
    s->src = NULL;
    s->fps_n = 60;
    s->fps_d = 1;
    s->clock_id = NULL;
    s->last = NULL;
    gst_base_src_set_live(GST_BASE_SRC(s), TRUE);
    gst_base_src_set_format(GST_BASE_SRC(s), GST_FORMAT_TIME);
}

static void ximg_class_init(gpointer klass, gpointer data) {
    (void)data;
    GObjectClass* oc = G_OBJECT_CLASS(klass);
    GstElementClass* ec = GST_ELEMENT_CLASS(klass);
    GstBaseSrcClass* bc = GST_BASE_SRC_CLASS(klass);
    GstPushSrcClass* pc = GST_PUSH_SRC_CLASS(klass);
    ximg_parent_class = (GstPushSrcClass*)g_type_class_peek_parent(klass);
    oc->set_property = ximg_set_property;
    oc->get_property = ximg_get_property;
    oc->finalize = ximg_finalize;
    bc->start = ximg_start;
    bc->stop = ximg_stop;
    bc->get_caps = ximg_get_caps;
    bc->fixate = ximg_fixate;
    bc->set_caps = ximg_set_caps;
    bc->unlock = ximg_unlock;
    bc->unlock_stop = ximg_unlock_stop;
    pc->create = ximg_create;
    const GParamFlags rw = (GParamFlags)(G_PARAM_READWRITE | G_PARAM_STATIC_STRINGS);
    g_object_class_install_property(oc, SPROP_DISPLAY,
        g_param_spec_string("display-name", "Display", "X display name (default: $DISPLAY)", NULL, rw));
    g_object_class_install_property(oc, SPROP_SHOW_POINTER,
        g_param_spec_boolean("show-pointer", "Show pointer", "Composite the mouse pointer (XFixes)", TRUE, rw));
    g_object_class_install_property(oc, SPROP_USE_DAMAGE,
        g_param_spec_boolean("use-damage", "Use damage",
                             "Repeat the last buffer without copying when XDamage reports no change", TRUE, rw));
    g_object_class_install_property(oc, SPROP_STARTX,
        g_param_spec_uint("startx", "Start X", "Left edge of the region", 0, G_MAXINT, 0, rw));
    g_object_class_install_property(oc, SPROP_STARTY,
        g_param_spec_uint("starty", "Start Y", "Top edge of the region", 0, G_MAXINT, 0, rw));
    g_object_class_install_property(oc, SPROP_ENDX,
        g_param_spec_uint("endx", "End X", "Right edge of the region, inclusive (0 = screen edge)", 0, G_MAXINT, 0, rw));
    g_object_class_install_property(oc, SPROP_ENDY,
        g_param_spec_uint("endy", "End Y", "Bottom edge of the region, inclusive (0 = screen edge)", 0, G_MAXINT, 0, rw));
    g_object_class_install_property(oc, SPROP_REMOTE,
        g_param_spec_boolean("remote", "Remote", "Accepted for ximagesrc compatibility (MIT-SHM is always used)", FALSE, rw));
    g_object_class_install_property(oc, SPROP_SOURCE,
        g_param_spec_enum("source", "Source", "Frame source", gst_hip_source_kind_get_type(), HIP_SRC_X11, rw));
    g_object_class_install_property(oc, SPROP_SEED,
        g_param_spec_uint("seed", "Seed", "Synthetic source seed", 0, G_MAXUINT, 0x1234567u, rw));
    GstCaps* caps = gst_caps_from_string("video/x-raw, format=(string)BGRx, width=(int)[ 16, 16384 ], "
                                         "height=(int)[ 16, 16384 ], framerate=(fraction)[ 1/1, MAX ]");
    gst_element_class_add_pad_template(ec, gst_pad_template_new("src", GST_PAD_SRC, GST_PAD_ALWAYS, caps));
    gst_caps_unref(caps);
    gst_element_class_set_static_metadata(ec, "X11 screen source (MIT-SHM, selkies-mi355x)", "Source/Video",
                                          "Captures an X11 screen region as BGRx frames (ximagesrc replacement)",
                                          "selkies-mi355x");
}

GType gst_hip_ximage_src_get_type(void) {
    static gsize id = 0;
    if (g_once_init_enter(&id)) {
        GTypeInfo info;
        memset(&info, 0, sizeof(info));
        info.class_size = sizeof(GstHipXImageSrcClass);
        info.class_init = ximg_class_init;
        info.instance_size = sizeof(GstHipXImageSrc);
        info.instance_init = ximg_init;
        g_once_init_leave(&id, g_type_register_static(GST_TYPE_PUSH_SRC, "GstHipXImageSrc", &info, (GTypeFlags)0));
    }
    return (GType)id;
}
