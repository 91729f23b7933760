/*
 * Fake libudev.so.1 (LD_PRELOAD / LD_LIBRARY_PATH) describing the four virtual
 * Xbox 360 pads served by the joystick interposer (js_interposer.c), so
 * SDL2 / Proton / browsers that enumerate game controllers through udev find
 * /dev/input/js0..3 and /dev/input/event1000..1003 with USB parents.
 * Same role and exported symbol set as the reference
 * (addons/fake-udev/fake-libudev-core.c, libudev.sym); implementation is a
 * small static device table plus generic list / lookup helpers.
 *
 * Per pad i the table holds: a USB device (parent), an "input" device
 * (inputN), the jsI node and the event100I node (both children of inputN).
 * Monitors never report hot-plug events; hwdb and queue calls are inert.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/eventfd.h>
#include <sys/sysmacros.h>
#include <sys/types.h>
#include <unistd.h>

#define NUM_PADS 4
#define EXPORT __attribute__((visibility("default")))

struct udev {
    int refs;
    void* userdata;
};

struct udev_list_entry {
    char* name;
    char* value;
    struct udev_list_entry* next;
};

typedef struct {
    char syspath[160], devpath[160], sysname[32], subsystem[16], devtype[24], devnode[32], driver[16];
    int parent;       /* index in g_nodes or -1 */
    dev_t devnum;
    const char* props[24];   /* "KEY=VALUE" */
    const char* attrs[12];   /* "name=value" */
    char buf[1024];   /* backing store for generated strings */
} node_t;

struct udev_device {
    int refs;
    struct udev* udev;
    int node;
    struct udev_list_entry* props;
    struct udev_list_entry* attrs;
};

struct udev_enumerate {
    int refs;
    struct udev* udev;
    char subsystems[8][32];
    int nsub;
    char sysname[64];
    char prop_key[64], prop_val[64];
    char devnode[64];    /* add_match_devicenode (glob) */
    char sysnum[16];     /* add_match_sysnum: the trailing digits of the sysname */
    int parent;          /* add_match_parent: node index, -1 none */
    struct udev_list_entry* list;
};

struct udev_monitor {
    int refs;
    struct udev* udev;
    int fd;
};

#define NODES_PER_PAD 4
static node_t g_nodes[NUM_PADS * NODES_PER_PAD];
static int g_init = 0;

static char* store(node_t* n, size_t* off, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    char* p = n->buf + *off;
    int w = vsnprintf(p, sizeof(n->buf) - *off, fmt, ap);
    va_end(ap);
    *off += (size_t)w + 1;
    return p;
}

static void init_nodes(void) {
    if (g_init) return;
    g_init = 1;
    for (int i = 0; i < NUM_PADS; i++) {
        node_t* usb = &g_nodes[i * NODES_PER_PAD + 0];
        node_t* inp = &g_nodes[i * NODES_PER_PAD + 1];
        node_t* js = &g_nodes[i * NODES_PER_PAD + 2];
        node_t* ev = &g_nodes[i * NODES_PER_PAD + 3];
        memset(usb, 0, sizeof(*usb) * NODES_PER_PAD);
        size_t o;
        /* USB parent */
        snprintf(usb->devpath, sizeof(usb->devpath), "/devices/pci0000:00/0000:00:14.0/usb9/9-%d", i + 1);
        snprintf(usb->syspath, sizeof(usb->syspath), "/sys%s", usb->devpath);
        snprintf(usb->sysname, sizeof(usb->sysname), "9-%d", i + 1);
        strcpy(usb->subsystem, "usb");
        strcpy(usb->devtype, "usb_device");
        strcpy(usb->driver, "usb");
        usb->parent = -1;
        o = 0;
        usb->props[0] = store(usb, &o, "DEVTYPE=usb_device");
        usb->props[1] = store(usb, &o, "ID_VENDOR_ID=045e");
        usb->props[2] = store(usb, &o, "ID_MODEL_ID=028e");
        usb->props[3] = store(usb, &o, "ID_SERIAL=Microsoft_Controller_SELKIES%d", i);
        usb->props[4] = store(usb, &o, "SUBSYSTEM=usb");
        usb->attrs[0] = store(usb, &o, "idVendor=045e");
        usb->attrs[1] = store(usb, &o, "idProduct=028e");
        usb->attrs[2] = store(usb, &o, "bcdDevice=0114");
        usb->attrs[3] = store(usb, &o, "manufacturer=Microsoft");
        usb->attrs[4] = store(usb, &o, "product=Controller");
        usb->attrs[5] = store(usb, &o, "serial=SELKIES%d", i);
        /* input device */
        snprintf(inp->devpath, sizeof(inp->devpath), "%s/9-%d:1.0/input/input%d", usb->devpath, i + 1, 100 + i);
        snprintf(inp->syspath, sizeof(inp->syspath), "/sys%s", inp->devpath);
        snprintf(inp->sysname, sizeof(inp->sysname), "input%d", 100 + i);
        strcpy(inp->subsystem, "input");
        inp->parent = i * NODES_PER_PAD + 0;
        o = 0;
        inp->props[0] = store(inp, &o, "NAME=\"Microsoft X-Box 360 pad\"");
        inp->props[1] = store(inp, &o, "PRODUCT=3/45e/28e/114");
        inp->props[2] = store(inp, &o, "ID_INPUT=1");
        inp->props[3] = store(inp, &o, "ID_INPUT_JOYSTICK=1");
        inp->props[4] = store(inp, &o, "SUBSYSTEM=input");
        inp->props[5] = store(inp, &o, "PHYS=\"usb-selkies-virtual-%d/input0\"", i);
        inp->props[6] = store(inp, &o, "UNIQ=\"SELKIES-PAD-%d\"", i);
        inp->attrs[0] = store(inp, &o, "name=Microsoft X-Box 360 pad");
        inp->attrs[1] = store(inp, &o, "phys=usb-selkies-virtual-%d/input0", i);
        inp->attrs[2] = store(inp, &o, "uniq=SELKIES-PAD-%d", i);
        inp->attrs[3] = store(inp, &o, "id/vendor=045e");
        inp->attrs[4] = store(inp, &o, "id/product=028e");
        inp->attrs[5] = store(inp, &o, "id/version=0114");
        inp->attrs[6] = store(inp, &o, "id/bustype=0003");
        /* jsN and event100N nodes */
        for (int k = 0; k < 2; k++) {
            node_t* n = k == 0 ? js : ev;
            int minor = k == 0 ? i : 1000 + i;       /* js: 13:0.., event1000+: 13:(64+1000+i) */
            const char* base = k == 0 ? "js" : "event";
            int num = k == 0 ? i : 1000 + i;
            snprintf(n->sysname, sizeof(n->sysname), "%s%d", base, num);
            snprintf(n->devpath, sizeof(n->devpath), "%s/%s", inp->devpath, n->sysname);
            snprintf(n->syspath, sizeof(n->syspath), "/sys%s", n->devpath);
            snprintf(n->devnode, sizeof(n->devnode), "/dev/input/%s", n->sysname);
            strcpy(n->subsystem, "input");
            n->parent = i * NODES_PER_PAD + 1;
            n->devnum = makedev(13, k == 0 ? minor : 64 + minor);
            o = 0;
            n->props[0] = store(n, &o, "DEVNAME=%s", n->devnode);
            n->props[1] = store(n, &o, "MAJOR=13");
            n->props[2] = store(n, &o, "MINOR=%u", minor(n->devnum));
            n->props[3] = store(n, &o, "ID_INPUT=1");
            n->props[4] = store(n, &o, "ID_INPUT_JOYSTICK=1");
            n->props[5] = store(n, &o, "ID_BUS=usb");
            n->props[6] = store(n, &o, "ID_VENDOR_ID=045e");
            n->props[7] = store(n, &o, "ID_MODEL_ID=028e");
            n->props[8] = store(n, &o, "ID_SERIAL=Microsoft_Controller_SELKIES%d", i);
            n->props[9] = store(n, &o, "SUBSYSTEM=input");
            n->props[10] = store(n, &o, "DEVPATH=%s", n->devpath);
            n->props[11] = store(n, &o, "TAGS=:seat:uaccess:");
        }
    }
}

/* ---------------------------------------------------------------- lists */
static struct udev_list_entry* list_add(struct udev_list_entry** head, const char* name, const char* value) {
    struct udev_list_entry* e = calloc(1, sizeof(*e));
    if (!e) return NULL;
    e->name = strdup(name);
    e->value = value ? strdup(value) : NULL;
    struct udev_list_entry** p = head;
    while (*p) p = &(*p)->next;
    *p = e;
    return e;
}

static void list_free(struct udev_list_entry* e) {
    while (e) {
        struct udev_list_entry* n = e->next;
        free(e->name);
        free(e->value);
        free(e);
        e = n;
    }
}

static void kv_list(const char* const* kv, int n, struct udev_list_entry** out) {
    for (int i = 0; i < n && kv[i]; i++) {
        const char* eq = strchr(kv[i], '=');
        if (!eq) continue;
        char key[96];
        size_t kl = (size_t)(eq - kv[i]) < sizeof(key) - 1 ? (size_t)(eq - kv[i]) : sizeof(key) - 1;
        memcpy(key, kv[i], kl);
        key[kl] = 0;
        list_add(out, key, eq + 1);
    }
}

static const char* kv_get(const char* const* kv, int n, const char* key) {
    size_t kl = strlen(key);
    for (int i = 0; i < n && kv[i]; i++)
        if (!strncmp(kv[i], key, kl) && kv[i][kl] == '=') return kv[i] + kl + 1;
    return NULL;
}

EXPORT struct udev_list_entry* udev_list_entry_get_next(struct udev_list_entry* e) { return e ? e->next : NULL; }
EXPORT const char* udev_list_entry_get_name(struct udev_list_entry* e) { return e ? e->name : NULL; }
EXPORT const char* udev_list_entry_get_value(struct udev_list_entry* e) { return e ? e->value : NULL; }
EXPORT struct udev_list_entry* udev_list_entry_get_by_name(struct udev_list_entry* e, const char* name) {
    for (; e; e = e->next)
        if (name && !strcmp(e->name, name)) return e;
    return NULL;
}

/* ---------------------------------------------------------------- udev */
EXPORT struct udev* udev_new(void) {
    init_nodes();
    struct udev* u = calloc(1, sizeof(*u));
    if (u) u->refs = 1;
    return u;
}
EXPORT struct udev* udev_ref(struct udev* u) {
    if (u) u->refs++;
    return u;
}
EXPORT struct udev* udev_unref(struct udev* u) {
    if (u && --u->refs == 0) {
        free(u);
        return NULL;
    }
    return u;
}
EXPORT void* udev_get_userdata(struct udev* u) { return u ? u->userdata : NULL; }
EXPORT void udev_set_userdata(struct udev* u, void* d) { if (u) u->userdata = d; }
EXPORT void udev_set_log_fn(struct udev* u, void* fn) { (void)u; (void)fn; }
EXPORT int udev_get_log_priority(struct udev* u) { (void)u; return 3; }
EXPORT void udev_set_log_priority(struct udev* u, int p) { (void)u; (void)p; }

/* ---------------------------------------------------------------- devices */
static struct udev_device* device_for(struct udev* u, int node) {
    if (node < 0) return NULL;
    struct udev_device* d = calloc(1, sizeof(*d));
    if (!d) return NULL;
    d->refs = 1;
    d->udev = udev_ref(u);
    d->node = node;
    kv_list(g_nodes[node].props, 24, &d->props);
    kv_list(g_nodes[node].attrs, 12, &d->attrs);
    return d;
}

static int node_by_syspath(const char* p) {
    init_nodes();
    for (int i = 0; i < NUM_PADS * NODES_PER_PAD; i++)
        if (p && !strcmp(g_nodes[i].syspath, p)) return i;
    return -1;
}

EXPORT struct udev_device* udev_device_new_from_syspath(struct udev* u, const char* syspath) {
    return device_for(u, node_by_syspath(syspath));
}
EXPORT struct udev_device* udev_device_new_from_devnum(struct udev* u, char type, dev_t devnum) {
    init_nodes();
    if (type != 'c') return NULL;
    for (int i = 0; i < NUM_PADS * NODES_PER_PAD; i++)
        if (g_nodes[i].devnode[0] && g_nodes[i].devnum == devnum) return device_for(u, i);
    return NULL;
}
EXPORT struct udev_device* udev_device_new_from_subsystem_sysname(struct udev* u, const char* sub, const char* name) {
    init_nodes();
    for (int i = 0; i < NUM_PADS * NODES_PER_PAD; i++)
        if (sub && name && !strcmp(g_nodes[i].subsystem, sub) && !strcmp(g_nodes[i].sysname, name))
            return device_for(u, i);
    return NULL;
}
EXPORT struct udev_device* udev_device_new_from_device_id(struct udev* u, const char* id) {
    (void)u; (void)id;
    return NULL;
}
EXPORT struct udev_device* udev_device_new_from_environment(struct udev* u) { (void)u; return NULL; }
EXPORT struct udev_device* udev_device_ref(struct udev_device* d) {
    if (d) d->refs++;
    return d;
}
EXPORT struct udev_device* udev_device_unref(struct udev_device* d) {
    if (d && --d->refs == 0) {
        list_free(d->props);
        list_free(d->attrs);
        udev_unref(d->udev);
        free(d);
        return NULL;
    }
    return d;
}
EXPORT struct udev* udev_device_get_udev(struct udev_device* d) { return d ? d->udev : NULL; }
#define NODE(d) (&g_nodes[(d)->node])
EXPORT const char* udev_device_get_syspath(struct udev_device* d) { return d ? NODE(d)->syspath : NULL; }
EXPORT const char* udev_device_get_devpath(struct udev_device* d) { return d ? NODE(d)->devpath : NULL; }
EXPORT const char* udev_device_get_sysname(struct udev_device* d) { return d ? NODE(d)->sysname : NULL; }
EXPORT const char* udev_device_get_sysnum(struct udev_device* d) {
    if (!d) return NULL;
    const char* s = NODE(d)->sysname;
    while (*s && (*s < '0' || *s > '9')) s++;
    return *s ? s : NULL;
}
EXPORT const char* udev_device_get_subsystem(struct udev_device* d) { return d ? NODE(d)->subsystem : NULL; }
EXPORT const char* udev_device_get_devtype(struct udev_device* d) {
    return d && NODE(d)->devtype[0] ? NODE(d)->devtype : NULL;
}
EXPORT const char* udev_device_get_devnode(struct udev_device* d) {
    return d && NODE(d)->devnode[0] ? NODE(d)->devnode : NULL;
}
EXPORT const char* udev_device_get_driver(struct udev_device* d) {
    return d && NODE(d)->driver[0] ? NODE(d)->driver : NULL;
}
EXPORT dev_t udev_device_get_devnum(struct udev_device* d) { return d ? NODE(d)->devnum : makedev(0, 0); }
EXPORT const char* udev_device_get_action(struct udev_device* d) { (void)d; return NULL; }
EXPORT unsigned long long udev_device_get_seqnum(struct udev_device* d) { (void)d; return 0; }
EXPORT unsigned long long udev_device_get_usec_since_initialized(struct udev_device* d) { (void)d; return 1000000; }
EXPORT int udev_device_get_is_initialized(struct udev_device* d) { return d ? 1 : 0; }
EXPORT const char* udev_device_get_property_value(struct udev_device* d, const char* key) {
    return d && key ? kv_get(NODE(d)->props, 24, key) : NULL;
}
EXPORT const char* udev_device_get_sysattr_value(struct udev_device* d, const char* name) {
    return d && name ? kv_get(NODE(d)->attrs, 12, name) : NULL;
}
EXPORT int udev_device_set_sysattr_value(struct udev_device* d, const char* n, const char* v) {
    (void)d; (void)n; (void)v;
    return -1;
}
EXPORT struct udev_list_entry* udev_device_get_properties_list_entry(struct udev_device* d) {
    return d ? d->props : NULL;
}
EXPORT struct udev_list_entry* udev_device_get_sysattr_list_entry(struct udev_device* d) {
    return d ? d->attrs : NULL;
}
EXPORT struct udev_list_entry* udev_device_get_devlinks_list_entry(struct udev_device* d) { (void)d; return NULL; }
EXPORT struct udev_list_entry* udev_device_get_tags_list_entry(struct udev_device* d) { (void)d; return NULL; }
EXPORT struct udev_list_entry* udev_device_get_current_tags_list_entry(struct udev_device* d) { (void)d; return NULL; }
EXPORT int udev_device_has_tag(struct udev_device* d, const char* tag) {
    return d && tag && (!strcmp(tag, "seat") || !strcmp(tag, "uaccess"));
}
EXPORT int udev_device_has_current_tag(struct udev_device* d, const char* tag) { return udev_device_has_tag(d, tag); }

/* The parent is owned by the child in libudev: cache it inside a static pool. */
static struct udev_device* g_parent_cache[NUM_PADS * NODES_PER_PAD];
EXPORT struct udev_device* udev_device_get_parent(struct udev_device* d) {
    if (!d || NODE(d)->parent < 0) return NULL;
    int p = NODE(d)->parent;
    if (!g_parent_cache[p]) g_parent_cache[p] = device_for(d->udev, p);
    return g_parent_cache[p];
}
EXPORT struct udev_device* udev_device_get_parent_with_subsystem_devtype(struct udev_device* d, const char* sub,
                                                                         const char* devtype) {
    for (struct udev_device* p = udev_device_get_parent(d); p; p = udev_device_get_parent(p)) {
        if (sub && strcmp(NODE(p)->subsystem, sub)) continue;
        if (devtype && strcmp(NODE(p)->devtype, devtype)) continue;
        return p;
    }
    return NULL;
}

/* ---------------------------------------------------------------- enumerate */
EXPORT struct udev_enumerate* udev_enumerate_new(struct udev* u) {
    init_nodes();
    struct udev_enumerate* e = calloc(1, sizeof(*e));
    if (!e) return NULL;
    e->refs = 1;
    e->udev = udev_ref(u);
    e->parent = -1;
    return e;
}
EXPORT struct udev_enumerate* udev_enumerate_ref(struct udev_enumerate* e) {
    if (e) e->refs++;
    return e;
}
EXPORT struct udev_enumerate* udev_enumerate_unref(struct udev_enumerate* e) {
    if (e && --e->refs == 0) {
        list_free(e->list);
        udev_unref(e->udev);
        free(e);
        return NULL;
    }
    return e;
}
EXPORT struct udev* udev_enumerate_get_udev(struct udev_enumerate* e) { return e ? e->udev : NULL; }
EXPORT int udev_enumerate_add_match_subsystem(struct udev_enumerate* e, const char* sub) {
    if (!e || !sub || e->nsub >= 8) return -1;
    snprintf(e->subsystems[e->nsub++], 32, "%s", sub);
    return 0;
}
EXPORT int udev_enumerate_add_nomatch_subsystem(struct udev_enumerate* e, const char* s) { (void)e; (void)s; return 0; }
EXPORT int udev_enumerate_add_match_sysattr(struct udev_enumerate* e, const char* a, const char* v) {
    (void)e; (void)a; (void)v;
    return 0;
}
EXPORT int udev_enumerate_add_nomatch_sysattr(struct udev_enumerate* e, const char* a, const char* v) {
    (void)e; (void)a; (void)v;
    return 0;
}
EXPORT int udev_enumerate_add_match_property(struct udev_enumerate* e, const char* k, const char* v) {
    if (!e || !k) return -1;
    snprintf(e->prop_key, sizeof(e->prop_key), "%s", k);
    snprintf(e->prop_val, sizeof(e->prop_val), "%s", v ? v : "");
    return 0;
}
EXPORT int udev_enumerate_add_match_sysname(struct udev_enumerate* e, const char* n) {
    if (!e || !n) return -1;
    snprintf(e->sysname, sizeof(e->sysname), "%s", n);
    return 0;
}
EXPORT int udev_enumerate_add_match_tag(struct udev_enumerate* e, const char* t) { (void)e; (void)t; return 0; }
EXPORT int udev_enumerate_add_match_parent(struct udev_enumerate* e, struct udev_device* p) {
    if (!e) return -1;
    e->parent = p ? node_by_syspath(NODE(p)->syspath) : -1;
    return 0;
}
EXPORT int udev_enumerate_add_match_devicenode(struct udev_enumerate* e, const char* n) {
    if (!e || !n) return -1;
    snprintf(e->devnode, sizeof(e->devnode), "%s", n);
    return 0;
}
EXPORT int udev_enumerate_add_match_sysnum(struct udev_enumerate* e, const char* n) {
    if (!e || !n) return -1;
    snprintf(e->sysnum, sizeof(e->sysnum), "%s", n);
    return 0;
}
EXPORT int udev_enumerate_add_match_is_initialized(struct udev_enumerate* e) { (void)e; return 0; }
EXPORT int udev_enumerate_add_syspath(struct udev_enumerate* e, const char* p) {
    return e && node_by_syspath(p) >= 0 && list_add(&e->list, p, NULL) ? 0 : -1;
}

static int glob_match(const char* pat, const char* s) {
    if (!*pat) return !*s;
    if (*pat == '*') return glob_match(pat + 1, s) || (*s && glob_match(pat, s + 1));
    return *s && (*pat == '?' || *pat == *s) && glob_match(pat + 1, s + 1);
}

/* The digits at the end of a sysname ("js2" -> "2"; "" when there are none). */
static const char* sysnum_of(const char* sysname) {
    const char* p = sysname + strlen(sysname);
    while (p > sysname && p[-1] >= '0' && p[-1] <= '9') p--;
    return p;
}
/* Whether node i is `anc` or below it (libudev's match_parent includes the parent itself). */
static int node_under(int i, int anc) {
    for (int k = i; k >= 0; k = g_nodes[k].parent)
        if (k == anc) return 1;
    return 0;
}
static int enum_match(const struct udev_enumerate* e, int i) {
    const node_t* n = &g_nodes[i];
    if (e->nsub) {
        int ok = 0;
        for (int k = 0; k < e->nsub; k++) ok |= !strcmp(e->subsystems[k], n->subsystem);
        if (!ok) return 0;
    }
    if (e->sysname[0] && !glob_match(e->sysname, n->sysname)) return 0;
    if (e->devnode[0] && !(n->devnode[0] && glob_match(e->devnode, n->devnode))) return 0;
    if (e->sysnum[0] && !glob_match(e->sysnum, sysnum_of(n->sysname))) return 0;
    if (e->prop_key[0]) {
        const char* v = kv_get(n->props, 24, e->prop_key);
        if (!v || (e->prop_val[0] && !glob_match(e->prop_val, v))) return 0;
    }
    if (e->parent >= 0 && !node_under(i, e->parent)) return 0;
    return 1;
}
/* scan_children: the devices below the add_match_parent device (that device included),
   the other filters applied as in scan_devices. */
EXPORT int udev_enumerate_scan_children(struct udev_enumerate* e) {
    if (!e) return -1;
    if (e->parent < 0) return -EINVAL;
    list_free(e->list);
    e->list = NULL;
    for (int i = 0; i < NUM_PADS * NODES_PER_PAD; i++)
        if (enum_match(e, i)) list_add(&e->list, g_nodes[i].syspath, NULL);
    return 0;
}
EXPORT int udev_enumerate_scan_devices(struct udev_enumerate* e) {
    if (!e) return -1;
    list_free(e->list);
    e->list = NULL;
    for (int i = 0; i < NUM_PADS * NODES_PER_PAD; i++) {
        if (!enum_match(e, i)) continue;
        node_t* n = &g_nodes[i];
        list_add(&e->list, n->syspath, NULL);
    }
    return 0;
}
EXPORT int udev_enumerate_scan_subsystems(struct udev_enumerate* e) {
    if (!e) return -1;
    list_free(e->list);
    e->list = NULL;
    list_add(&e->list, "/sys/bus/usb", NULL);
    list_add(&e->list, "/sys/class/input", NULL);
    return 0;
}
EXPORT struct udev_list_entry* udev_enumerate_get_list_entry(struct udev_enumerate* e) { return e ? e->list : NULL; }

/* ---------------------------------------------------------------- monitor */
EXPORT struct udev_monitor* udev_monitor_new_from_netlink(struct udev* u, const char* name) {
    (void)name;
    struct udev_monitor* m = calloc(1, sizeof(*m));
    if (!m) return NULL;
    m->refs = 1;
    m->udev = udev_ref(u);
    m->fd = eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);  /* valid, pollable, never readable */
    return m;
}
EXPORT struct udev_monitor* udev_monitor_ref(struct udev_monitor* m) {
    if (m) m->refs++;
    return m;
}
EXPORT struct udev_monitor* udev_monitor_unref(struct udev_monitor* m) {
    if (m && --m->refs == 0) {
        if (m->fd >= 0) close(m->fd);
        udev_unref(m->udev);
        free(m);
        return NULL;
    }
    return m;
}
EXPORT struct udev* udev_monitor_get_udev(struct udev_monitor* m) { return m ? m->udev : NULL; }
EXPORT int udev_monitor_enable_receiving(struct udev_monitor* m) { return m ? 0 : -1; }
EXPORT int udev_monitor_set_receive_buffer_size(struct udev_monitor* m, int s) { (void)m; (void)s; return 0; }
EXPORT int udev_monitor_get_fd(struct udev_monitor* m) { return m ? m->fd : -1; }
EXPORT struct udev_device* udev_monitor_receive_device(struct udev_monitor* m) { (void)m; return NULL; }
EXPORT int udev_monitor_filter_add_match_subsystem_devtype(struct udev_monitor* m, const char* s, const char* d) {
    (void)m; (void)s; (void)d;
    return 0;
}
EXPORT int udev_monitor_filter_add_match_tag(struct udev_monitor* m, const char* t) { (void)m; (void)t; return 0; }
EXPORT int udev_monitor_filter_update(struct udev_monitor* m) { (void)m; return 0; }
EXPORT int udev_monitor_filter_remove(struct udev_monitor* m) { (void)m; return 0; }

/* ---------------------------------------------------------------- hwdb / queue / util */
struct udev_hwdb { int refs; };
EXPORT struct udev_hwdb* udev_hwdb_new(struct udev* u) {
    (void)u;
    struct udev_hwdb* h = calloc(1, sizeof(*h));
    if (h) h->refs = 1;
    return h;
}
EXPORT struct udev_hwdb* udev_hwdb_ref(struct udev_hwdb* h) {
    if (h) h->refs++;
    return h;
}
EXPORT struct udev_hwdb* udev_hwdb_unref(struct udev_hwdb* h) {
    if (h && --h->refs == 0) {
        free(h);
        return NULL;
    }
    return h;
}
EXPORT struct udev_list_entry* udev_hwdb_get_properties_list_entry(struct udev_hwdb* h, const char* m, unsigned f) {
    (void)h; (void)m; (void)f;
    return NULL;
}

struct udev_queue { int refs; struct udev* udev; };
EXPORT struct udev_queue* udev_queue_new(struct udev* u) {
    struct udev_queue* q = calloc(1, sizeof(*q));
    if (q) {
        q->refs = 1;
        q->udev = udev_ref(u);
    }
    return q;
}
EXPORT struct udev_queue* udev_queue_ref(struct udev_queue* q) {
    if (q) q->refs++;
    return q;
}
EXPORT struct udev_queue* udev_queue_unref(struct udev_queue* q) {
    if (q && --q->refs == 0) {
        udev_unref(q->udev);
        free(q);
        return NULL;
    }
    return q;
}
EXPORT struct udev* udev_queue_get_udev(struct udev_queue* q) { return q ? q->udev : NULL; }
EXPORT int udev_queue_get_udev_is_active(struct udev_queue* q) { (void)q; return 1; }
EXPORT int udev_queue_get_queue_is_empty(struct udev_queue* q) { (void)q; return 1; }
EXPORT int udev_queue_get_seqnum_is_finished(struct udev_queue* q, unsigned long long s) { (void)q; (void)s; return 1; }
EXPORT int udev_queue_get_seqnum_sequence_is_finished(struct udev_queue* q, unsigned long long a, unsigned long long b) {
    (void)q; (void)a; (void)b;
    return 1;
}
EXPORT unsigned long long udev_queue_get_kernel_seqnum(struct udev_queue* q) { (void)q; return 0; }
EXPORT unsigned long long udev_queue_get_udev_seqnum(struct udev_queue* q) { (void)q; return 0; }
EXPORT struct udev_list_entry* udev_queue_get_queued_list_entry(struct udev_queue* q) { (void)q; return NULL; }
EXPORT int udev_queue_get_fd(struct udev_queue* q) { (void)q; return -1; }
EXPORT int udev_queue_flush(struct udev_queue* q) { (void)q; return 0; }

EXPORT int udev_util_encode_string(const char* str, char* out, size_t len) {
    if (!str || !out || !len) return -1;
    size_t j = 0;
    for (size_t i = 0; str[i]; i++) {
        unsigned char c = (unsigned char)str[i];
        if (c == '\\' || c == '/' || c <= ' ' || c >= 0x7f) {
            if (j + 4 >= len) return -1;
            j += (size_t)snprintf(out + j, len - j, "\\x%02x", c);
        } else {
            if (j + 1 >= len) return -1;
            out[j++] = (char)c;
        }
    }
    out[j] = 0;
    return 0;
}
