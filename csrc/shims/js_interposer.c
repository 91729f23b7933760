/*
 * Joystick interposer (LD_PRELOAD into the game / application process).
 *
 * Presents four virtual Xbox 360 pads as /dev/input/js0..3 (joystick API) and
 * /dev/input/event1000..1003 (evdev) backed by the unix sockets the streaming
 * server serves (selkies_gstreamer_amd/server/gamepad.py), with the same socket
 * ABI as the reference interposer (addons/js-interposer/joystick_interposer.c):
 *   server -> 1360-byte js_config_t, interposer -> 1 byte sizeof(long),
 *   then a stream of struct js_event / struct input_event.
 *
 * Hooks: open, open64, openat, openat64, __open_2, __open64_2, close, read,
 * ioctl, epoll_ctl, access. Device identity answers (JSIOC*, EVIOC*) come
 * from the config the server sent, so the fake libudev (fake_udev.c) and the
 * ioctls describe the same device.
 *
 * Environment: SELKIES_INTERPOSER_SOCKET_DIR (default /tmp),
 *              SELKIES_INTERPOSER_DEBUG=1 for stderr logging.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <linux/input.h>
#include <linux/joystick.h>
#include <pthread.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/ioctl.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#define NUM_PADS 4
#define NAME_LEN 255
#define MAX_BTNS 512
#define MAX_AXES 64

typedef struct {
    char name[NAME_LEN];
    uint16_t vendor, product, version, num_btns, num_axes;
    uint16_t btn_map[MAX_BTNS];
    uint8_t axes_map[MAX_AXES];
    uint8_t final_alignment_padding[6];
} js_config_t;

_Static_assert(sizeof(js_config_t) == 1360, "js_config_t ABI must stay 1360 bytes");

enum { KIND_JS = 0, KIND_EV = 1 };

typedef struct {
    int kind, pad;
    int fd;           /* socket fd handed to the application, -1 when closed */
    int app_flags;
    struct js_corr corr[MAX_AXES];
    js_config_t cfg;
} vdev_t;

static vdev_t g_dev[2 * NUM_PADS];
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_debug = -1;

static int (*real_open)(const char*, int, ...);
static int (*real_open64)(const char*, int, ...);
static int (*real_openat)(int, const char*, int, ...);
static int (*real_openat64)(int, const char*, int, ...);
static int (*real___open_2)(const char*, int);
static int (*real___open64_2)(const char*, int);
static int (*real_close)(int);
static ssize_t (*real_read)(int, void*, size_t);
static int (*real_ioctl)(int, unsigned long, ...);
static int (*real_epoll_ctl)(int, int, int, struct epoll_event*);
static int (*real_access)(const char*, int);

static void logf_(const char* fmt, ...) {
    if (g_debug < 0) {
        const char* e = getenv("SELKIES_INTERPOSER_DEBUG");
        g_debug = e && *e == '1';
    }
    if (!g_debug) return;
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "[selkies-js] ");
    vfprintf(stderr, fmt, ap);
    fputc('\n', stderr);
    va_end(ap);
}

__attribute__((constructor)) static void interposer_init(void) {
    real_open = dlsym(RTLD_NEXT, "open");
    real_open64 = dlsym(RTLD_NEXT, "open64");
    real_openat = dlsym(RTLD_NEXT, "openat");
    real_openat64 = dlsym(RTLD_NEXT, "openat64");
    real___open_2 = dlsym(RTLD_NEXT, "__open_2");
    real___open64_2 = dlsym(RTLD_NEXT, "__open64_2");
    real_close = dlsym(RTLD_NEXT, "close");
    real_read = dlsym(RTLD_NEXT, "read");
    real_ioctl = dlsym(RTLD_NEXT, "ioctl");
    real_epoll_ctl = dlsym(RTLD_NEXT, "epoll_ctl");
    real_access = dlsym(RTLD_NEXT, "access");
    for (int i = 0; i < 2 * NUM_PADS; i++) {
        g_dev[i].kind = i < NUM_PADS ? KIND_JS : KIND_EV;
        g_dev[i].pad = i % NUM_PADS;
        g_dev[i].fd = -1;
    }
}

/* Maps a device path to its table slot, or -1. */
static int match_path(const char* path) {
    if (!path) return -1;
    int n;
    char tail;
    if (sscanf(path, "/dev/input/js%d%c", &n, &tail) == 1 && n >= 0 && n < NUM_PADS) return n;
    if (sscanf(path, "/dev/input/event%d%c", &n, &tail) == 1 && n >= 1000 && n < 1000 + NUM_PADS)
        return NUM_PADS + (n - 1000);
    return -1;
}

static vdev_t* find_fd(int fd) {
    if (fd < 0) return NULL;
    for (int i = 0; i < 2 * NUM_PADS; i++)
        if (g_dev[i].fd == fd) return &g_dev[i];
    return NULL;
}

static void socket_path(const vdev_t* d, char* out, size_t n) {
    const char* dir = getenv("SELKIES_INTERPOSER_SOCKET_DIR");
    if (!dir || !*dir) dir = "/tmp";
    if (d->kind == KIND_JS)
        snprintf(out, n, "%s/selkies_js%d.sock", dir, d->pad);
    else
        snprintf(out, n, "%s/selkies_event%d.sock", dir, 1000 + d->pad);
}

static int read_full(int fd, void* buf, size_t n) {
    size_t got = 0;
    while (got < n) {
        ssize_t r = real_read(fd, (char*)buf + got, n - got);
        if (r > 0) {
            got += (size_t)r;
        } else if (r < 0 && errno == EINTR) {
            continue;
        } else {
            return -1;
        }
    }
    return 0;
}

static int open_virtual(int slot, int flags) {
    vdev_t* d = &g_dev[slot];
    pthread_mutex_lock(&g_mu);
    if (d->fd >= 0) { /* one open per device: a second open gets EBUSY like exclusive hardware */
        pthread_mutex_unlock(&g_mu);
        errno = EBUSY;
        return -1;
    }
    int s = socket(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0);
    if (s < 0) {
        pthread_mutex_unlock(&g_mu);
        return -1;
    }
    struct sockaddr_un addr;
    memset(&addr, 0, sizeof(addr));
    addr.sun_family = AF_UNIX;
    socket_path(d, addr.sun_path, sizeof(addr.sun_path));
    if (connect(s, (struct sockaddr*)&addr, sizeof(addr)) < 0 || read_full(s, &d->cfg, sizeof(d->cfg)) < 0) {
        int e = errno ? errno : ENOENT;
        logf_("cannot reach %s (%s)", addr.sun_path, strerror(e));
        real_close(s);
        pthread_mutex_unlock(&g_mu);
        errno = ENOENT;
        return -1;
    }
    uint8_t arch = (uint8_t)sizeof(long);
    if (write(s, &arch, 1) != 1) {
        real_close(s);
        pthread_mutex_unlock(&g_mu);
        errno = EIO;
        return -1;
    }
    if (flags & O_NONBLOCK) fcntl(s, F_SETFL, fcntl(s, F_GETFL) | O_NONBLOCK);
    d->fd = s;
    d->app_flags = flags;
    memset(d->corr, 0, sizeof(d->corr));
    pthread_mutex_unlock(&g_mu);
    logf_("opened %s pad %d -> fd %d ('%.*s', %u buttons, %u axes)", d->kind == KIND_JS ? "js" : "evdev", d->pad,
          s, NAME_LEN, d->cfg.name, d->cfg.num_btns, d->cfg.num_axes);
    return s;
}

#define OPEN_BODY(REAL, ...)                                          \
    int slot = match_path(path);                                      \
    if (slot >= 0) return open_virtual(slot, flags);                  \
    if (!REAL) { errno = ENOSYS; return -1; }                         \
    return REAL(__VA_ARGS__);

static mode_t mode_arg(int flags, va_list ap) {
    return (flags & (O_CREAT | O_TMPFILE)) ? (mode_t)va_arg(ap, int) : 0;
}

int open(const char* path, int flags, ...) {
    va_list ap;
    va_start(ap, flags);
    mode_t m = mode_arg(flags, ap);
    va_end(ap);
    OPEN_BODY(real_open, path, flags, m)
}
int open64(const char* path, int flags, ...) {
    va_list ap;
    va_start(ap, flags);
    mode_t m = mode_arg(flags, ap);
    va_end(ap);
    OPEN_BODY(real_open64, path, flags, m)
}
int openat(int dirfd, const char* path, int flags, ...) {
    va_list ap;
    va_start(ap, flags);
    mode_t m = mode_arg(flags, ap);
    va_end(ap);
    OPEN_BODY(real_openat, dirfd, path, flags, m)
}
int openat64(int dirfd, const char* path, int flags, ...) {
    va_list ap;
    va_start(ap, flags);
    mode_t m = mode_arg(flags, ap);
    va_end(ap);
    OPEN_BODY(real_openat64, dirfd, path, flags, m)
}
int __open_2(const char* path, int flags) { OPEN_BODY(real___open_2, path, flags) }
int __open64_2(const char* path, int flags) { OPEN_BODY(real___open64_2, path, flags) }

int close(int fd) {
    pthread_mutex_lock(&g_mu);
    vdev_t* d = find_fd(fd);
    if (d) d->fd = -1;
    pthread_mutex_unlock(&g_mu);
    return real_close(fd);
}

ssize_t read(int fd, void* buf, size_t n) {
    /* Events arrive already in js_event / input_event layout: plain pass-through,
       EAGAIN semantics of a non-blocking socket match the device's. */
    return real_read(fd, buf, n);
}

int access(const char* path, int mode) {
    if (match_path(path) >= 0) return (mode & W_OK) ? (errno = EACCES, -1) : 0;
    return real_access(path, mode);
}

int epoll_ctl(int epfd, int op, int fd, struct epoll_event* ev) {
    vdev_t* d = find_fd(fd);
    if (d && (op == EPOLL_CTL_ADD || op == EPOLL_CTL_MOD)) fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
    return real_epoll_ctl(epfd, op, fd, ev);
}

/* ---------------------------------------------------------------- ioctls */
static void set_bit(uint8_t* bits, int len, int bit) {
    if (bit >= 0 && bit / 8 < len) bits[bit / 8] |= (uint8_t)(1u << (bit % 8));
}

static int copy_str(void* arg, int len, const char* s) {
    if (len <= 0) return 0;
    strncpy((char*)arg, s, (size_t)len - 1);
    ((char*)arg)[len - 1] = 0;
    int n = (int)strlen(s) + 1;
    return n < len ? n : len;
}

static int js_ioctl(vdev_t* d, unsigned long req, void* arg) {
    const int len = (int)_IOC_SIZE(req);
    switch (_IOC_NR(req)) {
        case 0x01: *(uint32_t*)arg = JS_VERSION; return 0;                 /* JSIOCGVERSION */
        case 0x11: *(uint8_t*)arg = (uint8_t)d->cfg.num_axes; return 0;    /* JSIOCGAXES */
        case 0x12: *(uint8_t*)arg = (uint8_t)d->cfg.num_btns; return 0;    /* JSIOCGBUTTONS */
        case 0x13: return copy_str(arg, len, d->cfg.name);                 /* JSIOCGNAME(len) */
        case 0x21: memcpy(d->corr, arg, sizeof(struct js_corr) * (d->cfg.num_axes < MAX_AXES ? d->cfg.num_axes : MAX_AXES));
                   return 0;                                                /* JSIOCSCORR */
        case 0x22: memcpy(arg, d->corr, sizeof(struct js_corr) * (d->cfg.num_axes < MAX_AXES ? d->cfg.num_axes : MAX_AXES));
                   return 0;                                                /* JSIOCGCORR */
        case 0x32: {                                                       /* JSIOCGAXMAP */
            memset(arg, 0, (size_t)len);
            int n = d->cfg.num_axes < len ? d->cfg.num_axes : len;
            memcpy(arg, d->cfg.axes_map, (size_t)n);
            return 0;
        }
        case 0x34: {                                                       /* JSIOCGBTNMAP */
            memset(arg, 0, (size_t)len);
            int n = d->cfg.num_btns * 2 < len ? d->cfg.num_btns : len / 2;
            memcpy(arg, d->cfg.btn_map, (size_t)n * 2);
            return 0;
        }
        case 0x31: case 0x33: errno = EPERM; return -1;                    /* JSIOCSAXMAP / JSIOCSBTNMAP */
        default: errno = EINVAL; return -1;
    }
}

static void absinfo_for(int code, struct input_absinfo* a) {
    memset(a, 0, sizeof(*a));
    if (code == ABS_Z || code == ABS_RZ) {        /* analog triggers, 0..255 like xpad */
        a->minimum = 0;
        a->maximum = 255;
    } else if (code >= ABS_HAT0X && code <= ABS_HAT3Y) {
        a->minimum = -1;
        a->maximum = 1;
    } else {                                      /* sticks */
        a->minimum = -32767;
        a->maximum = 32767;
        a->fuzz = 16;
        a->flat = 128;
    }
}

static int ev_ioctl(vdev_t* d, unsigned long req, void* arg) {
    const unsigned type = _IOC_TYPE(req), nr = _IOC_NR(req);
    const int len = (int)_IOC_SIZE(req);
    if (type == 'j') return js_ioctl(d, req, arg);
    if (type != 'E') { errno = ENOTTY; return -1; }
    if (nr >= _IOC_NR(EVIOCGABS(0)) && nr < _IOC_NR(EVIOCGABS(0)) + ABS_CNT && _IOC_DIR(req) == _IOC_READ) {
        absinfo_for((int)(nr - _IOC_NR(EVIOCGABS(0))), (struct input_absinfo*)arg);
        return 0;
    }
    if (nr >= _IOC_NR(EVIOCGBIT(0, 0)) && nr < _IOC_NR(EVIOCGBIT(EV_MAX, 0))) {
        uint8_t* bits = (uint8_t*)arg;
        memset(bits, 0, (size_t)len);
        switch (nr - _IOC_NR(EVIOCGBIT(0, 0))) {
            case 0:
                set_bit(bits, len, EV_SYN);
                set_bit(bits, len, EV_KEY);
                set_bit(bits, len, EV_ABS);
                set_bit(bits, len, EV_FF);  /* advertised (rumble requests are accepted and ignored) */
                break;
            case EV_KEY:
                for (int i = 0; i < d->cfg.num_btns && i < MAX_BTNS; i++) set_bit(bits, len, d->cfg.btn_map[i]);
                break;
            case EV_ABS:
                for (int i = 0; i < d->cfg.num_axes && i < MAX_AXES; i++) set_bit(bits, len, d->cfg.axes_map[i]);
                break;
            default:
                break;
        }
        return len;
    }
    if (nr == _IOC_NR(EVIOCGNAME(0))) return copy_str(arg, len, d->cfg.name);
    if (nr == _IOC_NR(EVIOCGPHYS(0))) {
        char phys[64];
        snprintf(phys, sizeof(phys), "usb-selkies-virtual-%d/input0", d->pad);
        return copy_str(arg, len, phys);
    }
    if (nr == _IOC_NR(EVIOCGUNIQ(0))) {
        char uniq[32];
        snprintf(uniq, sizeof(uniq), "SELKIES-PAD-%d", d->pad);
        return copy_str(arg, len, uniq);
    }
    if (nr == _IOC_NR(EVIOCGPROP(0)) || nr == _IOC_NR(EVIOCGKEY(0)) || nr == _IOC_NR(EVIOCGLED(0)) ||
        nr == _IOC_NR(EVIOCGSW(0))) {
        memset(arg, 0, (size_t)len);  /* no properties; every key, LED and switch released */
        return len;
    }
    switch (req) {
        case EVIOCGVERSION: *(int*)arg = EV_VERSION; return 0;
        case EVIOCGID: {
            struct input_id* id = (struct input_id*)arg;
            id->bustype = BUS_USB;
            id->vendor = d->cfg.vendor;
            id->product = d->cfg.product;
            id->version = d->cfg.version;
            return 0;
        }
        case EVIOCGRAB: return 0;
        case EVIOCSFF: {
            struct ff_effect* e = (struct ff_effect*)arg;
            if (e->id < 0) e->id = 0;
            return 0;
        }
        case EVIOCRMFF: return 0;
        case EVIOCGEFFECTS: *(int*)arg = 0; return 0;
        default: errno = EINVAL; return -1;
    }
}

int ioctl(int fd, unsigned long req, ...) {
    va_list ap;
    va_start(ap, req);
    void* arg = va_arg(ap, void*);
    va_end(ap);
    vdev_t* d = find_fd(fd);
    if (!d) return real_ioctl(fd, req, arg);
    return d->kind == KIND_JS ? js_ioctl(d, req, arg) : ev_ioctl(d, req, arg);
}
