// X11 MIT-SHM region grabber. libX11 / libXext / libXfixes are resolved with
// dlopen at run time: the library loads on hosts without X, and the reference's
// XShm + XFixes capture path (ximagesrc / pixelflux) is used
// when an X server (Xvfb or Xorg) is reachable. The SHM segment is page-locked
// for HIP (hipHostRegister) so the H2D upload DMAs straight out of it.
#include "frame_source.h"
#include <X11/Xlib.h>
#include <dlfcn.h>
#include <algorithm>
#include <hip/hip_runtime_api.h>
#include <string.h>
#include <sys/ipc.h>
#include <sys/shm.h>
#include <vector>

namespace sk {
namespace {

struct XShmSegmentInfo_ {
    unsigned long shmseg;
    int shmid;
    char* shmaddr;
    int readOnly;
};
struct XFixesCursorImage_ {
    short x, y;
    unsigned short width, height, xhot, yhot;
    unsigned long cursor_serial;
    unsigned long* pixels;
    Atom atom;
    const char* name;
};

struct XApi {
    void* x11 = nullptr;
    void* xext = nullptr;
    void* xfixes = nullptr;
    Display* (*OpenDisplay)(const char*) = nullptr;
    int (*CloseDisplay)(Display*) = nullptr;
    Window (*DefRootWindow)(Display*) = nullptr;
    int (*DefScreen)(Display*) = nullptr;
    Visual* (*DefVisual)(Display*, int) = nullptr;
    int (*DefDepth)(Display*, int) = nullptr;
    int (*Sync)(Display*, Bool) = nullptr;
    int (*Free)(void*) = nullptr;
    Bool (*ShmQueryExtension)(Display*) = nullptr;
    XImage* (*ShmCreateImage)(Display*, Visual*, unsigned int, int, char*, XShmSegmentInfo_*,
                              unsigned int, unsigned int) = nullptr;
    Bool (*ShmAttach)(Display*, XShmSegmentInfo_*) = nullptr;
    Bool (*ShmDetach)(Display*, XShmSegmentInfo_*) = nullptr;
    Bool (*ShmGetImage)(Display*, Drawable, XImage*, int, int, unsigned long) = nullptr;
    XFixesCursorImage_* (*FixesGetCursorImage)(Display*) = nullptr;
    // XDamage (optional, libXdamage): which rows changed since the previous grab
    void* xdamage = nullptr;
    Bool (*DamageQueryExtension)(Display*, int*, int*) = nullptr;
    unsigned long (*DamageCreate)(Display*, Drawable, int) = nullptr;
    void (*DamageSubtract)(Display*, unsigned long, unsigned long, unsigned long) = nullptr;
    unsigned long (*FixesCreateRegion)(Display*, XRectangle*, int) = nullptr;
    XRectangle* (*FixesFetchRegion)(Display*, unsigned long, int*) = nullptr;

    bool load_damage() {
        if (!xfixes) return false;
        xdamage = dlopen("libXdamage.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!xdamage) return false;
        DamageQueryExtension = reinterpret_cast<decltype(DamageQueryExtension)>(dlsym(xdamage, "XDamageQueryExtension"));
        DamageCreate = reinterpret_cast<decltype(DamageCreate)>(dlsym(xdamage, "XDamageCreate"));
        DamageSubtract = reinterpret_cast<decltype(DamageSubtract)>(dlsym(xdamage, "XDamageSubtract"));
        FixesCreateRegion = reinterpret_cast<decltype(FixesCreateRegion)>(dlsym(xfixes, "XFixesCreateRegion"));
        FixesFetchRegion = reinterpret_cast<decltype(FixesFetchRegion)>(dlsym(xfixes, "XFixesFetchRegion"));
        return DamageQueryExtension && DamageCreate && DamageSubtract && FixesCreateRegion && FixesFetchRegion;
    }

    bool load(std::string* err) {
        x11 = dlopen("libX11.so.6", RTLD_NOW | RTLD_LOCAL);
        xext = dlopen("libXext.so.6", RTLD_NOW | RTLD_LOCAL);
        xfixes = dlopen("libXfixes.so.3", RTLD_NOW | RTLD_LOCAL);
        if (!x11 || !xext) {
            if (err) *err = "libX11/libXext not found";
            return false;
        }
#define SYM(lib, dst, name)                                    \
    dst = reinterpret_cast<decltype(dst)>(dlsym(lib, name));   \
    if (!dst) { if (err) *err = std::string("missing ") + name; return false; }
        SYM(x11, OpenDisplay, "XOpenDisplay");
        SYM(x11, CloseDisplay, "XCloseDisplay");
        SYM(x11, DefRootWindow, "XDefaultRootWindow");
        SYM(x11, DefScreen, "XDefaultScreen");
        SYM(x11, DefVisual, "XDefaultVisual");
        SYM(x11, DefDepth, "XDefaultDepth");
        SYM(x11, Sync, "XSync");
        SYM(x11, Free, "XFree");
        SYM(xext, ShmQueryExtension, "XShmQueryExtension");
        SYM(xext, ShmCreateImage, "XShmCreateImage");
        SYM(xext, ShmAttach, "XShmAttach");
        SYM(xext, ShmDetach, "XShmDetach");
        SYM(xext, ShmGetImage, "XShmGetImage");
#undef SYM
        if (xfixes)
            FixesGetCursorImage =
                reinterpret_cast<decltype(FixesGetCursorImage)>(dlsym(xfixes, "XFixesGetCursorImage"));
        return true;
    }
};

class X11Source : public FrameSource {
   public:
    X11Source(int x, int y, int w, int h, bool cursor) : x_(x), y_(y), w_(w), h_(h), cursor_(cursor) {}
    ~X11Source() override {
        for (Seg& g : seg_) {
            if (dpy_ && g.attached) api_.ShmDetach(dpy_, &g.shm);
            if (dpy_ && g.img) {
                g.img->data = nullptr;
                api_.Free(g.img);
            }
        }
        if (dpy_) api_.CloseDisplay(dpy_);
        for (Seg& g : seg_)
            if (g.shm.shmaddr && g.shm.shmaddr != (char*)-1) {
                if (g.registered) hipHostUnregister(g.shm.shmaddr);
                shmdt(g.shm.shmaddr);
            }
    }
    bool open(const char* display, std::string* err) {
        if (!api_.load(err)) return false;
        dpy_ = api_.OpenDisplay(display);
        if (!dpy_) {
            if (err) *err = "cannot open X display";
            return false;
        }
        if (!api_.ShmQueryExtension(dpy_)) {
            if (err) *err = "MIT-SHM extension unavailable";
            return false;
        }
        int scr = api_.DefScreen(dpy_);
        if (api_.DefDepth(dpy_, scr) < 24) {
            if (err) *err = "X screen depth < 24 not supported";
            return false;
        }
        // kRing MIT-SHM images used round robin: a grabbed frame stays valid while the
        // next one is captured (its H2D upload overlaps that grab, FrameSource::ring()).
        for (Seg& g : seg_) {
            memset(&g.shm, 0, sizeof(g.shm));
            g.img = api_.ShmCreateImage(dpy_, api_.DefVisual(dpy_, scr), 24, ZPixmap, nullptr, &g.shm,
                                        (unsigned)w_, (unsigned)h_);
            if (!g.img || g.img->bits_per_pixel != 32) {
                if (err) *err = "XShmCreateImage failed (need 32 bpp)";
                return false;
            }
            size_t bytes = (size_t)g.img->bytes_per_line * g.img->height;
            g.shm.shmid = shmget(IPC_PRIVATE, bytes, IPC_CREAT | 0600);
            if (g.shm.shmid < 0) {
                if (err) *err = "shmget failed";
                return false;
            }
            g.shm.shmaddr = (char*)shmat(g.shm.shmid, nullptr, 0);
            shmctl(g.shm.shmid, IPC_RMID, nullptr);
            if (g.shm.shmaddr == (char*)-1) {
                if (err) *err = "shmat failed";
                return false;
            }
            g.img->data = g.shm.shmaddr;
            g.shm.readOnly = False;
            if (!api_.ShmAttach(dpy_, &g.shm)) {
                if (err) *err = "XShmAttach failed";
                return false;
            }
            g.attached = true;
            api_.Sync(dpy_, False);
            g.registered = hipHostRegister(g.shm.shmaddr, bytes, hipHostRegisterDefault) == hipSuccess;
        }
        root_ = api_.DefRootWindow(dpy_);
        int ev = 0, er = 0;
        if (api_.load_damage() && api_.DamageQueryExtension(dpy_, &ev, &er)) {
            damage_ = api_.DamageCreate(dpy_, root_, 3 /* XDamageReportNonEmpty */);
            region_ = api_.FixesCreateRegion(dpy_, nullptr, 0);
        }
        return true;
    }
    const uint8_t* grab(int* stride) override {
        cur_ = (cur_ + 1) % kRing;
        XImage* img = seg_[cur_].img;
        // the damage accumulated so far, taken BEFORE the image: anything drawn in between
        // is in the pixels and reported again next frame (over-reporting is harmless)
        fetch_damage();
        if (!api_.ShmGetImage(dpy_, root_, img, x_, y_, AllPlanes)) {
            dmg_carry_ = true;   // the drained rows are not in any image yet: report them next time
            return nullptr;
        }
        dmg_carry_ = false;
        if (cursor_ && api_.FixesGetCursorImage) {
            if (overlay_cursor_) fetch_cursor();
            else composite_cursor(img);
        }
        *stride = img->bytes_per_line;
        return (const uint8_t*)img->data;
    }
    int ring() const override { return kRing; }
    const char* name() const override { return "x11-shm"; }
    // XDamage rows of the capture region; unknown on the first grab, without the
    // extension, or while the cursor is drawn into the image on the host.
    bool damage(std::vector<int>* rows) override {
        if (!dmg_ok_ || (cursor_ && !overlay_cursor_)) return false;
        *rows = dmg_rows_;
        return true;
    }
    void set_cursor_overlay(bool on) override { overlay_cursor_ = on; }
    bool cursor(int* x, int* y, int* w, int* h, unsigned long* serial, unsigned long have,
                std::vector<uint8_t>* bgra) override {
        if (!cursor_ || !overlay_cursor_ || !have_cursor_) return false;
        *x = cx_;
        *y = cy_;
        *w = cw_;
        *h = ch_;
        *serial = cserial_;
        if (have != cserial_ && bgra) *bgra = cpx_;
        return true;
    }

   private:
    void fetch_damage() {
        if (!damage_) return;
        api_.DamageSubtract(dpy_, damage_, 0, region_);
        int n = 0;
        XRectangle* r = api_.FixesFetchRegion(dpy_, region_, &n);
        if (!dmg_carry_) dmg_rows_.clear();   // after a failed grab the drained rows stay
        for (int i = 0; r && i < n; i++) {
            if (r[i].x >= x_ + w_ || r[i].x + (int)r[i].width <= x_) continue;   // outside the region
            const int y0 = std::max(0, r[i].y - y_), y1 = std::min(h_, r[i].y + (int)r[i].height - y_);
            if (y0 < y1) { dmg_rows_.push_back(y0); dmg_rows_.push_back(y1); }
        }
        if (r) api_.Free(r);
        api_.Sync(dpy_, True);   // drop the DamageNotify events nobody reads
        dmg_ok_ = grabs_++ > 0;  // the first grab has no previous frame
    }

    // Cursor state for the encoder overlay: position every grab, pixels when the
    // cursor image changes (XFixes cursor_serial).
    void fetch_cursor() {
        XFixesCursorImage_* ci = api_.FixesGetCursorImage(dpy_);
        if (!ci) return;
        cx_ = ci->x - ci->xhot - x_;
        cy_ = ci->y - ci->yhot - y_;
        if (!have_cursor_ || ci->cursor_serial != cserial_ || ci->width != cw_ || ci->height != ch_) {
            cw_ = ci->width;
            ch_ = ci->height;
            cserial_ = ci->cursor_serial;
            cpx_.resize((size_t)cw_ * ch_ * 4);
            for (int i = 0; i < cw_ * ch_; i++) {   // ARGB32 longs, premultiplied -> BGRA bytes
                const uint32_t argb = (uint32_t)ci->pixels[i];
                for (int c = 0; c < 4; c++) cpx_[(size_t)i * 4 + c] = (uint8_t)(argb >> (8 * c));
            }
        }
        have_cursor_ = true;
        api_.Free(ci);
    }

    // K13: server-side cursor composite (small, CPU; alpha in ARGB32 longs)
    void composite_cursor(XImage* img) {
        XFixesCursorImage_* ci = api_.FixesGetCursorImage(dpy_);
        if (!ci) return;
        int cx = ci->x - ci->xhot - x_, cy = ci->y - ci->yhot - y_;
        uint8_t* base = (uint8_t*)img->data;
        for (int j = 0; j < ci->height; j++) {
            int py = cy + j;
            if (py < 0 || py >= h_) continue;
            for (int i = 0; i < ci->width; i++) {
                int px = cx + i;
                if (px < 0 || px >= w_) continue;
                uint32_t argb = (uint32_t)ci->pixels[j * ci->width + i];
                uint32_t a = argb >> 24;
                if (!a) continue;
                uint8_t* d = base + (size_t)py * img->bytes_per_line + 4 * px;
                for (int c = 0; c < 3; c++) {
                    uint32_t s = (argb >> (8 * c)) & 255;  // premultiplied B, G, R
                    d[c] = (uint8_t)(s + (d[c] * (255 - a) + 127) / 255);
                }
            }
        }
        api_.Free(ci);
    }

    XApi api_;
    Display* dpy_ = nullptr;
    static constexpr int kRing = 2;
    struct Seg {
        XShmSegmentInfo_ shm{};
        XImage* img = nullptr;
        bool attached = false, registered = false;
    };
    Seg seg_[kRing];
    int cur_ = kRing - 1;
    Window root_ = 0;
    unsigned long damage_ = 0, region_ = 0;   // XDamage object and the XFixes region it is drained into
    std::vector<int> dmg_rows_;
    bool dmg_ok_ = false;
    bool dmg_carry_ = false;   // the last grab failed after draining damage
    long long grabs_ = 0;
    int x_, y_, w_, h_;
    bool cursor_;
    bool overlay_cursor_ = false, have_cursor_ = false;
    int cx_ = 0, cy_ = 0, cw_ = 0, ch_ = 0;
    unsigned long cserial_ = 0;
    std::vector<uint8_t> cpx_;
};

}  // namespace

std::unique_ptr<FrameSource> make_x11_source(const char* display, int x, int y, int w, int h,
                                             bool capture_cursor, std::string* err) {
    std::unique_ptr<X11Source> s(new X11Source(x, y, w, h, capture_cursor));
    if (!s->open(display, err)) return nullptr;
    return s;
}

}  // namespace sk
