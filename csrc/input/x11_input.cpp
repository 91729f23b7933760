// Native X11 input injection and cursor watching.
//
// Replaces the reference's mix of pynput, python-xlib XTest and `xdotool`
// subprocesses (input_handler.py:1032-1297) with direct XTest calls:
//  * keys: keysym -> keycode from the server keymap; a keysym that is missing
//    from the map, or whose shift level disagrees with the client's shift state,
//    is bound to a spare "scratch" keycode (both levels) with
//    XChangeKeyboardMapping, so any Unicode keysym types correctly with no
//    xdotool process per key;
//  * pointer: absolute (XTestFakeMotionEvent) and relative motion, buttons 1-9
//    (4/5 = wheel, 6/7 = horizontal wheel);
//  * cursor: XFixes DisplayCursorNotify events on a second connection, image as
//    ARGB32 (input_handler.py:1407-1501 does the same through python-xlib).
// libX11 / libXtst / libXfixes are dlopen'ed so the library loads without X.
#include "../runtime/sk_api.h"
#include "../runtime/encoder_iface.h"
#include <X11/Xlib.h>
#include <dlfcn.h>
#include <poll.h>
#include <string.h>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace sk {
namespace {

struct XFixesCursorImageX {
    short x, y;
    unsigned short width, height, xhot, yhot;
    unsigned long cursor_serial;
    unsigned long* pixels;
    Atom atom;
    const char* name;
};

struct XLib {
    void* x11 = nullptr;
    void* xtst = nullptr;
    void* xfixes = nullptr;
    Display* (*OpenDisplay)(const char*) = nullptr;
    int (*CloseDisplay)(Display*) = nullptr;
    int (*Flush)(Display*) = nullptr;
    int (*Sync)(Display*, Bool) = nullptr;
    int (*Free)(void*) = nullptr;
    int (*Pending)(Display*) = nullptr;
    int (*NextEvent)(Display*, XEvent*) = nullptr;
    int (*ConnNumber)(Display*) = nullptr;
    Window (*DefRootWindow)(Display*) = nullptr;
    int (*DefScreen)(Display*) = nullptr;
    int (*DispWidth)(Display*, int) = nullptr;
    int (*DispHeight)(Display*, int) = nullptr;
    int (*DispKeycodes)(Display*, int*, int*) = nullptr;
    KeySym* (*GetKeyboardMapping)(Display*, KeyCode, int, int*) = nullptr;
    int (*ChangeKeyboardMapping)(Display*, int, int, KeySym*, int) = nullptr;
    Bool (*XTestQueryExtension)(Display*, int*, int*, int*, int*) = nullptr;
    int (*FakeKeyEvent)(Display*, unsigned int, Bool, unsigned long) = nullptr;
    int (*FakeButtonEvent)(Display*, unsigned int, Bool, unsigned long) = nullptr;
    int (*FakeMotionEvent)(Display*, int, int, int, unsigned long) = nullptr;
    int (*FakeRelativeMotionEvent)(Display*, int, int, unsigned long) = nullptr;
    Bool (*FixesQueryExtension)(Display*, int*, int*) = nullptr;
    void (*FixesSelectCursorInput)(Display*, Window, unsigned long) = nullptr;
    XFixesCursorImageX* (*FixesGetCursorImage)(Display*) = nullptr;

    bool load(std::string* err) {
        x11 = dlopen("libX11.so.6", RTLD_NOW | RTLD_LOCAL);
        xtst = dlopen("libXtst.so.6", RTLD_NOW | RTLD_LOCAL);
        xfixes = dlopen("libXfixes.so.3", RTLD_NOW | RTLD_LOCAL);
        if (!x11) {
            *err = "libX11 not found";
            return false;
        }
#define SYM(lib, dst, name)                                                      \
    dst = lib ? reinterpret_cast<decltype(dst)>(dlsym(lib, name)) : nullptr;     \
    if (!dst) { *err = std::string("missing symbol ") + name; return false; }
        SYM(x11, OpenDisplay, "XOpenDisplay");
        SYM(x11, CloseDisplay, "XCloseDisplay");
        SYM(x11, Flush, "XFlush");
        SYM(x11, Sync, "XSync");
        SYM(x11, Free, "XFree");
        SYM(x11, Pending, "XPending");
        SYM(x11, NextEvent, "XNextEvent");
        SYM(x11, ConnNumber, "XConnectionNumber");
        SYM(x11, DefRootWindow, "XDefaultRootWindow");
        SYM(x11, DefScreen, "XDefaultScreen");
        SYM(x11, DispWidth, "XDisplayWidth");
        SYM(x11, DispHeight, "XDisplayHeight");
        SYM(x11, DispKeycodes, "XDisplayKeycodes");
        SYM(x11, GetKeyboardMapping, "XGetKeyboardMapping");
        SYM(x11, ChangeKeyboardMapping, "XChangeKeyboardMapping");
#undef SYM
        if (xtst) {
            XTestQueryExtension = (decltype(XTestQueryExtension))dlsym(xtst, "XTestQueryExtension");
            FakeKeyEvent = (decltype(FakeKeyEvent))dlsym(xtst, "XTestFakeKeyEvent");
            FakeButtonEvent = (decltype(FakeButtonEvent))dlsym(xtst, "XTestFakeButtonEvent");
            FakeMotionEvent = (decltype(FakeMotionEvent))dlsym(xtst, "XTestFakeMotionEvent");
            FakeRelativeMotionEvent = (decltype(FakeRelativeMotionEvent))dlsym(xtst, "XTestFakeRelativeMotionEvent");
        }
        if (xfixes) {
            FixesQueryExtension = (decltype(FixesQueryExtension))dlsym(xfixes, "XFixesQueryExtension");
            FixesSelectCursorInput = (decltype(FixesSelectCursorInput))dlsym(xfixes, "XFixesSelectCursorInput");
            FixesGetCursorImage = (decltype(FixesGetCursorImage))dlsym(xfixes, "XFixesGetCursorImage");
        }
        return true;
    }
};

class X11Input {
   public:
    ~X11Input() {
        if (dpy_) x_.CloseDisplay(dpy_);
    }
    bool open(const char* name, bool cursor_only, std::string* err) {
        if (!x_.load(err)) return false;
        dpy_ = x_.OpenDisplay(name && *name ? name : nullptr);
        if (!dpy_) {
            *err = "cannot open X display";
            return false;
        }
        root_ = x_.DefRootWindow(dpy_);
        if (cursor_only) {
            int eb, er;
            if (!x_.FixesQueryExtension || !x_.FixesQueryExtension(dpy_, &eb, &er)) {
                *err = "XFIXES unavailable";
                return false;
            }
            fixes_event_base_ = eb;
            x_.FixesSelectCursorInput(dpy_, root_, 1 /* XFixesDisplayCursorNotifyMask */);
            x_.Flush(dpy_);
            return true;
        }
        int a, b, c, d;
        if (!x_.XTestQueryExtension || !x_.XTestQueryExtension(dpy_, &a, &b, &c, &d)) {
            *err = "XTEST unavailable";
            return false;
        }
        x_.DispKeycodes(dpy_, &min_kc_, &max_kc_);
        load_keymap();
        return true;
    }

    int key(uint32_t keysym, bool down, bool shift_held) {
        std::lock_guard<std::mutex> g(mu_);
        KeyCode kc = 0;
        if (down) {
            kc = lookup(keysym, shift_held);
            if (!kc) kc = scratch(keysym);
            if (!kc) return -1;
            pressed_[keysym] = kc;
        } else {
            auto it = pressed_.find(keysym);
            if (it != pressed_.end()) {
                kc = it->second;
                pressed_.erase(it);
            } else {
                kc = lookup(keysym, shift_held);
                if (!kc) return 0;  // never pressed
            }
        }
        x_.FakeKeyEvent(dpy_, kc, down ? True : False, 0);
        x_.Flush(dpy_);
        return 0;
    }
    int motion(int x, int y) {
        std::lock_guard<std::mutex> g(mu_);
        x_.FakeMotionEvent(dpy_, -1, x, y, 0);
        x_.Flush(dpy_);
        return 0;
    }
    int motion_rel(int dx, int dy) {
        std::lock_guard<std::mutex> g(mu_);
        x_.FakeRelativeMotionEvent(dpy_, dx, dy, 0);
        x_.Flush(dpy_);
        return 0;
    }
    int button(int b, bool down) {
        std::lock_guard<std::mutex> g(mu_);
        x_.FakeButtonEvent(dpy_, (unsigned)b, down ? True : False, 0);
        x_.Flush(dpy_);
        return 0;
    }
    void screen_size(int* w, int* h) {
        int s = x_.DefScreen(dpy_);
        *w = x_.DispWidth(dpy_, s);
        *h = x_.DispHeight(dpy_, s);
    }
    // Waits up to timeout_ms for a cursor change; 1 = changed, 0 = timeout.
    int cursor_wait(int timeout_ms) {
        bool changed = drain_cursor_events();
        if (changed) return 1;
        pollfd p{x_.ConnNumber(dpy_), POLLIN, 0};
        if (poll(&p, 1, timeout_ms) > 0) changed = drain_cursor_events();
        return changed ? 1 : 0;
    }
    // Copies the current cursor image (ARGB32 premultiplied); returns pixel count or -1.
    int cursor_image(uint64_t* serial, int* w, int* h, int* xhot, int* yhot, uint32_t* argb, int cap) {
        XFixesCursorImageX* ci = x_.FixesGetCursorImage(dpy_);
        if (!ci) return -1;
        *serial = ci->cursor_serial;
        *w = ci->width;
        *h = ci->height;
        *xhot = ci->xhot;
        *yhot = ci->yhot;
        int n = ci->width * ci->height;
        for (int i = 0; i < n && i < cap; i++) argb[i] = (uint32_t)ci->pixels[i];
        x_.Free(ci);
        return n;
    }

   private:
    bool drain_cursor_events() {
        bool changed = false;
        while (x_.Pending(dpy_) > 0) {
            XEvent ev;
            x_.NextEvent(dpy_, &ev);
            if (ev.type == fixes_event_base_ + 1 /* XFixesCursorNotify */) changed = true;
        }
        return changed;
    }
    void load_keymap() {
        int n = max_kc_ - min_kc_ + 1;
        if (map_) x_.Free(map_);
        map_ = x_.GetKeyboardMapping(dpy_, (KeyCode)min_kc_, n, &per_);
        // spare keycodes = ones with no keysym at all (usually several at the top)
        if (scratch_.empty()) {
            for (int kc = max_kc_; kc >= min_kc_ && scratch_.size() < 10; kc--) {
                bool empty = true;
                for (int l = 0; l < per_; l++)
                    if (map_[(kc - min_kc_) * per_ + l] != NoSymbol) empty = false;
                if (empty) scratch_.push_back((KeyCode)kc);
            }
        }
    }
    KeyCode lookup(uint32_t ks, bool shift_held) {
        if (!map_) return 0;
        const int levels = per_ < 2 ? per_ : 2;
        for (int kc = min_kc_; kc <= max_kc_; kc++) {
            // skip our scratch codes: they are handled by scratch()
            for (int l = 0; l < levels; l++) {
                if ((uint32_t)map_[(kc - min_kc_) * per_ + l] != ks) continue;
                bool needs_shift = l == 1;
                // Modifier keys and keys whose level matches the client's shift
                // state are pressed directly.
                if (needs_shift == shift_held || is_modifier(ks) || (l == 0 && lower_equals_upper(kc)))
                    return (KeyCode)kc;
            }
        }
        return 0;
    }
    bool lower_equals_upper(int kc) {
        if (per_ < 2) return true;
        KeySym a = map_[(kc - min_kc_) * per_], b = map_[(kc - min_kc_) * per_ + 1];
        return b == NoSymbol || a == b;
    }
    static bool is_modifier(uint32_t ks) { return (ks >= 0xffe1 && ks <= 0xffee) || ks == 0xfe03; }
    KeyCode scratch(uint32_t ks) {
        if (scratch_.empty()) return 0;
        auto it = scratch_owner_.find(ks);
        if (it != scratch_owner_.end()) return it->second;
        KeyCode kc = scratch_[next_scratch_ % scratch_.size()];
        next_scratch_++;
        for (auto i = scratch_owner_.begin(); i != scratch_owner_.end(); ++i)
            if (i->second == kc) {
                scratch_owner_.erase(i);
                break;
            }
        std::vector<KeySym> syms((size_t)per_, NoSymbol);
        syms[0] = ks;
        if (per_ > 1) syms[1] = ks;
        x_.ChangeKeyboardMapping(dpy_, kc, per_, syms.data(), 1);
        x_.Sync(dpy_, False);
        for (int l = 0; l < per_; l++) map_[(kc - min_kc_) * per_ + l] = syms[(size_t)l];
        scratch_owner_[ks] = kc;
        return kc;
    }

    XLib x_;
    Display* dpy_ = nullptr;
    Window root_ = 0;
    int min_kc_ = 8, max_kc_ = 255, per_ = 0;
    KeySym* map_ = nullptr;
    std::vector<KeyCode> scratch_;
    std::map<uint32_t, KeyCode> scratch_owner_, pressed_;
    size_t next_scratch_ = 0;
    int fixes_event_base_ = 0;
    std::mutex mu_;
};

}  // namespace
}  // namespace sk

using sk::X11Input;

extern "C" {
void* sk_x11_input_open(const char* display, int cursor_only) {
    X11Input* x = new X11Input();
    std::string err;
    if (!x->open(display, cursor_only != 0, &err)) {
        sk::set_last_error("x11 input: " + err);
        delete x;
        return nullptr;
    }
    return x;
}
void sk_x11_input_close(void* h) { delete static_cast<X11Input*>(h); }
int sk_x11_key(void* h, uint32_t keysym, int down, int shift_held) {
    return static_cast<X11Input*>(h)->key(keysym, down != 0, shift_held != 0);
}
int sk_x11_motion(void* h, int x, int y) { return static_cast<X11Input*>(h)->motion(x, y); }
int sk_x11_motion_rel(void* h, int dx, int dy) { return static_cast<X11Input*>(h)->motion_rel(dx, dy); }
int sk_x11_button(void* h, int button, int down) { return static_cast<X11Input*>(h)->button(button, down != 0); }
void sk_x11_screen_size(void* h, int* w, int* hh) { static_cast<X11Input*>(h)->screen_size(w, hh); }
int sk_x11_cursor_wait(void* h, int timeout_ms) { return static_cast<X11Input*>(h)->cursor_wait(timeout_ms); }
int sk_x11_cursor_image(void* h, uint64_t* serial, int* w, int* hh, int* xhot, int* yhot, uint32_t* argb,
                        int cap) {
    return static_cast<X11Input*>(h)->cursor_image(serial, w, hh, xhot, yhot, argb, cap);
}
}
