// Frame sources for the capture thread: an X11 MIT-SHM grabber (libX11/libXext
// loaded with dlopen at run time, so the library has no X link dependency) and
// a synthetic desktop renderer for headless hosts.
#pragma once
#include <stdint.h>
#include <memory>
#include <string>
#include <vector>

namespace sk {

class FrameSource {
   public:
    virtual ~FrameSource() = default;
    // Captures one frame; returns a pointer to BGRx pixels (valid until the next
    // grab) and the row stride in bytes, or nullptr on failure.
    virtual const uint8_t* grab(int* stride) = 0;
    // A pointer returned by grab() stays valid for this many grabs (the one that
    // returned it included): with ring() >= 2 the capture loop grabs and uploads
    // frame n+1 while frame n is still being encoded.
    virtual int ring() const { return 1; }
    // Row ranges [y0, y1) (pairs in `rows`) of the last grab that differ from the grab
    // before it; false when the source does not know (the whole frame counts as changed).
    virtual bool damage(std::vector<int>* rows) { (void)rows; return false; }
    virtual const char* name() const = 0;
    // K13 on the GPU: with set_cursor_overlay(true) a source that captures the cursor
    // stops drawing it into the frame and reports it instead; cursor() returns the
    // state as of the last grab (top-left position in frame coordinates, visibility,
    // an image serial) and fills `bgra` (premultiplied) when the serial is not `have`.
    virtual void set_cursor_overlay(bool on) { (void)on; }
    virtual bool cursor(int* x, int* y, int* w, int* h, unsigned long* serial, unsigned long have,
                        std::vector<uint8_t>* bgra) {
        (void)x; (void)y; (void)w; (void)h; (void)serial; (void)have; (void)bgra;
        return false;
    }
};

// X11 region grabber (XShmGetImage of the root window at x,y,w,h). Returns
// nullptr if no display/extension is available.
std::unique_ptr<FrameSource> make_x11_source(const char* display, int x, int y, int w, int h,
                                             bool capture_cursor, std::string* err);

// Synthetic desktop (moving windows, scrolling text, a video-like region).
std::unique_ptr<FrameSource> make_synthetic_source(int w, int h, int kind, uint32_t seed);

// Caller-owned pool of `frames` BGRx frames (stride bytes per row, h rows each),
// grabbed round robin starting at `phase`.
std::unique_ptr<FrameSource> make_pool_source(const uint8_t* base, int frames, int stride, int h, int phase);

}  // namespace sk
