// roctx ranges around the host-side stages (capture grab, H2D + graph launch,
// wait, packet assembly) so rocprofv3 --marker-trace lines them up with the
// kernels of the same frame. librocprofiler-sdk-roctx is opened
// at run time: no link dependency, and a missing library or SK_ROCTX=0 turns
// every range into two predictable branches.
#pragma once
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

namespace sk {
namespace trace {

struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    void (*mark)(const char*) = nullptr;
    bool on = false;

    static Roctx& get() {
        static Roctx r = [] {
            Roctx x;
            const char* env = getenv("SK_ROCTX");
            if (env && strcmp(env, "0") == 0) return x;
            void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
            if (!h) return x;
            x.push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
            x.pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
            x.mark = reinterpret_cast<void (*)(const char*)>(dlsym(h, "roctxMarkA"));
            x.on = x.push && x.pop;
            return x;
        }();
        return r;
    }
};

class Range {
public:
    explicit Range(const char* name) : on_(Roctx::get().on) {
        if (on_) Roctx::get().push(name);
    }
    ~Range() {
        if (on_) Roctx::get().pop();
    }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;

private:
    bool on_;
};

inline void mark(const char* name) {
    Roctx& r = Roctx::get();
    if (r.on && r.mark) r.mark(name);
}

}  // namespace trace
}  // namespace sk
