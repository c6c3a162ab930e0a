// rvz_trace.h — roctx ranges around the C-ABI's host calls (select, eval, backup, env),
// for rocprofv3 --marker-trace timelines. Off unless RVZ_ROCTX=1 in the environment; the roctx
// library (librocprofiler-sdk-roctx.so, ROCm) is opened on first use, so librvz.so has no link
// dependency on it and a disabled range costs one predictable branch. Ranges bracket the
// enqueue of the work (device time is in the kernel trace beside them); under HIP-graph replay
// only the host-side graph launch is bracketed.
#pragma once
#include <dlfcn.h>
#include <stdint.h>
#include <stdlib.h>

namespace rvz {

struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    Roctx() {
        const char* on = getenv("RVZ_ROCTX");
        if (!on || on[0] == '\0' || on[0] == '0') return;
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
        pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
        if (!push || !pop) push = nullptr, pop = nullptr;
    }
    static const Roctx& get() {
        static const Roctx r;
        return r;
    }
};

struct Range {   // RAII: push on construction, pop on every return path
    bool on;
    explicit Range(const char* name) : on(Roctx::get().push != nullptr) {
        if (on) Roctx::get().push(name);
    }
    ~Range() {
        if (on) Roctx::get().pop();
    }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;
};

}  // namespace rvz
