// HIP error checking: every failing runtime call raises (and is surfaced to Python as
// RuntimeError by pybind11), so a missing/broken GPU path fails loudly.
#pragma once
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#define HIP_CHECK(expr)                                                                              \
    do {                                                                                             \
        hipError_t _e = (expr);                                                                      \
        if (_e != hipSuccess)                                                                        \
            throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " +   \
                                     __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);        \
    } while (0)

#include <mutex>
#include <set>
#include <tuple>

namespace mx {
// Function attributes (e.g. the dynamic-LDS limit) are per device: raise one once for every
// (device, kernel, attribute, value), thread-safe -- sessions of one process run on several
// host threads (run_sessions) and a process may drive more than one GPU.
inline void ensure_func_attr(const void* fn, hipFuncAttribute attr, int value) {
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    static std::mutex mu;
    static std::set<std::tuple<int, const void*, int, int>> done;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_tuple(dev, fn, (int)attr, value);
    if (done.count(key)) return;
    HIP_CHECK(hipFuncSetAttribute(fn, attr, value));
    done.insert(key);
}
}  // namespace mx

#include <chrono>
#include <cstdlib>
#include <thread>

namespace mx {
// Wait for a frame's completion event.  MXDESK_WAIT=spin polls hipEventQuery (the collecting
// thread owns a core: wake-up within ~1 us of the GPU finishing); MXDESK_WAIT=sleep polls it
// every 25 us and sleeps in between (many sessions per process: a hundred frame threads waiting
// in hipEventSynchronize kept the serve processes' host CPUs busy, profiles/r06_density); default
// hipEventSynchronize.
// Rate of the device wall clock (wall_clock64() / s_memrealtime) in kHz = ticks per ms.
inline double device_clock_khz() {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
        return 100000.0;  // 100 MHz on CDNA
    return (double)khz;
}
inline void wait_event(hipEvent_t e) {
    static const int mode = [] {
        const char* v = std::getenv("MXDESK_WAIT");
        const std::string s = v ? v : "";
        return s == "spin" ? 1 : (s == "sleep" ? 2 : 0);
    }();
    if (mode == 0) {
        HIP_CHECK(hipEventSynchronize(e));
        return;
    }
    for (;;) {
        const hipError_t r = hipEventQuery(e);
        if (r == hipSuccess) return;
        if (r != hipErrorNotReady) HIP_CHECK(r);
        if (mode == 2) std::this_thread::sleep_for(std::chrono::microseconds(25));
    }
}
}  // namespace mx
