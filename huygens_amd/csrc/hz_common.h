// hz_common.h -- shared host/device helpers of libhuygens_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "../../include/huygens_hip.h"

namespace hz {

// src/includes.h:30-32: the reference's own constants (truncated PI, int SR).
constexpr double kPI = 3.14159265359;
constexpr double kE = 2.718281828459045;
constexpr int kSR = 48000;

// src/includes.h:38-48
double relaxation(double k);

// per-thread last-error message (hz_last_error)
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));

// Checks that a gfx950 device is visible and selects it; returns HZ_OK or an error.
int select_device(int device);

// Timing events of the profile counters: no system-scope fence on record, so a record between
// two kernels does not write back / invalidate L2 (it cost 5-10 us per record on the C2 step).
// Only hipEventElapsedTime after a stream synchronize reads them.
inline hipError_t prof_event_create(hipEvent_t* e) {
    return hipEventCreateWithFlags(e, hipEventDisableSystemFence);
}

}  // namespace hz

#define HZ_TRY_HIP(expr)                                                                   \
    do {                                                                                   \
        hipError_t hz_e_ = (expr);                                                         \
        if (hz_e_ != hipSuccess) {                                                         \
            hz::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(hz_e_),       \
                          __FILE__, __LINE__);                                             \
            return HZ_E_HIP;                                                               \
        }                                                                                  \
    } while (0)

#define HZ_TRY(expr)                  \
    do {                              \
        int hz_r_ = (expr);           \
        if (hz_r_ != HZ_OK) return hz_r_; \
    } while (0)

// ---------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------
namespace hz {

// Distortion functors (replacing the host function pointer of
// Filterbank::operator()(T, T(*)(T)), src/filterbank.h:133-139).
// softclip's tail (|v| >= width): out of line, so the engines' unrolled per-sample loops keep one
// call site per sample instead of 16 inlined atan sequences -- inline, the general engine's mix
// kernel spilled its recurrence registers (244 B per lane of scratch, 23.8 GB of scratch traffic
// per C2 call, rocprofv3 PMC round 6); the identity branch, the common one at the reference's width
// 0.125, stays inline
__device__ __noinline__ double softclip_tail(double v, double width);
__device__ __noinline__ inline double softclip_tail(double v, double width) {
    const double sign = (v > 0.0) ? 1.0 : ((v < 0.0) ? -1.0 : 0.0);
    const double gap = v - sign * width;
    return sign * width + (1 - width) * 2.0 / kPI * atan(kPI * gap / (2 * (1 - width)));
}

template <int DIST>
__device__ __forceinline__ double dist_apply(double v, double param) {
    if constexpr (DIST == HZ_DIST_SOFTCLIP) {
        // tests/filterbank.cpp:158-166 (abs taken as fabs)
        const double width = param;
        if (fabs(v) < width) return v;
        return softclip_tail(v, width);
    } else if constexpr (DIST == HZ_DIST_SATURATE) {
        return 2.0 / kPI * atan(2 * kPI * v / 2.0);  // tests/filterbank.cpp:173-176
    } else if constexpr (DIST == HZ_DIST_LIMITER) {
        return 2.0 / kPI * atan(v);  // src/wave.h:150 (FUNCTIONAL lookup)
    } else {
        return v;
    }
}

}  // namespace hz
