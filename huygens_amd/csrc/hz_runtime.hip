// hz_runtime.hip -- library-wide C ABI helpers (errors, device discovery).
#include <cmath>
#include <cfloat>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "hz_common.h"

namespace hz {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

double relaxation(double k) {
    if (k == 0) return 0;
    return std::pow(2.0, std::log2(DBL_EPSILON) / (std::fmax(0, k) * kSR));
}

int select_device(int device) {
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count == 0) {
        set_error("no HIP device visible (hipGetDeviceCount: %s); libhuygens_hip has no CPU fallback",
                  hipGetErrorString(e));
        return HZ_E_NODEV;
    }
    if (device < 0 || device >= count) {
        set_error("device %d out of range [0, %d)", device, count);
        return HZ_E_RANGE;
    }
    hipDeviceProp_t prop;
    HZ_TRY_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device %d is %s, libhuygens_hip is built for gfx950 only", device, prop.gcnArchName);
        return HZ_E_NODEV;
    }
    HZ_TRY_HIP(hipSetDevice(device));
    return HZ_OK;
}

}  // namespace hz

extern "C" {

const char* hz_last_error(void) { return hz::g_err; }

int hz_version(void) { return 1; }

int hz_device_count(void) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return 0;
    return count;
}

}  // extern "C"
