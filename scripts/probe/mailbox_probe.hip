// mailbox_probe.hip -- per-request round trip of a resident GPU poller when the request word and
// its arguments live in (a) pinned host memory (the per-sample server's layout) or (b) fine-grained
// device memory the host stores into directly; the answer goes to pinned host memory in both.
// hipcc --offload-arch=gfx950 -O2 -o mailbox_probe mailbox_probe.hip
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

struct alignas(64) Box {
    long long req;
    long long args[15];
};

__global__ void poller(Box* box, long long* answer, long long count, long long timeout_ticks) {
    if (threadIdx.x != 0) return;
    long long seen = 0;
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (seen < count) {
        long long r;
        for (;;) {
            r = __hip_atomic_load(&box->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
            if (r != seen) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) return;   // bounded
            __builtin_amdgcn_s_sleep(1);
        }
        long long s = 0;
        for (int i = 0; i < 15; ++i) s += __hip_atomic_load(&box->args[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&answer[1], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&answer[0], r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        seen = r;
    }
}

static int run(const char* name, Box* host_view, Box* dev_view, long long* ans_h, long long* ans_d, bool wc) {
    const long long N = 20000;
    hipStream_t s;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return 1;
    host_view->req = 0;
    if (wc) _mm_sfence();
    __atomic_store_n(&ans_h[0], 0LL, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(poller, dim3(1), dim3(64), 0, s, dev_view, ans_d, N, 100LL * 5000000);   // 5 s cap
    if (hipGetLastError() != hipSuccess) return 2;
    std::vector<double> lat;
    bool ok = true;
    for (long long i = 1; i <= N; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < 15; ++k) host_view->args[k] = i + k;
        if (wc) _mm_sfence();
        __atomic_store_n(&host_view->req, i, __ATOMIC_RELEASE);
        if (wc) _mm_sfence();
        while (__atomic_load_n(&ans_h[0], __ATOMIC_ACQUIRE) != i) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                std::printf("%s: request %lld unanswered\n", name, i);
                ok = false;
                break;
            }
        }
        if (!ok) break;
        if (ans_h[1] != 15 * i + 105) {
            std::printf("%s: request %lld wrong sum %lld (torn arguments)\n", name, i, ans_h[1]);
            ok = false;
            break;
        }
        lat.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
    if (!ok) return 3;
    std::sort(lat.begin() + 200, lat.end());
    const size_t m = lat.size() - 200;
    std::printf("%s: round trip median %.2f us, p99 %.2f us, max %.2f us (%zu requests)\n", name, lat[200 + m / 2],
                lat[200 + m * 99 / 100], lat.back(), m);
    return 0;
}

int main() {
    long long* ans_h;
    if (hipHostMalloc((void**)&ans_h, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
    long long* ans_d;
    if (hipHostGetDevicePointer((void**)&ans_d, ans_h, 0) != hipSuccess) return 1;
    // (a) pinned host mailbox
    Box* hb;
    if (hipHostMalloc((void**)&hb, sizeof(Box), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
    Box* hbd;
    if (hipHostGetDevicePointer((void**)&hbd, hb, 0) != hipSuccess) return 1;
    int rc = run("pinned host mailbox", hb, hbd, ans_h, ans_d, false);
    // (b) fine-grained device memory, host stores through the same pointer
    Box* db = nullptr;
    hipError_t e = hipExtMallocWithFlags((void**)&db, sizeof(Box), hipDeviceMallocFinegrained);
    std::printf("fine-grained device alloc: %s\n", hipGetErrorString(e));
    if (e == hipSuccess) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, db) == hipSuccess)
            std::printf("  attributes: type %d, hostPointer %p, devicePointer %p\n", (int)at.type, at.hostPointer,
                        at.devicePointer);
        rc |= run("device mailbox (host stores, sfence)", db, db, ans_h, ans_d, true) << 4;
    }
    std::printf("mailbox probe done rc=%d\n", rc);
    return 0;
}
