// anyorder_probe.hip -- does hipExtLaunchKernel(..., hipExtAnyOrderLaunch) let a kernel start before
// the previous kernel on the same stream has finished (AQL barrier bit cleared) on gfx950?
// hipcc --offload-arch=gfx950 -O2 -o anyorder_probe anyorder_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void spin_kernel(long long* t, long long ticks) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    if (threadIdx.x == 0) {
        t[0] = t0;
        t[1] = __builtin_amdgcn_s_memrealtime();
    }
}

__global__ void stamp_kernel(long long* t) {
    if (threadIdx.x == 0) t[2] = __builtin_amdgcn_s_memrealtime();
}

int main() {
    long long* d;
    if (hipMalloc(&d, 64) != hipSuccess) return 1;
    hipStream_t s;
    if (hipStreamCreate(&s) != hipSuccess) return 1;
    for (int flags : {0, hipExtAnyOrderLaunch}) {
        long long ticks = 100 * 200;   // 200 us at 100 MHz
        void* a1[] = {&d, &ticks};
        void* a2[] = {&d};
        hipError_t e1 = hipExtLaunchKernel((const void*)spin_kernel, dim3(1), dim3(64), a1, 0, s, nullptr, nullptr, 0);
        hipError_t e2 = hipExtLaunchKernel((const void*)stamp_kernel, dim3(1), dim3(64), a2, 0, s, nullptr, nullptr, flags);
        if (hipStreamSynchronize(s) != hipSuccess) return 1;
        long long h[3];
        if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
        std::printf("flags %d (launch %d %d): spin [0, %lld] ticks, second kernel at %lld -> %s\n", flags, (int)e1,
                    (int)e2, h[1] - h[0], h[2] - h[0], h[2] < h[1] ? "OVERLAPPED" : "after");
    }
    // cross-stream ordering by stream memory operations: s2 waits (CP-side) for a value s writes
    hipStream_t s2;
    if (hipStreamCreate(&s2) != hipSuccess) return 1;
    unsigned long long* flag;
    if (hipMalloc(&flag, 64) != hipSuccess || hipMemset(flag, 0, 64) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    for (int mode = 0; mode < 3; ++mode) {   // 0: one stream, 1: value write/wait hand-off, 2: events
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        const int reps = 200;
        long long ticks = 0;
        void* a1[] = {&d, &ticks};
        hipEvent_t ev;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return 1;
        if (hipEventRecord(e0, s) != hipSuccess) return 1;
        for (int r = 0; r < reps; ++r) {
            hipStream_t sa = s, sb = mode ? s2 : s;
            if (hipExtLaunchKernel((const void*)spin_kernel, dim3(1), dim3(64), a1, 0, sa, nullptr, nullptr, 0) != hipSuccess) return 1;
            if (mode == 1) {
                if (hipStreamWriteValue64(sa, flag, (uint64_t)(2 * r + 1), 0) != hipSuccess) return 2;
                if (hipStreamWaitValue64(sb, flag, (uint64_t)(2 * r + 1), hipStreamWaitValueGte, ~0ull) != hipSuccess) return 3;
            } else if (mode == 2) {
                if (hipEventRecord(ev, sa) != hipSuccess || hipStreamWaitEvent(sb, ev, 0) != hipSuccess) return 4;
            }
            if (hipExtLaunchKernel((const void*)spin_kernel, dim3(1), dim3(64), a1, 0, sb, nullptr, nullptr, 0) != hipSuccess) return 1;
            if (mode == 1) {
                if (hipStreamWriteValue64(sb, flag, (uint64_t)(2 * r + 2), 0) != hipSuccess) return 2;
                if (hipStreamWaitValue64(sa, flag, (uint64_t)(2 * r + 2), hipStreamWaitValueGte, ~0ull) != hipSuccess) return 3;
            } else if (mode == 2) {
                if (hipEventRecord(ev, sb) != hipSuccess || hipStreamWaitEvent(sa, ev, 0) != hipSuccess) return 4;
            }
        }
        if (hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        std::printf("mode %s: %.2f us per ping-pong of two empty kernels\n",
                    mode == 0 ? "one stream" : mode == 1 ? "write/wait value" : "event record/wait", 1e3f * ms / reps);
        (void)hipEventDestroy(ev);
        if (hipMemset(flag, 0, 64) != hipSuccess) return 1;
    }
    std::printf("anyorder probe ok\n");
    return 0;
}
