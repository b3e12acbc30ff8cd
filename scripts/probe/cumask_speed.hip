// cumask_speed.hip -- does a CU-masked stream run a latency-bound kernel as fast as a full-chip
// stream with the same number of resident workgroups, and alone vs beside a busy complementary
// stream?  hipcc --offload-arch=gfx950 -O2 -o cumask_speed cumask_speed.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

// a window-transform-shaped kernel: 256 threads read 4096 doubles, do FP64 work, write 4096
__global__ __launch_bounds__(256) void work_kernel(const double* __restrict__ x, double* __restrict__ y, int iters) {
    __shared__ double s[4096];
    const long base = (long)blockIdx.x * 4096;
    double v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = x[base + threadIdx.x + 256 * i];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; ++i) s[threadIdx.x + 256 * i] = v[i];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = fma(v[i], 0.999, s[(threadIdx.x * 17 + 256 * i + it) & 4095]);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) y[base + threadIdx.x + 256 * i] = v[i];
}

__global__ void busy_kernel(long long spin) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(4);
}

int main() {
    const int nwg = 258;
    double *x, *y;
    CK(hipMalloc(&x, sizeof(double) * 4096 * nwg));
    CK(hipMalloc(&y, sizeof(double) * 4096 * nwg));
    CK(hipMemset(x, 0, sizeof(double) * 4096 * nwg));
    hipStream_t s0, sA, sB;
    CK(hipStreamCreate(&s0));
    std::vector<unsigned> mA(8, 0xFF00FF00u), mB(8, 0x00FF00FFu);
    CK(hipExtStreamCreateWithCUMask(&sA, 8, mA.data()));
    CK(hipExtStreamCreateWithCUMask(&sB, 8, mB.data()));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](hipStream_t s, int reps, int iters) -> float {
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(work_kernel, dim3(nwg), dim3(256), 0, s, x, y, iters);
        hipEventRecord(e0, s);
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(work_kernel, dim3(nwg), dim3(256), 0, s, x, y, iters);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        return 1e3f * ms / reps;
    };
    for (int iters : {1, 20}) {
        std::printf("iters %d: full-chip stream %.2f us, masked A alone %.2f us", iters, timeit(s0, 50, iters),
                    timeit(sA, 50, iters));
        // beside a busy kernel on B (256 WGs spinning 2 ms)
        hipLaunchKernelGGL(busy_kernel, dim3(256), dim3(256), 0, sB, 200000LL);
        std::printf(", masked A beside busy B %.2f us", timeit(sA, 50, iters));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(busy_kernel, dim3(256), dim3(256), 0, sB, 200000LL);
        std::printf(", full-chip beside busy B %.2f us\n", timeit(s0, 50, iters));
        CK(hipDeviceSynchronize());
    }
    // event fork / join cost: s0 -> A, B -> s0 with empty work
    hipEvent_t ef, ea, eb;
    CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ea, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
    for (int pass = 0; pass < 2; ++pass) {
        hipEventRecord(e0, s0);
        const int reps = 100;
        for (int r = 0; r < reps; ++r) {
            hipEventRecord(ef, s0);
            hipStreamWaitEvent(sA, ef, 0);
            hipStreamWaitEvent(sB, ef, 0);
            hipLaunchKernelGGL(work_kernel, dim3(nwg), dim3(256), 0, sA, x, y, 1);
            hipLaunchKernelGGL(work_kernel, dim3(nwg), dim3(256), 0, sB, x, y, 1);
            hipEventRecord(ea, sA);
            hipEventRecord(eb, sB);
            hipStreamWaitEvent(s0, ea, 0);
            hipStreamWaitEvent(s0, eb, 0);
        }
        hipEventRecord(e1, s0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        if (pass) std::printf("fork/join of one kernel on A and one on B: %.2f us per step\n", 1e3f * ms / reps);
    }
    std::printf("cumask speed ok\n");
    return 0;
}
