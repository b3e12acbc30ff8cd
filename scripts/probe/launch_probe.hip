// Probe: what a kernel boundary costs on the stream against an in-kernel grid barrier -- sizes the
// stationary engine's kernel fusion.  Back-to-back dependent launches of small kernels (1 and 256
// workgroups), and one 256-workgroup kernel crossing a device-scope counter barrier R times.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/probe/launch_probe scripts/probe/launch_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void tiny_kernel(double* p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1.0;
}

// every workgroup arrives (release), waits until all have arrived (acquire); the counter only grows
__global__ __launch_bounds__(256) void barrier_kernel(unsigned* count, int rounds, double* p) {
    for (int r = 1; r <= rounds; ++r) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)r * gridDim.x;
            long spins = 0;
            while (__hip_atomic_load(count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1L << 26)) break;   // a bounded wait: never hang the device
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) p[blockIdx.x] += 1.0;
}

// the same barrier with a relaxed spin (no cache invalidation per poll) and one acquire fence after
__global__ __launch_bounds__(256) void barrier2_kernel(unsigned* count, int rounds, double* p) {
    for (int r = 1; r <= rounds; ++r) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (unsigned)r * gridDim.x;
            long spins = 0;
            while (__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1L << 26)) break;   // a bounded wait: never hang the device
            }
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) p[blockIdx.x] += 1.0;
}

__global__ void empty_kernel() {}

static float time_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    double* p;
    unsigned* cnt;
    hipMalloc(&p, 4096 * sizeof(double));
    hipMalloc(&cnt, sizeof(unsigned));
    hipMemset(p, 0, 4096 * sizeof(double));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int blocks : {1, 256, 1024}) {
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(tiny_kernel, dim3(blocks), dim3(256), 0, 0, p);
        hipDeviceSynchronize();
        const int reps = 200;
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(tiny_kernel, dim3(blocks), dim3(256), 0, 0, p);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        std::printf("back-to-back tiny kernels, %4d workgroups: %.2f us per kernel\n", blocks,
                    1e3 * time_ms(e0, e1) / reps);
    }
    for (int rounds : {1, 10, 100}) {
        hipMemset(cnt, 0, sizeof(unsigned));
        hipLaunchKernelGGL(barrier_kernel, dim3(256), dim3(256), 0, 0, cnt, rounds, p);
        hipDeviceSynchronize();
        hipMemset(cnt, 0, sizeof(unsigned));
        hipEventRecord(e0);
        hipLaunchKernelGGL(barrier_kernel, dim3(256), dim3(256), 0, 0, cnt, rounds, p);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        unsigned c = 0;
        hipMemcpy(&c, cnt, sizeof(c), hipMemcpyDeviceToHost);
        std::printf("one kernel, 256 workgroups, %3d grid barriers: %.2f us total (count %u of %u)\n", rounds,
                    1e3 * time_ms(e0, e1), c, 256u * rounds);
    }
    for (int rounds : {1, 10, 100}) {
        hipMemset(cnt, 0, sizeof(unsigned));
        hipLaunchKernelGGL(barrier2_kernel, dim3(256), dim3(256), 0, 0, cnt, rounds, p);
        hipDeviceSynchronize();
        hipMemset(cnt, 0, sizeof(unsigned));
        hipEventRecord(e0);
        hipLaunchKernelGGL(barrier2_kernel, dim3(256), dim3(256), 0, 0, cnt, rounds, p);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        std::printf("one kernel, 256 workgroups, %3d relaxed-spin grid barriers: %.2f us total\n", rounds,
                    1e3 * time_ms(e0, e1));
    }
    for (int blocks : {1, 256}) {
        for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, 0);
        hipDeviceSynchronize();
        const int reps = 200;
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(256), 0, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        std::printf("back-to-back empty kernels, %4d workgroups: %.2f us per kernel\n", blocks,
                    1e3 * time_ms(e0, e1) / reps);
    }
    return 0;
}
