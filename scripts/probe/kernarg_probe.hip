// Probe: the cost of reading kernel arguments on MI355X.  Three kernels, one workgroup each, timed by
// HIP events over 2000 back-to-back launches:
//   empty:   nothing
//   karg:    16 kernel-argument dwords read in a dependent chain (each read waits for the last)
//   devbuf:  the same 16 dwords from a device buffer (one pointer argument)
// Output: microseconds per launch.
#include <hip/hip_runtime.h>
#include <cstdio>

struct Big {
    int v[64];
};

__global__ void k_empty(Big b, int* out) {
    if (threadIdx.x == 0 && b.v[0] == 12345) out[0] = 1;
}
__global__ void k_karg(Big b, int* out) {
    int acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        acc += b.v[(4 * i + (acc & 1)) & 63];   // the index depends on the previous value: a chain
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    if (threadIdx.x == 0 && acc == 12345) out[0] = acc;
}
__global__ void k_devbuf(const int* __restrict__ v, int* out) {
    int acc = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        acc += v[(4 * i + (acc & 1)) & 63];
        asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
    }
    if (threadIdx.x == 0 && acc == 12345) out[0] = acc;
}

int main() {
    Big b{};
    for (int i = 0; i < 64; ++i) b.v[i] = 2 * i;
    int *out, *dv;
    hipMalloc(&out, 64);
    hipMalloc(&dv, sizeof(b));
    hipMemcpy(dv, &b, sizeof(b), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int n = 2000;
    for (int rep = 0; rep < 2; ++rep) {
        float ms[3];
        for (int k = 0; k < 3; ++k) {
            for (int i = 0; i < 50; ++i) {
                if (k == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, b, out);
                if (k == 1) hipLaunchKernelGGL(k_karg, dim3(1), dim3(64), 0, 0, b, out);
                if (k == 2) hipLaunchKernelGGL(k_devbuf, dim3(1), dim3(64), 0, 0, (const int*)dv, out);
            }
            hipEventRecord(e0, 0);
            for (int i = 0; i < n; ++i) {
                if (k == 0) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, b, out);
                if (k == 1) hipLaunchKernelGGL(k_karg, dim3(1), dim3(64), 0, 0, b, out);
                if (k == 2) hipLaunchKernelGGL(k_devbuf, dim3(1), dim3(64), 0, 0, (const int*)dv, out);
            }
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
            hipEventElapsedTime(&ms[k], e0, e1);
        }
        std::printf("{\"empty_us\": %.3f, \"karg16_chain_us\": %.3f, \"devbuf16_chain_us\": %.3f}\n", 1e3 * ms[0] / n,
                    1e3 * ms[1] / n, 1e3 * ms[2] / n);
    }
    return 0;
}
