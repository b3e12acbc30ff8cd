// Probe: cost of G x n FP64 no-return atomic adds into an n-sample output (the cross-group
// mix of the Filterbank if it used atomics instead of a partial slab + reduce), vs writing
// the G x n slab and reducing it.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void atomics(double* out, long n, int G) {
    // block g adds its row into out; 1024 threads stride over n
    const int g = blockIdx.x;
    for (long t = threadIdx.x; t < n; t += blockDim.x) atomicAdd(out + t, 1e-3 * (g + 1));
}
__global__ void slab_write(double* slab, long n, int G) {
    const int g = blockIdx.x;
    for (long t = threadIdx.x; t < n; t += blockDim.x) slab[(long)g * n + t] = 1e-3 * (g + 1);
}
__global__ void slab_reduce(const double* slab, long n, int G, double* out) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    double s = 0;
    for (int g = 0; g < G; ++g) s += slab[(long)g * n + t];
    out[t] = s;
}
int main() {
    const long n = 480000; const int G = 256;
    double *out, *slab;
    (void)hipMalloc(&out, n * 8); (void)hipMalloc(&slab, (size_t)G * n * 8);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    float ms;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipMemset(out, 0, n * 8);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(atomics, dim3(G), dim3(1024), 0, 0, out, n, G);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("atomics G=%d n=%ld: %.3f ms\n", G, n, ms);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(slab_write, dim3(G), dim3(1024), 0, 0, slab, n, G);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("slab write: %.3f ms\n", ms);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(slab_reduce, dim3((n + 255) / 256), dim3(256), 0, 0, slab, n, G, out);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("slab reduce: %.3f ms\n", ms);
    }
    return 0;
}
