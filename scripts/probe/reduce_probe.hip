// Probe: cross-group reduce of a G x n FP64 slab, row-major [g][n] vs tile-major [tile][g][T].
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(128) void red_rowmajor(const double* slab, long n, int G, double* out) {
    const long t = 2 * ((long)blockIdx.x * 128 + threadIdx.x);
    if (t >= n) return;
    d2 s0 = {0, 0}, s1 = {0, 0};
    for (int g = 0; g < G; g += 8) {
        d2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *(const d2*)(slab + (long)(g + u) * n + t);
#pragma unroll
        for (int u = 0; u < 8; u += 2) { s0 += v[u]; s1 += v[u + 1]; }
    }
    *(d2*)(out + t) = s0 + s1;
}
template <int T>
__global__ __launch_bounds__(256) void red_tilemajor(const double* slab, long n, int G, double* out) {
    // block: one tile, 512 samples (256 threads x 2); grid.x = tiles * (T / 512)
    const int tile = blockIdx.x / (T / 512), part = blockIdx.x % (T / 512);
    const int loc = part * 512 + 2 * threadIdx.x;
    const double* base = slab + (long)tile * G * T + loc;
    d2 s0 = {0, 0}, s1 = {0, 0};
    for (int g = 0; g < G; g += 8) {
        d2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *(const d2*)(base + (long)(g + u) * T);
#pragma unroll
        for (int u = 0; u < 8; u += 2) { s0 += v[u]; s1 += v[u + 1]; }
    }
    const long t = (long)tile * T + loc;
    if (t < n) *(d2*)(out + t) = s0 + s1;
}
int main() {
    const long n = 481280; const int G = 256; constexpr int T = 2048;
    double *out, *slab;
    (void)hipMalloc(&out, n * 8); (void)hipMalloc(&slab, (size_t)G * n * 8);
    (void)hipMemset(slab, 0, (size_t)G * n * 8);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    float ms;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(red_rowmajor, dim3((n / 2 + 127) / 128), dim3(128), 0, 0, slab, n, G, out);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("row-major reduce: %.3f ms  %.2f TB/s\n", ms, G * n * 8.0 / ms / 1e9);
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(red_tilemajor<T>, dim3((n / T) * (T / 512)), dim3(256), 0, 0, slab, n, G, out);
        (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
        printf("tile-major reduce: %.3f ms  %.2f TB/s\n", ms, G * n * 8.0 / ms / 1e9);
    }
    return 0;
}
