// Probe: sustained v_mfma_f64_16x16x4f64 rate on gfx950 vs independent chains per wave and
// waves per SIMD, with the shader clock measured in the kernel (clock64 vs wall_clock64).
// Build: hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ __launch_bounds__(1024) void k(double* out, long long* clk, int iters) {
    d4 c[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) c[i] = d4{0, 0, 0, 0};
    const double x = 0.999999 + threadIdx.x * 1e-9, y = 1e-7;
    const long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
            for (int q = 0; q < CH; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c[q], 0, 0, 0);
    }
    const long long c1 = clock64(), w1 = wall_clock64();
    double s = 0;
#pragma unroll
    for (int q = 0; q < CH; ++q) s += c[q][0] + c[q][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = w1 - w0;
    }
}

template <int CH>
void run(double* d, long long* clk, int wavesPerSimd) {
    const int block = 64 * 4 * wavesPerSimd;   // one workgroup per CU, wavesPerSimd waves per SIMD
    const int grid = 256;
    const int iters = 2000 / CH;
    hipLaunchKernelGGL(k<CH>, dim3(grid), dim3(block), 0, 0, d, clk, 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k<CH>, dim3(grid), dim3(block), 0, 0, d, clk, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    long long h[2];
    (void)hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
    const double waves = grid * 4.0 * wavesPerSimd;
    const double flop = waves * (double)iters * 8 * CH * 2048;
    const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;   // wall_clock64: 100 MHz
    const double cyc_per_mfma = (double)h[0] / ((double)iters * 8 * CH * wavesPerSimd);
    printf("chains %d waves/SIMD %d: %.3f ms  %.1f TF/s  shader clock %.2f GHz  %.1f cycles per MFMA per SIMD\n", CH,
           wavesPerSimd, ms, flop / ms / 1e9, ghz, cyc_per_mfma);
}

int main() {
    double* d;
    long long* clk;
    (void)hipMalloc(&d, 256 * 1024 * 8);
    (void)hipMalloc(&clk, 16);
    for (int w : {1, 2, 4}) {
        run<1>(d, clk, w);
        run<2>(d, clk, w);
        run<4>(d, clk, w);
        run<8>(d, clk, w);
    }
    return 0;
}
