// Probe: does v_mfma_f64_16x16x4f64 co-execute with VALU v_fma_f64 on gfx950?
// mode 0: VALU-only waves; 1: MFMA-only waves; 2: half the waves VALU, half MFMA.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k(double* out, int mode, int iters) {
    const int w = threadIdx.x >> 6;
    const bool do_mfma = mode == 1 || (mode == 2 && (w & 1));
    double a0 = threadIdx.x * 1e-3, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    const double x = 0.999999, y = 1e-7;
    if (do_mfma) {
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c3, 0, 0, 0);
        }
    } else {
        for (int i = 0; i < iters * 8; ++i) {  // 8 independent chains x 8 FMAs per iteration
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                a0 = fma(a0, x, y); a1 = fma(a1, x, y); a2 = fma(a2, x, y); a3 = fma(a3, x, y);
                a4 = fma(a4, x, y); a5 = fma(a5, x, y); a6 = fma(a6, x, y); a7 = fma(a7, x, y);
            }
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + c0[0] + c1[1] + c2[2] + c3[3];
}
int main() {
    double* d; (void)hipMalloc(&d, 1024 * 256 * 8 * 8);
    hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    const int iters = 4000;
    for (int blocksPerCU : {1, 2}) {
        for (int mode = 0; mode < 3; ++mode) {
            const int grid = 256 * blocksPerCU;
            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, mode, 10);
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, d, mode, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1);
            // per wave: VALU waves do iters*8*32 FMA (wave64) ; MFMA waves do iters*4 MFMA
            const double waves = grid * 4.0;
            const double vw = mode == 0 ? waves : (mode == 2 ? waves / 2 : 0), mw = waves - vw;
            const double vflop = vw * 64 * 2.0 * iters * 8 * 32, mflop = mw * 4.0 * iters * 2048;
            printf("blocks/CU %d mode %d: %.3f ms  VALU %.1f TF  MFMA %.1f TF  total %.1f TF\n", blocksPerCU, mode, ms,
                   vflop / ms / 1e9, mflop / ms / 1e9, (vflop + mflop) / ms / 1e9);
        }
    }
    return 0;
}
