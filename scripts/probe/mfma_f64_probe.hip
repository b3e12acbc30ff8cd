// Probe: v_mfma_f64_16x16x4f64 issue rate on gfx950 -- per-SIMD throughput and the cost of a
// dependent accumulator chain, by independent chains per wave (CH) and waves per SIMD.
// Sizes the band-state pass (hz_fb_state.hip) against the FP64 matrix peak.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_f64_probe scripts/probe/mfma_f64_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

template <int CH>
__global__ void chain_kernel(const double* __restrict__ in, double* __restrict__ out, int iters) {
    const int lane = threadIdx.x & 63;
    // operands differ per wave and lane (random-looking data: the clock the chip holds under an
    // FP64 MFMA load depends on the operand bits)
    const int wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    double a = in[(lane + 7 * wv) & 127], b = in[(64 + lane + 13 * wv) & 127];
    f64x4 acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = f64x4{0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the VALU comparison: plain FP64 FMA chains, CH independent per lane
template <int CH>
__global__ void fma_kernel(const double* __restrict__ in, double* __restrict__ out, int iters) {
    const int lane = threadIdx.x & 63;
    const double a = in[lane], b = in[64 + lane];
    double acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int c = 0; c < CH; ++c) acc[c] = fma(a, acc[c], b);
    }
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
static void run(const char* name, K k, int waves_per_cu, int ch, bool mfma, double* din, double* dout) {
    const int blocks = 256 * 4, threads = 64 * waves_per_cu / 4;   // 4 blocks per CU
    const int iters = 2000;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, din, dout, 10);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, din, dout, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = (double)blocks * threads / 64;
    const double ops = waves * iters * 8 * ch;                       // instructions
    const double flops = ops * (mfma ? 2.0 * 16 * 16 * 4 : 2.0 * 64);
    std::printf("%-10s waves/CU %2d chains %d: %8.3f ms  %7.2f TFLOP/s  %6.1f cycles/instr/SIMD @2.4GHz\n", name,
                waves_per_cu, ch, ms, flops / (ms * 1e-3) / 1e12,
                (ms * 1e-3 * 2.4e9) / (ops / (256.0 * 4)));
}

int main(int argc, char**) {
    double *din, *dout;
    hipMalloc(&din, 128 * sizeof(double));
    hipMalloc(&dout, 1 << 24);
    double h[128];
    const bool rnd = argc > 1;   // any argument: random operands in [-1, 1)
    unsigned long long z = 88172645463325252ull;
    for (int i = 0; i < 128; ++i) {
        z ^= z << 13;
        z ^= z >> 7;
        z ^= z << 17;
        h[i] = rnd ? (double)(z >> 11) * 0x1p-52 - 1.0 : 1.0 + 1e-9 * i;
    }
    std::printf("operands: %s\n", rnd ? "random [-1, 1)" : "1 + 1e-9 i");
    hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice);
    for (int w : {4, 8, 16}) {
        run("mfma", chain_kernel<1>, w, 1, true, din, dout);
        run("mfma", chain_kernel<2>, w, 2, true, din, dout);
        run("mfma", chain_kernel<4>, w, 4, true, din, dout);
    }
    for (int w : {4, 8, 16}) {
        run("fma", fma_kernel<4>, w, 4, false, din, dout);
        run("fma", fma_kernel<8>, w, 8, false, din, dout);
    }
    return 0;
}
