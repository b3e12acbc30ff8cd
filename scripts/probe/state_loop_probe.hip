// Probe: what slows the band-state pass's MFMA loop (fb_state_kernel, hz_fb_state.hip) below the
// FP64 matrix peak.  The kernel's loop shape -- 256 workgroups x 8 waves, per 8192-sample tile one
// 33-step v_mfma_f64_16x16x4f64 chain per wave, A operands from an LDS slab read 4 steps ahead, B
// operands in registers, the next tile staged global -> registers -> LDS between two barriers --
// built up one ingredient at a time:
//   V0  MFMA chain only (A from registers)
//   V1  + A operands read from the LDS slab (4 k-steps ahead)
//   V2  + the per-tile staging: buffer loads of the next-next tile, ds_write of the next, 2 barriers
// Each variant runs 6 tiles (C2's 49,152-sample window); the probe prints µs per launch and the
// MFMA rate.  Build: hipcc --offload-arch=gfx950 -O3 -o scripts/probe/state_loop_probe scripts/probe/state_loop_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int KE = 33, kL = 128, kTile = 8192, kSlab = 16 * kL + 4, kSlabPos = kSlab + 34, kStage = 33;
constexpr int kHalf = 17;

template <int V>
__global__ __launch_bounds__(512) void loop_kernel(const double* __restrict__ x, const double* __restrict__ eop,
                                                   double* __restrict__ out, int tiles, long len,
                                                   long long* __restrict__ clk) {
    const long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, m = w & 3, sb = w >> 2;
    double e[KE];
#pragma unroll
    for (int q = 0; q < KE; ++q) e[q] = eop[(((long)blockIdx.x * 2 + sb) * KE + q) * 64 + lane];
    __shared__ double slab_lds[4][kSlabPos];
    double* slab = slab_lds[m];
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)(len * 8), 0x00020000);
    const int i0 = sb * kHalf;
    const int voff0 = (int)(((long)(16 * m) * kL - 2 + lane + 64 * i0) * 8);
    double st[kHalf];
    auto load_tile = [&](int it) {
        const int v = voff0 + it * kTile * 8;
#pragma unroll
        for (int i = 0; i < kHalf; ++i)
            st[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, v + 512 * i, 0, 0));
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            const int e2 = lane + 64 * (i0 + i);
            if (e2 < kSlab) slab[e2 + 2 * (e2 / kL)] = st[i];
        }
    };
    const int a_pos = (lane & 15) * (kL + 2) + (lane >> 4);
    auto a_at = [&](int q) {
        const int t = 4 * q;
        return t < kL ? slab[a_pos + t] : slab[a_pos + t + 2];
    };
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    load_tile(0);
    store_tile();
    if (V >= 2 && tiles > 1) load_tile(1);
    __syncthreads();
    double areg[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) areg[q] = a_at(q);
    for (int it = 0; it < tiles; ++it) {
        if constexpr (V == 0) {
#pragma unroll
            for (int q = 0; q < KE; ++q) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(areg[q & 3], e[q], acc, 0, 0, 0);
        } else {
            constexpr int EP = 4;
            double xq[EP];
#pragma unroll
            for (int q = 0; q < EP; ++q) xq[q] = a_at(q);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < KE; ++q) {
                const double xa = xq[q % EP];
                if (q + EP < KE) xq[q % EP] = a_at(q + EP);
                __builtin_amdgcn_sched_barrier(0);
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, e[q], acc, 0, 0, 0);
            }
        }
        if constexpr (V >= 2) {
            if (it + 1 < tiles) {
                __syncthreads();
                store_tile();
                if (it + 2 < tiles) load_tile(it + 2);
                __syncthreads();
            }
        }
    }
    out[((long)blockIdx.x * 512 + threadIdx.x) * 4 + 0] = acc[0] + acc[1] + acc[2] + acc[3];
    if (threadIdx.x == 0) {   // in-kernel clock: shader cycles over 100 MHz real-time ticks
        const long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        clk[2 * blockIdx.x] = c1 - c0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    const int G = 256, tiles_max = 60;
    const long len = (long)tiles_max * kTile;
    std::vector<double> hx(len), he((long)G * 2 * KE * 64);
    unsigned long long z = 5;
    auto rnd = [&] {
        z ^= z << 13;
        z ^= z >> 7;
        z ^= z << 17;
        return (double)(z >> 11) * 0x1p-52 - 0.5;
    };
    for (auto& v : hx) v = rnd();
    for (auto& v : he) v = rnd();
    double *dx, *de, *dout;
    long long* dclk;
    hipMalloc(&dclk, (long)G * 2 * 8);
    hipMalloc(&dx, len * 8);
    hipMalloc(&de, he.size() * 8);
    hipMalloc(&dout, (long)G * 512 * 4 * 8);
    hipMemcpy(dx, hx.data(), len * 8, hipMemcpyHostToDevice);
    hipMemcpy(de, he.data(), he.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto run = [&](const char* name, auto k, int tiles) {
        for (int i = 0; i < 2000; ++i) hipLaunchKernelGGL(k, dim3(G), dim3(512), 0, 0, dx, de, dout, tiles, len, dclk);
        std::vector<float> ts;
        for (int r = 0; r < 30; ++r) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(G), dim3(512), 0, 0, dx, de, dout, tiles, len, dclk);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::vector<long long> hc(2 * G);
        hipMemcpy(hc.data(), dclk, hc.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> ghz;
        for (int b = 0; b < G; ++b) ghz.push_back(hc[2 * b + 1] ? 0.1 * hc[2 * b] / hc[2 * b + 1] : 0.0);
        std::sort(ghz.begin(), ghz.end());
        const double mf = (double)G * 8 * tiles * KE * 2048.0;
        std::printf("%-44s %2d tiles %8.2f us  %6.1f TF/s MFMA  in-kernel clock %.2f GHz (median WG), WG span %.2f us\n",
                    name, tiles, 1e3 * ts[15], mf / (ts[15] * 1e-3) / 1e12, ghz[G / 2], hc[1] * 0.01);
    };
    for (int tiles : {6, 60}) {
        run("V0 MFMA chain only", loop_kernel<0>, tiles);
        run("V1 + A from the LDS slab", loop_kernel<1>, tiles);
        run("V2 + staging (loads, ds_write, 2 barriers)", loop_kernel<2>, tiles);
    }
    return 0;
}
