// A/B for the C4 STFT frame transform: the 4096-point FP64 DFT of every frame
// of a C4 call (468 frames) as
//   (A) the shipped VALU radix-8 FFT (hz_fft.h fft_fwd_lead<3>, 512 threads per frame, as
//       stft_frame_kernel / stft_pair_kernel run it), and
//   (B) a 64 x 64 four-step DFT on the FP64 matrix cores: Y = X F64 (X[n1][n2] = x[n1 + 64 n2]),
//       Y *= W_4096^(n1 k2), X' = F64 Y (X'[k1][k2] = X[k2 + 64 k1]) -- two complex 64 x 64 x 64
//       GEMMs = 2048 v_mfma_f64_16x16x4f64 per frame (4 real products per complex product).
// Both read the same frames (hop 1024 over a C4 input) and write full spectra; the probe reports
// each kernel's time (HIP events, median of 20), its formulated FP64 rate, MFMA utilisation for B
// (formulated MFMA flops / (78.6 TF/s x time)) and the max difference of the spectra.
// Build: hipcc --offload-arch=gfx950 -O3 -I huygens_amd/csrc -o scripts/probe/stft_mfma_ab scripts/probe/stft_mfma_ab.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "hz_fft.h"

constexpr int kN = 4096, kLg = 12, kHop = 1024;
typedef double f64x4 __attribute__((ext_vector_type(4)));

// (A) one frame per workgroup, 512 threads, natural in -> bit-reversed out (stored bit-reversed)
__global__ __launch_bounds__(512) void fft_valu_kernel(const double* __restrict__ x, const double2* __restrict__ tw,
                                                       double2* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + hz::padded_len(kN);
    double2* T = (double2*)(im + hz::padded_len(kN));
    for (int k = threadIdx.x; k < hz::twc_len(kLg); k += blockDim.x) T[k] = tw[k];
    const double* xf = x + (long)blockIdx.x * kHop;
    for (int n = threadIdx.x; n < kN; n += blockDim.x) {
        re[hz::pad16(n)] = xf[n];
        im[hz::pad16(n)] = 0.0;
    }
    __syncthreads();
    hz::fft_fwd_lead<3>(re, im, kLg, T, true);
    double2* o = out + (long)blockIdx.x * kN;
    for (int q = threadIdx.x; q < kN; q += blockDim.x) o[q] = make_double2(re[hz::pad16(q)], im[hz::pad16(q)]);
}

// (B) one frame per workgroup, 4 waves; wave w owns rows 16w .. 16w + 15 of both products.
// LDS: the frame as X[n1][n2] (re, im planes, row stride 65), W_64^j (j < 64), W_4096^j (j < 4096
// would be 64 KB: the twiddle of step 2 comes from the global table instead)
constexpr int kRow = 65;
__global__ __launch_bounds__(256) void dft_mfma_kernel(const double* __restrict__ x, const double2* __restrict__ tw4096,
                                                       double2* __restrict__ out) {
    __shared__ double xr[64 * kRow], xi[64 * kRow];
    __shared__ double2 w64[64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x < 64) w64[threadIdx.x] = tw4096[threadIdx.x * 64];   // W_64^j = W_4096^(64 j)
    const double* xf = x + (long)blockIdx.x * kHop;
    for (int n = threadIdx.x; n < kN; n += blockDim.x) {   // x[n1 + 64 n2] -> X[n1][n2]
        const int n1 = n & 63, n2 = n >> 6;
        xr[n1 * kRow + n2] = xf[n];
        xi[n1 * kRow + n2] = 0.0;
    }
    __syncthreads();
    // step 1: Y[n1][k2] = sum_n2 X[n1][n2] W_64^(n2 k2): A = X rows 16w + (l & 15), k = n2;
    // B = W_64^(n2 k2), column k2 = 16 cb + (l & 15)
    f64x4 yr[4], yi[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) yr[cb] = yi[cb] = f64x4{0.0, 0.0, 0.0, 0.0};
    const int row = 16 * w + (lane & 15), kk = lane >> 4;
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
        const int n2 = 4 * q + kk;
        const double ar = xr[row * kRow + n2], ai = xi[row * kRow + n2];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            const double2 f = w64[(n2 * (16 * cb + (lane & 15))) & 63];
            yr[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, f.x, yr[cb], 0, 0, 0);
            yr[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, -f.y, yr[cb], 0, 0, 0);
            yi[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar, f.y, yi[cb], 0, 0, 0);
            yi[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ai, f.x, yi[cb], 0, 0, 0);
        }
    }
    __syncthreads();   // every wave has read X: Y (twiddled) overwrites it
    // D layout: row n1 = 16w + (l >> 4) + 4 rr, col k2 = 16 cb + (l & 15); step 2 twiddle
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int n1 = 16 * w + (lane >> 4) + 4 * rr, k2 = 16 * cb + (lane & 15);
            const double2 t = tw4096[(n1 * k2) & (kN - 1)];   // W_4096^(n1 k2), n1 k2 < 4096
            const double a = yr[cb][rr], b = yi[cb][rr];
            xr[n1 * kRow + k2] = a * t.x - b * t.y;
            xi[n1 * kRow + k2] = a * t.y + b * t.x;
        }
    __syncthreads();
    // step 3: X'[k1][k2] = sum_n1 W_64^(k1 n1) Y[n1][k2]: A = W_64^(k1 n1) rows k1 = 16w + (l & 15),
    // k = n1; B = Y[n1][k2], column k2 = 16 cb + (l & 15)
    f64x4 zr[4], zi[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) zr[cb] = zi[cb] = f64x4{0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int q = 0; q < 16; ++q) {
        const int n1 = 4 * q + kk;
        const double2 f = w64[(row * n1) & 63];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
            const int k2 = 16 * cb + (lane & 15);
            const double br = xr[n1 * kRow + k2], bi = xi[n1 * kRow + k2];
            zr[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.x, br, zr[cb], 0, 0, 0);
            zr[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(-f.y, bi, zr[cb], 0, 0, 0);
            zi[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.x, bi, zi[cb], 0, 0, 0);
            zi[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(f.y, br, zi[cb], 0, 0, 0);
        }
    }
    double2* o = out + (long)blockIdx.x * kN;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int k1 = 16 * w + (lane >> 4) + 4 * rr, k2 = 16 * cb + (lane & 15);
            o[k2 + 64 * k1] = make_double2(zr[cb][rr], zi[cb][rr]);
        }
}

static int bitrev_h(int p, int lg) {
    int r = 0;
    for (int i = 0; i < lg; ++i) r |= ((p >> i) & 1) << (lg - 1 - i);
    return r;
}

int main() {
    const int frames = 468;                       // a C4 call: 480,000 samples, hop 1024
    const long nx = (long)(frames - 1) * kHop + kN;
    std::vector<double> hx(nx);
    unsigned long long z = 3;
    for (long i = 0; i < nx; ++i) {                // C4-like input: noise + 8 partials
        z ^= z << 13;
        z ^= z >> 7;
        z ^= z << 17;
        double v = 0.1 * ((double)(z >> 11) * 0x1p-52 - 0.5);
        for (int k = 1; k <= 8; ++k) v += 0.5 * std::sin(2 * M_PI * 220.0 * std::pow(k, 1.5) * i / 48000.0);
        hx[i] = v;
    }
    std::vector<double2> htw(kN);
    for (int k = 0; k < kN; ++k) {
        const long double a = -2.0L * acosl(-1.0L) * k / kN;
        htw[k] = make_double2((double)cosl(a), (double)sinl(a));
    }
    std::vector<double2> hc(hz::twc_len(kLg));
    for (int k = 0; k < hz::twc_len(kLg); ++k) hc[k] = htw[k];
    double* dx;
    double2 *dtw, *dtc, *da, *db;
    hipMalloc(&dx, nx * sizeof(double));
    hipMalloc(&dtw, kN * sizeof(double2));
    hipMalloc(&dtc, hc.size() * sizeof(double2));
    hipMalloc(&da, (long)frames * kN * sizeof(double2));
    hipMalloc(&db, (long)frames * kN * sizeof(double2));
    hipMemcpy(dx, hx.data(), nx * sizeof(double), hipMemcpyHostToDevice);
    hipMemcpy(dtw, htw.data(), kN * sizeof(double2), hipMemcpyHostToDevice);
    hipMemcpy(dtc, hc.data(), hc.size() * sizeof(double2), hipMemcpyHostToDevice);
    const size_t lds_a = sizeof(double) * 2 * hz::padded_len(kN) + sizeof(double2) * hz::twc_len(kLg);
    hipFuncSetAttribute((const void*)fft_valu_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_a);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](auto launch) {
        for (int i = 0; i < 5; ++i) launch();
        std::vector<float> t;
        for (int r = 0; r < 20; ++r) {
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    const float ta = timeit([&] { hipLaunchKernelGGL(fft_valu_kernel, dim3(frames), dim3(512), lds_a, 0, dx, dtc, da); });
    const float tb = timeit([&] { hipLaunchKernelGGL(dft_mfma_kernel, dim3(frames), dim3(256), 0, 0, dx, dtw, db); });
    std::vector<double2> ha((long)frames * kN), hb((long)frames * kN);
    hipMemcpy(ha.data(), da, ha.size() * sizeof(double2), hipMemcpyDeviceToHost);
    hipMemcpy(hb.data(), db, hb.size() * sizeof(double2), hipMemcpyDeviceToHost);
    double err = 0, mag = 0;
    for (int f = 0; f < frames; ++f)
        for (int k = 0; k < kN; ++k) {
            const double2 a = ha[(long)f * kN + bitrev_h(k, kLg)], b = hb[(long)f * kN + k];   // A is bit-reversed
            err = std::max(err, std::max(std::fabs(a.x - b.x), std::fabs(a.y - b.y)));
            mag = std::max(mag, std::max(std::fabs(a.x), std::fabs(a.y)));
        }
    const double fft_flops = 5.0 * kN * kLg * frames;   // algorithmic (radix-2 count)
    const double mfma_flops = 2048.0 * 2 * 16 * 16 * 4 * frames;
    std::printf("C4 frame transforms, %d frames of %d points (forward only):\n", frames, kN);
    std::printf("  A  VALU radix-8 FFT       : %8.2f us   %6.2f TF/s algorithmic (frac %.3f of 78.6)\n", 1e3 * ta,
                fft_flops / (ta * 1e-3) / 1e12, fft_flops / (ta * 1e-3) / 78.6e12);
    std::printf("  B  MFMA 64x64 four-step DFT: %8.2f us   %6.2f TF/s on the matrix cores (MFMA utilisation %.3f); "
                "%6.2f TF/s algorithmic\n", 1e3 * tb, mfma_flops / (tb * 1e-3) / 1e12,
                mfma_flops / (tb * 1e-3) / 78.6e12, fft_flops / (tb * 1e-3) / 1e12);
    std::printf("  max |A - B| = %.3e (max |X| %.3e, relative %.2e)\n", err, mag, err / mag);
    std::printf("  B / A time = %.2f\n", tb / ta);
    return 0;
}
