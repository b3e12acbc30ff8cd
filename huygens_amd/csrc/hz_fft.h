// hz_fft.h -- LDS-resident FP64 complex FFT building blocks for gfx950 (device side).
//
// Forward: radix-2^2 decimation in frequency, natural order in -> bit-reversed order out.
// Inverse: radix-2^2 decimation in time, bit-reversed in -> natural order out.
// Neither needs a permutation pass: a spectrum is only ever consumed bin-wise (gates,
// masks) or by the matching inverse, so it stays bit-reversed in LDS.  Both are
// unnormalised (FFTW FORWARD e^{-2 pi i jk/N} / BACKWARD e^{+}).
//
// Data: separate re[] / im[] double arrays in LDS (N <= 8192 -> 128 KB).  Twiddles come from
// a global table tw[k] = e^{-2 pi i k/N}, k < N/2, built on the host in long double.
#pragma once

#include <hip/hip_runtime.h>

namespace hz {

__device__ __forceinline__ void cmul_tw(double& r, double& i, double2 w, bool conj) {
    const double wi = conj ? -w.y : w.y;
    const double nr = r * w.x - i * wi;
    const double ni = r * wi + i * w.x;
    r = nr;
    i = ni;
}

// one radix-2 DIF stage of span h: (x[e], x[e+h]) -> (a+c, (a-c) W_{2h}^pos)
__device__ __forceinline__ void dif2_stage(double* re, double* im, int N, int h, const double2* __restrict__ tw) {
    for (int b = threadIdx.x; b < N / 2; b += blockDim.x) {
        const int pos = b & (h - 1), g = b / h;
        const int e0 = g * 2 * h + pos, e1 = e0 + h;
        double ar = re[e0], ai = im[e0], cr = re[e1], ci = im[e1];
        double dr = ar - cr, di = ai - ci;
        cmul_tw(dr, di, tw[pos * (N / (2 * h))], false);
        re[e0] = ar + cr;
        im[e0] = ai + ci;
        re[e1] = dr;
        im[e1] = di;
    }
}

// two DIF stages (spans h, h/2) in registers per quad {p, p+h/2, p+h, p+3h/2}
__device__ __forceinline__ void dif4_stage(double* re, double* im, int N, int h, const double2* __restrict__ tw) {
    const int q = h >> 1;
    for (int b = threadIdx.x; b < N / 4; b += blockDim.x) {
        const int p = b & (q - 1), g = b / q;
        const int e0 = g * 2 * h + p, e1 = e0 + q, e2 = e0 + h, e3 = e2 + q;
        double x0r = re[e0], x0i = im[e0], x1r = re[e1], x1i = im[e1];
        double x2r = re[e2], x2i = im[e2], x3r = re[e3], x3i = im[e3];
        // stage h
        double a0r = x0r + x2r, a0i = x0i + x2i;
        double a2r = x0r - x2r, a2i = x0i - x2i;
        double a1r = x1r + x3r, a1i = x1i + x3i;
        double a3r = x1r - x3r, a3i = x1i - x3i;
        const int st = N / (2 * h);
        cmul_tw(a2r, a2i, tw[p * st], false);
        cmul_tw(a3r, a3i, tw[(p + q) * st], false);
        // stage h/2
        double b1r = a0r - a1r, b1i = a0i - a1i;
        double b3r = a2r - a3r, b3i = a2i - a3i;
        const double2 w = tw[p * 2 * st];
        cmul_tw(b1r, b1i, w, false);
        cmul_tw(b3r, b3i, w, false);
        re[e0] = a0r + a1r;
        im[e0] = a0i + a1i;
        re[e1] = b1r;
        im[e1] = b1i;
        re[e2] = a2r + a3r;
        im[e2] = a2i + a3i;
        re[e3] = b3r;
        im[e3] = b3i;
    }
}

// forward: natural -> bit-reversed (lg = log2 N); caller synchronises before/after
__device__ __forceinline__ void lds_fft_fwd(double* re, double* im, int N, int lg, const double2* __restrict__ tw) {
    int h = N >> 1;
    for (int s = 0; s + 1 < lg; s += 2, h >>= 2) {
        dif4_stage(re, im, N, h, tw);
        __syncthreads();
    }
    if (lg & 1) {
        dif2_stage(re, im, N, 1, tw);
        __syncthreads();
    }
}

// one radix-2 DIT stage of span h with conjugate twiddles: (a + c w̄, a - c w̄)
__device__ __forceinline__ void dit2_stage(double* re, double* im, int N, int h, const double2* __restrict__ tw) {
    for (int b = threadIdx.x; b < N / 2; b += blockDim.x) {
        const int pos = b & (h - 1), g = b / h;
        const int e0 = g * 2 * h + pos, e1 = e0 + h;
        double cr = re[e1], ci = im[e1];
        cmul_tw(cr, ci, tw[pos * (N / (2 * h))], true);
        const double ar = re[e0], ai = im[e0];
        re[e0] = ar + cr;
        im[e0] = ai + ci;
        re[e1] = ar - cr;
        im[e1] = ai - ci;
    }
}

// two DIT stages (spans h, 2h) per quad {p, p+h, p+2h, p+3h}
__device__ __forceinline__ void dit4_stage(double* re, double* im, int N, int h, const double2* __restrict__ tw) {
    for (int b = threadIdx.x; b < N / 4; b += blockDim.x) {
        const int p = b & (h - 1), g = b / h;
        const int e0 = g * 4 * h + p, e1 = e0 + h, e2 = e1 + h, e3 = e2 + h;
        double x0r = re[e0], x0i = im[e0], x1r = re[e1], x1i = im[e1];
        double x2r = re[e2], x2i = im[e2], x3r = re[e3], x3i = im[e3];
        const int st = N / (2 * h);
        const double2 w = tw[p * st];
        cmul_tw(x1r, x1i, w, true);
        cmul_tw(x3r, x3i, w, true);
        const double a0r = x0r + x1r, a0i = x0i + x1i, a1r = x0r - x1r, a1i = x0i - x1i;
        double a2r = x2r + x3r, a2i = x2i + x3i, a3r = x2r - x3r, a3i = x2i - x3i;
        cmul_tw(a2r, a2i, tw[p * (st >> 1)], true);
        cmul_tw(a3r, a3i, tw[(p + h) * (st >> 1)], true);
        re[e0] = a0r + a2r;
        im[e0] = a0i + a2i;
        re[e2] = a0r - a2r;
        im[e2] = a0i - a2i;
        re[e1] = a1r + a3r;
        im[e1] = a1i + a3i;
        re[e3] = a1r - a3r;
        im[e3] = a1i - a3i;
    }
}

// inverse: bit-reversed -> natural, unnormalised
__device__ __forceinline__ void lds_fft_inv(double* re, double* im, int N, int lg, const double2* __restrict__ tw) {
    int h = 1;
    if (lg & 1) {
        dit2_stage(re, im, N, 1, tw);
        __syncthreads();
        h = 2;
    }
    for (; h < N; h <<= 2) {
        dit4_stage(re, im, N, h, tw);
        __syncthreads();
    }
}

__device__ __forceinline__ int bitrev(int p, int lg) { return (int)(__builtin_bitreverse32((unsigned)p) >> (32 - lg)); }

// double-double helpers (stand-ins for the reference's long double accumulators)
__device__ __forceinline__ void two_sum(double a, double b, double& s, double& e) {
    s = a + b;
    const double bb = s - a;
    e = (a - (s - bb)) + (b - bb);
}

__device__ __forceinline__ void dd_add(double& hi, double& lo, double v) {
    double s, e;
    two_sum(hi, v, s, e);
    e += lo;
    hi = s + e;
    lo = e - (hi - s);
}

}  // namespace hz
