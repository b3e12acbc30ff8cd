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
#if defined(HZ_STFT_ABLATE) && (HZ_STFT_ABLATE & 16)
    w = make_double2(0.70710678118654752, -0.70710678118654752);
#endif
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

// ---- register-blocked passes over a padded LDS layout (the STFT frame kernel) ----------
// A pass runs R radix-2 stages (radix 2^R, R <= 4) on 2^R elements held in registers, so
// each element makes one LDS round trip per pass instead of one per stage.  Stage twiddles
// are one table lookup per stage, W_N^(p 2^s), times compile-time roots W_L^m of the pass.
// The table is compact (W_N^k for k <= N/8, the rest by symmetry) and lives in LDS.
// Layout: element i lives at pad16(i) = i + i/16 so 2^R-apart strides spread over banks.
__device__ __forceinline__ int pad16(int i) { return i + (i >> 4); }
__host__ __device__ constexpr int padded_len(int N) { return N + (N >> 4); }

// compact twiddle table length: W_N^k for k in [0, N/8] (N >= 8), k in [0, N/4) (N = 4)
__host__ __device__ constexpr int twc_len(int lg) { return lg >= 3 ? (1 << (lg - 3)) + 1 : 1 << (lg - 2); }

// W_N^k for k in [0, N/2) from the compact table
__device__ __forceinline__ double2 twc(const double2* T, int k, int lg) {
    const int q = 1 << (lg - 2);                       // N/4: W^k = -i W^(k - N/4)
    const int e = lg >= 3 ? 1 << (lg - 3) : q;         // N/8: W^m = -i conj(W^(N/4 - m)) above it
    const bool hi = k >= q;
    const int m = hi ? k - q : k;
    const bool mir = m > e;
    const double2 t = T[mir ? q - m : m];
    const double x = mir ? -t.y : t.x, y = mir ? -t.x : t.y;
    return hi ? make_double2(y, -x) : make_double2(x, y);
}

// (x + iy) *= W_16^q = e^(-2 pi i q/16), q in [0, 8) a compile-time constant after
// unrolling (the conjugate root when conj)
__device__ __forceinline__ void mul_root16(double& x, double& y, int q, bool conj) {
    constexpr double r2 = 0.70710678118654752440, c1 = 0.92387953251128675613, s1 = 0.38268343236508977173;
    if (q == 0) return;
    double c, s;   // W = c - i s
    switch (q) {
    case 4: {
        const double t = x;
        x = conj ? -y : y;
        y = conj ? t : -t;
        return;
    }
    case 2: c = r2; s = r2; break;
    case 6: c = -r2; s = r2; break;
    case 1: c = c1; s = s1; break;
    case 3: c = s1; s = c1; break;
    case 5: c = -s1; s = c1; break;
    default: c = -c1; s = s1; break;   // 7
    }
    if (conj) s = -s;
    const double nx = x * c + y * s, ny = y * c - x * s;
    x = nx;
    y = ny;
}

// DIF stages of spans h, h/2, ..., h >> (R-1) (h = 2^lh) on one group in registers; p is
// the group's offset within its span (BASE false: p = 0, every stage twiddle is a root)
template <int R, bool BASE>
__device__ __forceinline__ void dif_regs(double* xr, double* xi, int lg, int lh, int p, const double2* T) {
    constexpr int M = 1 << R;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int S = M >> (k + 1);
        double2 w = make_double2(1.0, 0.0);
        if (BASE) w = twc(T, p << (lg - 1 - lh + k), lg);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            if (j & S) continue;
            const double ar = xr[j], ai = xi[j], cr = xr[j + S], ci = xi[j + S];
            double dr = ar - cr, di = ai - ci;
            if (BASE) cmul_tw(dr, di, w, false);
            mul_root16(dr, di, (j & (S - 1)) << (4 - R + k), false);
            xr[j] = ar + cr;
            xi[j] = ai + ci;
            xr[j + S] = dr;
            xi[j + S] = di;
        }
    }
}

// DIT stages of spans h, 2h, ..., h << (R-1) with conjugate twiddles
template <int R, bool BASE>
__device__ __forceinline__ void dit_regs(double* xr, double* xi, int lg, int lh, int p, const double2* T) {
    constexpr int M = 1 << R;
#pragma unroll
    for (int k = 0; k < R; ++k) {
        const int S = 1 << k;
        double2 w = make_double2(1.0, 0.0);
        if (BASE) w = twc(T, p << (lg - 1 - lh - k), lg);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            if (j & S) continue;
            double cr = xr[j + S], ci = xi[j + S];
            if (BASE) cmul_tw(cr, ci, w, true);
            mul_root16(cr, ci, (j & (S - 1)) << (3 - k), true);
            const double ar = xr[j], ai = xi[j];
            xr[j] = ar + cr;
            xi[j] = ai + ci;
            xr[j + S] = ar - cr;
            xi[j + S] = ai - ci;
        }
    }
}

// one DIF pass over the frame: group b owns {g 2h + p + j d}, d = h >> (R-1)
template <int R>
__device__ __forceinline__ void dif_pass(double* re, double* im, int lg, int lh, const double2* T) {
    constexpr int M = 1 << R;
    const int ld = lh - (R - 1);
    for (int b = threadIdx.x; b < (1 << (lg - R)); b += blockDim.x) {
        const int p = b & ((1 << ld) - 1), base = ((b >> ld) << (lh + 1)) + p;
        double xr[M], xi[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const int e = pad16(base + (j << ld));
            xr[j] = re[e];
            xi[j] = im[e];
        }
        dif_regs<R, true>(xr, xi, lg, lh, p, T);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const int e = pad16(base + (j << ld));
            re[e] = xr[j];
            im[e] = xi[j];
        }
    }
}

// one DIT pass over the frame: group b owns {g h 2^R + p + j h}
template <int R>
__device__ __forceinline__ void dit_pass(double* re, double* im, int lg, int lh, const double2* T) {
    constexpr int M = 1 << R;
    for (int b = threadIdx.x; b < (1 << (lg - R)); b += blockDim.x) {
        const int p = b & ((1 << lh) - 1), base = ((b >> lh) << (lh + R)) + p;
        double xr[M], xi[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const int e = pad16(base + (j << lh));
            xr[j] = re[e];
            xi[j] = im[e];
        }
        dit_regs<R, true>(xr, xi, lg, lh, p, T);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const int e = pad16(base + (j << lh));
            re[e] = xr[j];
            im[e] = xi[j];
        }
    }
}

// Pass plan for N = 2^lg: forward = [lg mod RMAX (if nonzero)], RMAX, ..., RMAX; inverse is
// its mirror.  The last forward and first inverse passes (size fft_rlast) then touch the
// same contiguous groups {b 2^R + j}, which lets a caller fuse them (and a processor) in
// registers.  Each helper ends with a barrier.
template <int RMAX>
__host__ __device__ constexpr int fft_rlast(int lg) { return lg >= RMAX ? RMAX : lg; }

template <int R, bool INV>
__device__ __forceinline__ void fft_pass(double* re, double* im, int lg, int lh, const double2* T) {
    if constexpr (INV) dit_pass<R>(re, im, lg, lh, T);
    else dif_pass<R>(re, im, lg, lh, T);
}

template <int RMAX, bool INV>
__device__ __forceinline__ void fft_pass_r(int R, double* re, double* im, int lg, int lh, const double2* T) {
    switch (R) {
    case 4: if constexpr (RMAX >= 4) fft_pass<4, INV>(re, im, lg, lh, T); break;
    case 3: fft_pass<3, INV>(re, im, lg, lh, T); break;
    case 2: fft_pass<2, INV>(re, im, lg, lh, T); break;
    default: fft_pass<1, INV>(re, im, lg, lh, T); break;
    }
}

// forward passes; `all` false stops before the last one (caller fuses it)
template <int RMAX>
__device__ __forceinline__ void fft_fwd_lead(double* re, double* im, int lg, const double2* T, bool all) {
    int lh = lg - 1, left = lg;
    const int rem = lg % RMAX;
    if (rem && lg > RMAX) {
        fft_pass_r<RMAX, false>(rem, re, im, lg, lh, T);
        __syncthreads();
        lh -= rem;
        left -= rem;
    }
    for (; left > (all ? 0 : fft_rlast<RMAX>(lg)); left -= RMAX, lh -= RMAX) {
        fft_pass_r<RMAX, false>(left < RMAX ? left : RMAX, re, im, lg, lh, T);
        __syncthreads();
    }
}

// inverse passes; `all` false skips the first one (caller fused it)
template <int RMAX>
__device__ __forceinline__ void fft_inv_tail(double* re, double* im, int lg, const double2* T, bool all) {
    const int r0 = fft_rlast<RMAX>(lg);
    int lh = 0, left = lg;
    if (!all) {
        lh = r0;
        left -= r0;
    }
    for (; left > 0;) {
        const int R = left >= RMAX ? RMAX : left;   // the remainder pass comes last
        fft_pass_r<RMAX, true>(R, re, im, lg, lh, T);
        __syncthreads();
        lh += R;
        left -= R;
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
