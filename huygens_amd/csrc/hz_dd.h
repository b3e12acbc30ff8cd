// hz_dd.h -- double-double (hi + lo, ~106-bit) arithmetic for the carry powers of the block
// engines, host and device.
//
// Why: the block engines move a band's state over long spans with a power of its transition
// matrix (M^256 in the general engine's row carries, M^(64 L) per LTI tile, M^(seg_len) per time
// segment).  The SAME rounded matrix is then applied hundreds of times, so its rounding acts as a
// fixed perturbation of the dynamics.  For a (near-)defective pole pair -- the reference recipe's
// last band sits on Nyquist, a double pole at -R (tests/resynthesis.cpp:48-54) -- a relative
// perturbation eps of M^k moves the double eigenvalue by ~k sqrt(eps) (Jordan block), and over the
// horizon 1/(1-R) of an R = 0.9999 band that grew to 1e-4 .. 1e-3 relative output error against
// the sequential recurrence.  The sequential recurrence's own roundings differ at every sample and
// do not add up that way.  With the powers held to ~2^-106 (hi, lo) and applied as hi S + lo S,
// the fixed perturbation drops below the per-application rounding and the engines agree with the
// recurrence again (tests/test_fb_highq_gpu.py).
//
// Every function below turns FMA contraction off: hipcc contracts a * b + c by default on the
// device, which fused a product into the sum of the following two_sum / quick_two_sum and broke
// the error-free transformations (measured: the carries came out ~1e-14 off, like plain double).
#pragma once

#include <hip/hip_runtime.h>

namespace hz_dd {

struct dd {
    double hi, lo;
};

__host__ __device__ inline dd two_sum(double a, double b) {
#pragma clang fp contract(off)
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline dd quick_two_sum(double a, double b) {
#pragma clang fp contract(off)
    const double s = a + b;
    return {s, b - (s - a)};
}
__host__ __device__ inline dd two_prod(double a, double b) {
#pragma clang fp contract(off)
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
__host__ __device__ inline dd add(dd a, dd b) {
#pragma clang fp contract(off)
    dd s = two_sum(a.hi, b.hi);
    const dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_two_sum(s.hi, s.lo);
}
__host__ __device__ inline dd mul(dd a, dd b) {
#pragma clang fp contract(off)
    dd p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return quick_two_sum(p.hi, p.lo);
}
__host__ __device__ inline dd mul(dd a, double b) {
#pragma clang fp contract(off)
    dd p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return quick_two_sum(p.hi, p.lo);
}
__host__ __device__ inline dd neg(dd a) { return {-a.hi, -a.lo}; }

// C = A B, O x O row-major
template <int O>
__host__ __device__ inline void mat_mul(const dd (&A)[O][O], const dd (&B)[O][O], dd (&C)[O][O]) {
    for (int i = 0; i < O; ++i)
        for (int j = 0; j < O; ++j) {
            dd acc{0.0, 0.0};
            for (int q = 0; q < O; ++q) acc = add(acc, mul(A[i][q], B[q][j]));
            C[i][j] = acc;
        }
}

// P = B^e by binary powering (e >= 0)
template <int O>
__host__ __device__ inline void mat_pow(const dd (&B)[O][O], long e, dd (&P)[O][O]) {
    dd Pw[O][O], T[O][O];
    for (int i = 0; i < O; ++i)
        for (int j = 0; j < O; ++j) {
            Pw[i][j] = B[i][j];
            P[i][j] = {i == j ? 1.0 : 0.0, 0.0};
        }
    for (; e > 0; e >>= 1) {
        if (e & 1) {
            mat_mul<O>(P, Pw, T);
            for (int i = 0; i < O; ++i)
                for (int j = 0; j < O; ++j) P[i][j] = T[i][j];
        }
        if (e > 1) {
            mat_mul<O>(Pw, Pw, T);
            for (int i = 0; i < O; ++i)
                for (int j = 0; j < O; ++j) Pw[i][j] = T[i][j];
        }
    }
}

// (hi, lo) planes -> dd matrix
template <int O>
__host__ __device__ inline void load(const double* hi, const double* lo, dd (&M)[O][O]) {
    for (int i = 0; i < O; ++i)
        for (int j = 0; j < O; ++j) M[i][j] = {hi[i * O + j], lo[i * O + j]};
}

}  // namespace hz_dd
