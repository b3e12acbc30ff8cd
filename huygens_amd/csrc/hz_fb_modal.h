// hz_fb_modal.h -- modal band states for the stationary engine (hz_fb_resp.hip): the band states
// after a stationary call, for banks whose poles sit on one circle at angles on the 2 pi / 8192
// grid (the reference's own resonator recipe: f_i = 0.5 (i + 1) SR / N, R shared,
// tests/resynthesis.cpp:48-54), from one fold of the call's last K inputs and one 8192-point DFT
// instead of the N O K multiply-adds of the MFMA pass (hz_fb_state.h).
//
// A second-order band y = pin (b0 x[t] + b1 x[t-1] + b2 x[t-2]) / (1 + a1 z^-1 + a2 z^-2)
// (src/filterbank.h:178-179 at pre = pin) with poles p, conj p has g[tau] = (p^(tau+1) -
// conj p^(tau+1)) / (p - conj p), so over the window of the last K inputs (the MFMA pass's zero-start
// semantics)
//     y[t] = Im(p U(t)) / Im p,   U(t) = pin (b0 Z(t) + b1 Z(t-1) + b2 Z(t-2)),
//     Z(t) = sum_{tau < K} p^tau x[t - tau],   Z(t-1) = (Z(t) - x[t]) / p.
// With p = p_g e^c, p_g = R_g e^(2 pi i m / L) on the grid (c: the coefficients' own rounding off
// it, |c| K <= 1e-6, checked on the host in long double):
//     Z(T-1) = G0[m] + c G1[m]  (+ O((c K)^2) <= 5e-13),
//     G_j[m] = sum_{r < L} e^(2 pi i m r / L) F_j[r],  F_j[r] = sum_{tau = r mod L} tau^j R_g^tau x[T-1-tau].
// The DFT is four-step, L = 8192 = 64 x 128 (r = r1 + 128 r2, m = k1 + 64 k2, W = e^(2 pi i / L)):
//   phase 1 (workgroup r1, extra workgroups of the forward kernel):
//     A_j[k1][r1] = W^(r1 k1) sum_{r2 < 64} F_j[r1 + 128 r2] W64^(r2 k1)  -- the fold included;
//   phase 2 (workgroup k1, extra workgroups of the inverse kernel, two launches later):
//     G_j[k1 + 64 k2] = sum_{r1 < 128} W128^(r1 k2) A_j[k1][r1], then the states of the bands whose
//     m = k1 (mod 64).
// Bands whose poles (nearly) coincide -- the recipe's Nyquist band is a double pole at -R -- are
// exceptional: a direct dot product of the window with their own response (host, long double),
// accumulated in double-double per 16384-sample chunk (phase 1) and summed in phase 2.
// numpy model and CPU checks: tests/modal_model.py, tests/test_modal_model_cpu.py.
#pragma once

#include <hip/hip_runtime.h>

#include "hz_dd.h"

namespace hz_modal {

constexpr int kL = 8192;           // grid / DFT length
constexpr int kR1 = 128, kR2 = 64; // r = r1 + 128 r2; k = k1 + 64 k2
constexpr int kMaxExc = 8;         // exceptional bands handled by direct dot products
constexpr long kExcChunk = 2048;   // samples per exceptional partial (8 per thread, loaded at once)
constexpr int kThreads = 256;
constexpr int kPhase1 = kR1;       // phase-1 workgroups (one per r1)
constexpr int kParts = 4;          // phase-2 workgroups per k1 (16 bins k2 < 64 each)
constexpr int kPhase2 = kR2 * kParts;   // phase-2 workgroups, + 1 for the exceptional sums

struct BandPar {                   // regular band n
    double pr, pi;                 // pole p = (-a1 / 2, sqrt(a2 - a1^2 / 4))
    double cr, ci;                 // c = log(p / p_g)
    double inv_im;                 // 1 / Im p
    double b0, b1, b2;             // pin * fwd
};

struct ModalArgs {
    int on;                        // 0: no modal work in this launch
    // the window w[i] = x[T - K + i], i < K, in two pieces: w[i] = xw[i] for i < split (the history
    // before a call shorter than K), xw2[i - split] after (the call's input)
    const double* xw;
    const double* xw2;
    long split;
    long K;
    int S;                         // K / kL
    const double* wR;              // [kL] R_g^r
    const double* RL;              // [S] R_g^(kL s)
    const double2* tw;             // [kL] e^(2 pi i q / kL)
    double2* A;                    // [2][64][128]
    const BandPar* par;            // [N]
    const int* csr_ptr;            // [257] bands of bin group w = 4 k1 + k2 / 16 (k1 = m mod 64, k2 = m / 64)
    const int2* csr;               // (band, k2)
    int nexc;
    const int* exc_band;           // [nexc]
    const double* exc_r;           // [nexc][K + 1] responses (pin included)
    double* exc_part;              // [nexc][chunks][4] (hi, lo) of both components
    int exc_chunks;
    int first2, n2;                // the launch's phase-2 workgroups: blockIdx.x in [first2, first2 + n2)
    int per1, per2;                // residues r1 per phase-1 workgroup, k1 per phase-2 workgroup
    int n1, n2p;                   // phase-1 workgroups (128 / per1), phase-2 DFT workgroups (64 / per2)
    double* out;                   // [N][2]: y[T-1], y[T-2]
    int first1, n1l;               // the launch's phase-1 (+ exceptional partial) workgroups when they
                                   // ride in the MAC launch: blockIdx.x in [first1, first1 + n1l)
};

// (the DFT twiddles are staged in LDS: a global table read inside the MAC loops cost one L2
// latency per unrolled batch -- phase 2 took ~19 us that way)
struct Lds1 {
    double red[4][64][2];
    double F[2][64];
    double2 w64[kR2];
};
struct Lds2 {
    double2 a[2][kR1];
    double2 g[2][kR1];
    double2 w128[kR1];
    hz_dd::dd part[kThreads][2];
};

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

__device__ __forceinline__ double win(const ModalArgs& a, long i) { return i < a.split ? a.xw[i] : a.xw2[i - a.split]; }

// phase 1, workgroup r1 < 128: the fold of residues r1 + 128 r2 (r2 < 64) and their 64-point DFTs
__device__ __forceinline__ void phase1(const ModalArgs& a, int r1, Lds1& L) {
    const int t = threadIdx.x, r2 = t & 63, g = t >> 6;
    const int r = r1 + kR1 * r2;
    if (t < kR2) L.w64[t] = a.tw[kR1 * t];   // W64^t
    const double2 wr = a.tw[(r1 * ((t >> 1) & 63)) & (kL - 1)];   // W^(r1 k1) of this thread's output
    const double w0 = a.wR[r];
    double f0 = 0.0, f1 = 0.0;
#pragma unroll 4
    for (int s = g; s < a.S; s += 4) {
        const long tau = r + (long)kL * s;
        const double v = w0 * a.RL[s] * win(a, a.K - 1 - tau);
        f0 += v;
        f1 = fma((double)tau, v, f1);
    }
    L.red[g][r2][0] = f0;
    L.red[g][r2][1] = f1;
    __syncthreads();
    if (t < 128) {
        const int j = t >> 6, q = t & 63;
        L.F[j][q] = ((L.red[0][q][j] + L.red[1][q][j]) + L.red[2][q][j]) + L.red[3][q][j];
    }
    __syncthreads();
    {   // output (j, k1) by two threads, q halves, summed through a lane exchange
        const int j = t >> 7, k1 = (t >> 1) & 63, h = t & 1;
        double re = 0.0, im = 0.0;
#pragma unroll 8
        for (int q = 32 * h; q < 32 * h + 32; ++q) {
            const double2 w = L.w64[(q * k1) & 63];   // W64^(q k1)
            const double f = L.F[j][q];
            re = fma(f, w.x, re);
            im = fma(f, w.y, im);
        }
        re += __shfl_xor(re, 1);
        im += __shfl_xor(im, 1);
        if (!h) a.A[((long)j * kR2 + k1) * kR1 + r1] = cmul(make_double2(re, im), wr);
    }
}

// phase 1, exceptional band e, chunk q: both components' partial dot products in double-double
__device__ __forceinline__ void exc_partial(const ModalArgs& a, int e, int q, Lds2& L) {
    using hz_dd::dd;
    const int t = threadIdx.x;
    const double* r = a.exc_r + (long)e * (a.K + 1);
    const long t0 = (long)q * kExcChunk, t1 = min(t0 + kExcChunk, a.K);
    constexpr int kPer = (int)(kExcChunk / kThreads);
    double rv[kPer], xa[kPer], xb[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {   // every load of the thread first
        const long tau = t0 + t + (long)i * kThreads;
        const bool ok = tau < t1;
        rv[i] = ok ? r[tau] : 0.0;
        xa[i] = ok ? win(a, a.K - 1 - tau) : 0.0;
        xb[i] = (ok && tau < a.K - 1) ? win(a, a.K - 2 - tau) : 0.0;
    }
    dd s0{0.0, 0.0}, s1{0.0, 0.0};
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        s0 = hz_dd::add(s0, hz_dd::two_prod(rv[i], xa[i]));
        s1 = hz_dd::add(s1, hz_dd::two_prod(rv[i], xb[i]));
    }
    // the wave's partials by an xor-shuffle tree, then the four waves in order (lane 0's order is
    // fixed; the LDS tree this replaces spent eight barriers and left the forward launch's last
    // workgroups 1.2 us behind its transforms, stamps in profiles/r5/final/stamps.txt)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s0 = hz_dd::add(s0, dd{__shfl_xor(s0.hi, o, 64), __shfl_xor(s0.lo, o, 64)});
        s1 = hz_dd::add(s1, dd{__shfl_xor(s1.hi, o, 64), __shfl_xor(s1.lo, o, 64)});
    }
    if ((t & 63) == 0) {
        L.part[t >> 6][0] = s0;
        L.part[t >> 6][1] = s1;
    }
    __syncthreads();
    if (t < 2) {
        dd acc = L.part[0][t];
        for (int w = 1; w < kThreads / 64; ++w) acc = hz_dd::add(acc, L.part[w][t]);
        double* o = a.exc_part + ((long)e * a.exc_chunks + q) * 4 + 2 * t;
        o[0] = acc.hi;
        o[1] = acc.lo;
    }
}

// phase 2, workgroup k1 < 64: G_j[k1 + 64 k2] and the states of the bands of residue k1
// phase 2, workgroup w = 4 k1 + part (part < 4): G_j[k1 + 64 k2] for k2 in [16 part, 16 part + 16)
// (32 outputs, eight threads each over r1 eighths; bands use m < L / 2, i.e. k2 < 64) and the
// states of the bands in that bin range
__device__ __forceinline__ void phase2(const ModalArgs& a, int w, Lds2& L) {
    const int t = threadIdx.x, k1 = w >> 2, part = w & 3;
    // every global operand is requested before the first barrier: A, the twiddles, this thread's
    // first band (csr entry, then its parameters) and the last inputs
    const int i0 = a.csr_ptr[w], i1 = a.csr_ptr[w + 1];
    // no band of this shard in the bin range (band shards of a time-sharded bank): nothing to do
    // (uniform over the workgroup, before its first barrier)
    if (i0 == i1) return;
    const bool has = i0 + t < i1;
    int2 bk0 = make_int2(0, 0);
    BandPar P0 = BandPar();
    if (has) {
        bk0 = a.csr[i0 + t];
        P0 = a.par[bk0.x];
    }
    const double x1 = win(a, a.K - 1), x2 = win(a, a.K - 2), x3 = win(a, a.K - 3);
    {
        const int j = t >> 7, r1 = t & 127;
        L.a[j][r1] = a.A[((long)j * kR2 + k1) * kR1 + r1];
        if (t < kR1) L.w128[t] = a.tw[kR2 * t];   // W128^t
    }
    __syncthreads();
    {
        const int o = t >> 3, qq = t & 7;          // output o = (j, k2 - 16 part), r1 eighth qq
        const int j = o >> 4, k2 = 16 * part + (o & 15);
        double re = 0.0, im = 0.0;
#pragma unroll 8
        for (int r1 = 16 * qq; r1 < 16 * qq + 16; ++r1) {
            const double2 wv = L.w128[(r1 * k2) & 127];   // W128^(r1 k2)
            const double2 v = L.a[j][r1];
            re = fma(v.x, wv.x, re);
            re = fma(-v.y, wv.y, re);
            im = fma(v.x, wv.y, im);
            im = fma(v.y, wv.x, im);
        }
        re += __shfl_xor(re, 1);
        im += __shfl_xor(im, 1);
        re += __shfl_xor(re, 2);
        im += __shfl_xor(im, 2);
        re += __shfl_xor(re, 4);
        im += __shfl_xor(im, 4);
        if (!qq) L.g[j][k2] = make_double2(re, im);
    }
    __syncthreads();
    auto state = [&](const int2 bk, const BandPar& P) {
        const double2 g0 = L.g[0][bk.y], g1 = L.g[1][bk.y];
        // Z1 = G0 + c G1; Z(t-1) = (Z(t) - x[t]) / p = (Z(t) - x[t]) conj(p) / |p|^2
        const double2 z1 = make_double2(g0.x + (P.cr * g1.x - P.ci * g1.y), g0.y + (P.cr * g1.y + P.ci * g1.x));
        const double in2 = 1.0 / (P.pr * P.pr + P.pi * P.pi);
        const double2 pc = make_double2(P.pr * in2, -P.pi * in2);
        const double2 z2 = cmul(make_double2(z1.x - x1, z1.y), pc);
        const double2 z3 = cmul(make_double2(z2.x - x2, z2.y), pc);
        const double2 z4 = cmul(make_double2(z3.x - x3, z3.y), pc);
        const double2 u1 = make_double2(P.b0 * z1.x + P.b1 * z2.x + P.b2 * z3.x, P.b0 * z1.y + P.b1 * z2.y + P.b2 * z3.y);
        const double2 u2 = make_double2(P.b0 * z2.x + P.b1 * z3.x + P.b2 * z4.x, P.b0 * z2.y + P.b1 * z3.y + P.b2 * z4.y);
        // Im(p u) / Im p
        a.out[2L * bk.x] = (P.pr * u1.y + P.pi * u1.x) * P.inv_im;
        a.out[2L * bk.x + 1] = (P.pr * u2.y + P.pi * u2.x) * P.inv_im;
    };
    if (has) state(bk0, P0);
    for (int i = i0 + t + kThreads; i < i1; i += kThreads) state(a.csr[i], a.par[a.csr[i].x]);
}

// per1 residues / per2 columns per workgroup, one after the other
__device__ __forceinline__ void phase1_group(const ModalArgs& a, int w, Lds1& L) {
    for (int i = 0; i < a.per1; ++i) {
        phase1(a, w * a.per1 + i, L);
        __syncthreads();
    }
}
__device__ __forceinline__ void phase2_group(const ModalArgs& a, int w, Lds2& L) {
    for (int i = 0; i < a.per2; ++i) {
        phase2(a, w * a.per2 + i, L);
        __syncthreads();
    }
}

// phase 2, the extra workgroup: the exceptional bands' partials summed in double-double, 16 lanes
// per (band, component) series -- lane l takes chunks l, l + 16, ..., then a fixed xor-shuffle tree
// (one lane walking all chunks was a dependent chain of K / 2048 double-double adds: ~17 us at
// R = 0.9999's 248 chunks, the inverse launch's last workgroup)
__device__ __forceinline__ void exc_sum(const ModalArgs& a) {
    const int t = threadIdx.x, ser = t >> 4, sub = t & 15;
    if (ser >= 2 * a.nexc) return;   // whole 16-lane groups: the shuffles below stay inside a group
    const int e = ser >> 1, c = ser & 1;
    hz_dd::dd acc{0.0, 0.0};
    for (int q = sub; q < a.exc_chunks; q += 16) {
        const double* p = a.exc_part + ((long)e * a.exc_chunks + q) * 4 + 2 * c;
        acc = hz_dd::add(acc, hz_dd::dd{p[0], p[1]});
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) acc = hz_dd::add(acc, hz_dd::dd{__shfl_xor(acc.hi, o, 64), __shfl_xor(acc.lo, o, 64)});
    if (sub == 0) a.out[2L * a.exc_band[e] + c] = acc.hi + acc.lo;
}

}  // namespace hz_modal
