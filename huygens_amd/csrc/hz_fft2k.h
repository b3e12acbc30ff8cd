// hz_fft2k.h -- the 2048-point FP64 complex FFT of the stationary engine (hz_fb_resp.hip), one
// transform per 256-thread workgroup, 8 points per thread, fully unrolled for that one size.
//
// The generic LDS passes (hz_fft.h: runtime pass loop, twiddles from a compact LDS table through
// twc) measured ~2 us per radix-8 pass for a lone workgroup on a CU (scripts/probe/
// fft_phase_probe.hip): every instruction's latency is exposed at one wave per SIMD, and the
// table lookups sit on each butterfly's critical path.  Here every pass is a compile-time
// instance, its stage twiddles are loaded from the L2-resident W_4096 table at kernel start
// together with the data (one memory latency for everything), and the first forward / last
// inverse pass run on registers: their groups are exactly the 8 points t + 256 i a thread loads
// or stores.
//
// Forward: DIF, natural order in -> bit-reversed order out (in LDS): R 2 (registers), 3, 3, 3.
// Inverse: DIT, bit-reversed order in (LDS) -> natural order out: R 3, 3, 3, 2 (registers).
// Pass (R, LH): group b owns elements base + (j << LD), j < 2^R, LD = LH - (R - 1) (DIF) with
// base = ((b >> LD) << (LH + 1)) + p, p = b mod 2^LD; DIT: base = ((b >> LH) << (LH + R)) + p,
// p = b mod 2^LH, elements base + (j << LH) -- hz_fft.h's dif_pass / dit_pass, specialised.
#pragma once

#include "hz_fft.h"

namespace hz2k {

constexpr int kLg = 11, kN = 1 << kLg, kT = 256, kPT = kN / kT;

// The transform sits in LDS as interleaved complex (one ds_read_b128 / ds_write_b128 per point) at
// ix(e) = e ^ ((e >> 3) & 31) ^ ((e >> 8) & 31): conflict-free for every pass of the plan and for
// the register pass's stride-256 stores, and at most two-way for the caller's split / merge reads
// at bit-reversed positions (scripts/probe/fft2k_layout.py; the planar layout with one pad per 16
// it replaces cost ~550 LDS bank-conflict cycles per wave in each of the forward and inverse
// kernels, rocprofv3 SQ_LDS_BANK_CONFLICT, profiles/r5/c2_sq)
struct Lds {
    double2 z[kN];
};
__device__ __forceinline__ int ix(int e) { return e ^ ((e >> 3) & 31) ^ ((e >> 8) & 31); }

// forward passes 2-4 and inverse passes 1-3 touch only the 512-point block of the group's wave
// (group b = thread t: block b >> 6 = t >> 6), so between them a wave's own LDS writes need only
// land -- the workgroup barrier stays where data crosses waves (after the register pass, before
// the caller's reads)
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// W_2048^m from the W_4096 table (tw[k] = e^{-2 pi i k / 4096}, k < 2048)
__device__ __forceinline__ double2 w2k(const double2* __restrict__ tw, int m) { return tw[2 * m]; }

// ---- forward (DIF) -------------------------------------------------------------------------
template <int R, int LH>
struct Dif {
    static constexpr int LD = LH - (R - 1), M = 1 << R;
    // stage twiddles of group b: W^(p << (kLg - 1 - LH + k)), k < R
    static __device__ __forceinline__ void load_tw(double2 (&w)[R], int b, const double2* __restrict__ tw) {
        const int p = b & ((1 << LD) - 1);
#pragma unroll
        for (int k = 0; k < R; ++k) w[k] = LD == 0 ? make_double2(1.0, 0.0) : w2k(tw, p << (kLg - 1 - LH + k));
    }
    static __device__ __forceinline__ void regs(double* xr, double* xi, const double2 (&w)[R]) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int S = M >> (k + 1);
#pragma unroll
            for (int j = 0; j < M; ++j) {
                if (j & S) continue;
                const double ar = xr[j], ai = xi[j], cr = xr[j + S], ci = xi[j + S];
                double dr = ar - cr, di = ai - ci;
                if (LD != 0) hz::cmul_tw(dr, di, w[k], false);
                hz::mul_root16(dr, di, (j & (S - 1)) << (4 - R + k), false);
                xr[j] = ar + cr;
                xi[j] = ai + ci;
                xr[j + S] = dr;
                xi[j + S] = di;
            }
        }
    }
    static __device__ __forceinline__ void lds(Lds& s, int b, const double2 (&w)[R]) {
        const int p = b & ((1 << LD) - 1), base = ((b >> LD) << (LH + 1)) + p;
        double xr[M], xi[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const double2 v = s.z[ix(base + (j << LD))];
            xr[j] = v.x;
            xi[j] = v.y;
        }
        regs(xr, xi, w);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            s.z[ix(base + (j << LD))] = make_double2(xr[j], xi[j]);
        }
    }
};

// every twiddle of a thread's forward transform, loaded at kernel start
struct FwdTw {
    double2 p1[2][2], p2[3], p3[3];
    __device__ __forceinline__ void load(const double2* __restrict__ tw) {
        const int t = threadIdx.x;
        Dif<2, 10>::load_tw(p1[0], t, tw);
        Dif<2, 10>::load_tw(p1[1], t + kT, tw);
        Dif<3, 8>::load_tw(p2, t, tw);
        Dif<3, 5>::load_tw(p3, t, tw);
    }
};

// v[i] = z[t + 256 i] in registers -> bit-reversed spectrum in LDS (ends with a barrier)
__device__ __forceinline__ void fwd(Lds& s, double (&vr)[kPT], double (&vi)[kPT], const FwdTw& w) {
    const int t = threadIdx.x;
    // pass 1 (R 2, LH 10) on registers: group t = points t + 512 j (v[0, 2, 4, 6]), group t + 256 =
    // t + 256 + 512 j (v[1, 3, 5, 7])
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        double xr[4], xi[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            xr[j] = vr[g + 2 * j];
            xi[j] = vi[g + 2 * j];
        }
        Dif<2, 10>::regs(xr, xi, w.p1[g]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            vr[g + 2 * j] = xr[j];
            vi[g + 2 * j] = xi[j];
        }
    }
#pragma unroll
    for (int i = 0; i < kPT; ++i) {
        s.z[ix(t + kT * i)] = make_double2(vr[i], vi[i]);
    }
    __syncthreads();
    Dif<3, 8>::lds(s, t, w.p2);
    wave_sync();
    Dif<3, 5>::lds(s, t, w.p3);
    wave_sync();
    const double2 one[3] = {make_double2(1.0, 0.0), make_double2(1.0, 0.0), make_double2(1.0, 0.0)};
    Dif<3, 2>::lds(s, t, one);
    __syncthreads();
}

// ---- inverse (DIT, conjugate twiddles) ---------------------------------------------------------
template <int R, int LH>
struct Dit {
    static constexpr int M = 1 << R;
    // stage twiddles of group b: conj W^(p << (kLg - 1 - LH - k)), k < R
    static __device__ __forceinline__ void load_tw(double2 (&w)[R], int b, const double2* __restrict__ tw) {
        const int p = b & ((1 << LH) - 1);
#pragma unroll
        for (int k = 0; k < R; ++k) w[k] = LH == 0 ? make_double2(1.0, 0.0) : w2k(tw, p << (kLg - 1 - LH - k));
    }
    static __device__ __forceinline__ void regs(double* xr, double* xi, const double2 (&w)[R]) {
#pragma unroll
        for (int k = 0; k < R; ++k) {
            const int S = 1 << k;
#pragma unroll
            for (int j = 0; j < M; ++j) {
                if (j & S) continue;
                double cr = xr[j + S], ci = xi[j + S];
                if (LH != 0) hz::cmul_tw(cr, ci, w[k], true);
                hz::mul_root16(cr, ci, (j & (S - 1)) << (3 - k), true);
                const double ar = xr[j], ai = xi[j];
                xr[j] = ar + cr;
                xi[j] = ai + ci;
                xr[j + S] = ar - cr;
                xi[j + S] = ai - ci;
            }
        }
    }
    static __device__ __forceinline__ void lds(Lds& s, int b, const double2 (&w)[R]) {
        const int p = b & ((1 << LH) - 1), base = ((b >> LH) << (LH + R)) + p;
        double xr[M], xi[M];
#pragma unroll
        for (int j = 0; j < M; ++j) {
            const double2 v = s.z[ix(base + (j << LH))];
            xr[j] = v.x;
            xi[j] = v.y;
        }
        regs(xr, xi, w);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            s.z[ix(base + (j << LH))] = make_double2(xr[j], xi[j]);
        }
    }
};

struct InvTw {
    double2 p2[3], p3[3], p4[2][2];
    __device__ __forceinline__ void load(const double2* __restrict__ tw) {
        const int t = threadIdx.x;
        Dit<3, 3>::load_tw(p2, t, tw);
        Dit<3, 6>::load_tw(p3, t, tw);
        Dit<2, 9>::load_tw(p4[0], t, tw);
        Dit<2, 9>::load_tw(p4[1], t + kT, tw);
    }
};

// bit-reversed spectrum in LDS (the caller's stores, not yet synchronised) -> v[i] = z[t + 256 i]
// in registers, natural order
__device__ __forceinline__ void inv(Lds& s, double (&vr)[kPT], double (&vi)[kPT], const InvTw& w) {
    const int t = threadIdx.x;
    __syncthreads();
    const double2 one[3] = {make_double2(1.0, 0.0), make_double2(1.0, 0.0), make_double2(1.0, 0.0)};
    Dit<3, 0>::lds(s, t, one);
    wave_sync();
    Dit<3, 3>::lds(s, t, w.p2);
    wave_sync();
    Dit<3, 6>::lds(s, t, w.p3);
    __syncthreads();
    // pass 4 (R 2, LH 9) on registers: group t = t + 512 j, group t + 256 = t + 256 + 512 j
#pragma unroll
    for (int i = 0; i < kPT; ++i) {
        const double2 v = s.z[ix(t + kT * i)];
        vr[i] = v.x;
        vi[i] = v.y;
    }
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        double xr[4], xi[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            xr[j] = vr[g + 2 * j];
            xi[j] = vi[g + 2 * j];
        }
        Dit<2, 9>::regs(xr, xi, w.p4[g]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            vr[g + 2 * j] = xr[j];
            vi[g + 2 * j] = xi[j];
        }
    }
}

}  // namespace hz2k
