// hz_fb_resp.hip -- the stationary Filterbank<double> engine (bank response convolution).
//
// Once a bank has run converged (pre = pin, gain = gin: hz_fb_lti.hip) with unchanged
// coefficients for K samples, K = its horizon (||M^K||_inf < 2^-53 for every band's state
// transition M, fb_lti_horizon, rounded up to 8192), every band's state is the zero-state response
// of the last K input samples to below an ulp of itself, and the bank's mixdown
// (src/filterbank.h:130,178-179) is ONE linear filter of the input:
//     out[t] = sum_n gin_n y_n[t] = sum_{tau < K} h[tau] x[t - tau],   h[tau] = sum_n gin_n r_n[tau]
// with r_n band n's impulse response at pre = pin_n.  A call then runs as a uniformly partitioned
// overlap-save convolution on FP64 real transforms (P = 2048-sample partitions / output blocks,
// F = 4096-sample windows, each a 2048-point complex FFT of its even/odd samples plus a split):
//   resp_fwd_kernel   one workgroup per window W_j = u[jP, jP + F) of u = [last K inputs | call
//                     input]: its 2049 bins, stored as 2048 complex (bin 0 = X_0) + X_2048 apart
//   resp_mac_kernel   Y_b = sum_{p < Q} H_p Z_{b+Q-1-p} per bin (Q = K / P partition spectra)
//   resp_inv_kernel   one workgroup per output block: the merge + inverse FFT, out = its last P
// Every window and every output block is a transform of its own: roundoff in one block scales
// with that block's own data, never with a louder block elsewhere in the call (the r2 engine's
// packed complex pairs -- window j in the real part, j + D in the imaginary -- leaked 2^-53 of
// block j + D into block j: tests/test_c2_pinned_gpu.py::test_impulse_then_silence_horizon_bound).
// Per output sample that is O(Q + log F) work whatever the number of bands; the bands enter once,
// through h, when coefficients or targets change (resp_h_kernel: each band's response by the
// reference's own recurrence, summed in a fixed order).
//
// The per-band state is kept exact: the last K inputs are the handle's history (updated by every
// converged long call the engine could take, whatever engine ran it), and the band states at the
// call end are their zero-start response over those K samples (the band-state pass on the FP64
// matrix cores, hz_fb_state.h; for calls n >= K it runs as extra workgroups of resp_inv_kernel)
// -- after every call (HZ_FB_RESP_EAGER, default) or only when a later call, get_state, tick or a
// setter needs them (HZ_FB_RESP_LAZY).
// Multi-GPU: time-range shards (hz_fb_set_bank_response + hz_fb_set_time_shard) convolve one
// rank's run of output blocks with the whole bank's response; DESIGN.md 3.6 and 5.
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <string>

#include "hz_fb_impl.h"
#include "hz_fb_state.h"
#include "hz_fft2k.h"
#include "hz_fb_col.h"
#include "hz_fb_modal.h"

namespace {

constexpr int kLgP = 11, kP = 1 << kLgP;   // partition / output block (samples)
constexpr int kF = 2 * kP;                 // window (samples): real transform length
constexpr int kLgH = kLgP, kH = kP;        // complex transform length = bins stored per row
constexpr int kThreads = 256;              // per window / output block
constexpr int kPT = kH / kThreads;         // complex points per thread (8)
constexpr int kMacR = 8;                   // output blocks per MAC thread (partitions padded to it)
constexpr long kMinCall = 16384;           // shortest call that keeps the history
// cost model: stationary when N n >= kBandsPerSample (K + n) (hz_fb_tune_response overrides it)
constexpr long kBandsPerSample = 256;
// The band-state pass of EAGER calls n >= K runs as extra workgroups of the inverse kernel.  Measured
// at C2 (rocprof, per call): every piece of the pass pays its prologue (~4.7 us: the 12.6 MB of B
// operands and the x window arrive at HBM rate) and a CU holds two of these 256-register
// workgroups, so pieces in all three transform kernels made them 17.3 + 15.6 + 14.2 us, pieces in
// the MAC and inverse kernels 9.3 + 17.5 + 16.0, the whole pass in the inverse kernel 9.5 + 9.4 +
// 21.9 us (the transforms run in the state pass's prologue and beside it), against 9.4 + 9.0 + 8.4
// + 19.3 for a separate state kernel, and 51 us per step with that kernel on a second stream (an
// MFMA chain starves the waves beside it on its SIMD: the older wave issues first; s_setprio
// changed nothing)
static_assert(kH == hz2k::kN && kThreads == hz2k::kT, "hz_fft2k.h: 2048 points on 256 threads");

#ifdef HZ_DIAG_STAMPS
// (diagnostic builds) per-workgroup stamps of the forward [0] and MAC [1] kernels: start, operands
// arrived, transform / MACs done, end
__device__ long long g_diag[3][1024][4];   // forward, MAC, inverse
__device__ __forceinline__ void diag_stamp(int k, int i) {
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_diag[k][blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();
}
#define HZ_DIAG_AT(k, i) diag_stamp(k, i)
#else
#define HZ_DIAG_AT(k, i) ((void)0)
#endif

// Aggregate impulse response, one wave (64 bands) per workgroup: part[g][tau] = sum over the
// group's bands of gin_n r_n[tau], r_n = band n's response to a unit impulse with pre = pin_n,
// by the recurrence of filterbank.h:178-179 (oracle order: ff = F[0] x[t] + ... ; y = ff pre -
// sum_k B[k] y[t-1-k]); lanes = bands, 64-sample tiles summed through LDS in band order.
template <int O>
__global__ __launch_bounds__(64) void resp_h_kernel(const double* __restrict__ F, const double* __restrict__ B,
                                                    const double* __restrict__ pin, const double* __restrict__ gin,
                                                    int nbands, long K, double* __restrict__ part) {
#pragma clang fp contract(off)
    __shared__ double s[64][65];
    const int lane = threadIdx.x;
    const int band = blockIdx.x * 64 + lane;
    const bool live = band < nbands;
    double f[O + 1], b[O], y[O];
#pragma unroll
    for (int i = 0; i <= O; ++i) f[i] = live ? F[(long)band * (O + 1) + i] : 0.0;
#pragma unroll
    for (int k = 0; k < O; ++k) {
        b[k] = live ? B[(long)band * O + k] : 0.0;
        y[k] = 0.0;   // y[k] = r[t - 1 - k]
    }
    const double p = live ? pin[band] : 0.0, g = live ? gin[band] : 0.0;
    for (long t0 = 0; t0 < K; t0 += 64) {
        for (int j = 0; j < 64; ++j) {
            const long t = t0 + j;
            double ff = 0.0;   // sum_i F[i] delta[t - i] = F[t] for t <= O
#pragma unroll
            for (int i = 0; i <= O; ++i)
                if (t == i) ff = f[i];
            double bs = 0.0;
#pragma unroll
            for (int k = 0; k < O; ++k) bs += b[k] * y[k];
            const double yt = ff * p - bs;
#pragma unroll
            for (int k = O - 1; k >= 1; --k) y[k] = y[k - 1];
            y[0] = yt;
            s[j][lane] = g * yt;
        }
        __syncthreads();
        double acc = 0.0;
        for (int q = 0; q < 64; ++q) acc += s[lane][q];
        if (t0 + lane < K) part[(long)blockIdx.x * K + t0 + lane] = acc;
        __syncthreads();
    }
}

// h[tau] = sum_g part[g][tau] (fixed order)
__global__ __launch_bounds__(256) void resp_hsum_kernel(const double* __restrict__ part, int G, long K,
                                                        double* __restrict__ h) {
    const long t = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= K) return;
    double acc = 0.0;
    for (int g = 0; g < G; ++g) acc += part[(long)g * K + t];
    h[t] = acc;
}

// ---- real transforms of one window -----------------------------------------------------------
// A window of F real samples x[m] is the 2048-point complex sequence z[n] = x[2n] + i x[2n+1];
// with Zh = FFT(z) (hz_fft2k.h, bit-reversed out), E = (Zh[k] + conj Zh[kH-k]) / 2 and
// O = (Zh[k] - conj Zh[kH-k]) / 2i are the even and odd samples' spectra and
//     X[k] = E + W^k O,   X[kH - k] = conj(E - W^k O),   W = e^{-2 pi i / F},
// one thread per pair (k, kH - k), k = t + 256 i (k = 0 pairs with itself: X_0 and X_kH; thread
// 0 also takes k = kH / 2).  Rows hold X_0 .. X_{kH-1} (X_0 real, imaginary part 0); X_kH (real)
// is kept apart (nyq), so the MAC is one complex product per stored bin.
template <class Load>
__device__ __forceinline__ void real_window_fwd(hz2k::Lds& s, Load load, const double2* __restrict__ tw,
                                                double2* __restrict__ zrow, double* __restrict__ nyq,
                                                bool stamps = false) {
    const int t = threadIdx.x;
    if (stamps) HZ_DIAG_AT(0, 0);
    // every global load of the thread (data, pass twiddles, split twiddles) before the first use
    double vr[kPT], vi[kPT];
#pragma unroll
    for (int i = 0; i < kPT; ++i) {
        const int n = t + i * kThreads;
        const double2 v = load(2 * n);   // samples 2n, 2n + 1
        vr[i] = v.x;
        vi[i] = v.y;
    }
    hz2k::FwdTw ft;
    ft.load(tw);
    double2 w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = tw[t + i * kThreads];
#ifdef HZ_DIAG_STAMPS
    if (stamps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        HZ_DIAG_AT(0, 1);
    }
#endif
    hz2k::fwd(s, vr, vi, ft);   // ends with a barrier
    if (stamps) HZ_DIAG_AT(0, 2);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = t + i * kThreads, kb = (kH - k) & (kH - 1);
        const double2 za = s.z[hz2k::ix(hz::bitrev(k, kLgH))], zb = s.z[hz2k::ix(hz::bitrev(kb, kLgH))];
        const double ar = za.x, ai = za.y, br = zb.x, bi = zb.y;
        const double er = 0.5 * (ar + br), ei = 0.5 * (ai - bi);
        const double orr = 0.5 * (ai + bi), oi = -0.5 * (ar - br);
        const double wr = w[i].x * orr - w[i].y * oi, wi = w[i].x * oi + w[i].y * orr;
        zrow[k] = make_double2(er + wr, ei + wi);
        if (k) zrow[kb] = make_double2(er - wr, wi - ei);
        else *nyq = er - wr;   // X_kH
    }
    if (t == 0) {   // X_{kH/2} = conj Zh[kH/2] (bit-reversed position 1)
        const double2 zm = s.z[hz2k::ix(1)];
        zrow[kH / 2] = make_double2(zm.x, -zm.y);
    }
    if (stamps) HZ_DIAG_AT(0, 3);
}

// Partition spectra H_p = FFT(h[pP, (p+1)P) zero-padded to F) / F (the inverse is unnormalised;
// 1/F is a power of two)
__global__ __launch_bounds__(kThreads) void resp_hspec_kernel(const double* __restrict__ h, long K,
                                                             const double2* __restrict__ tw, double2* __restrict__ H,
                                                             double* __restrict__ Hn) {
    __shared__ hz2k::Lds s;
    const long p0 = (long)blockIdx.x * kP;
    real_window_fwd(
        s,
        [&](int m) {
            auto g = [&](int k) { return (k < kP && p0 + k < K) ? h[p0 + k] * (1.0 / kF) : 0.0; };
            return make_double2(g(m), g(m + 1));
        },
        tw,
        H + (long)blockIdx.x * kH, Hn + blockIdx.x);
}

struct RespArgs {
    const double* hist;   // [K] the K inputs before the call
    const double* x;      // [n] the call's input
    long K, n;            // horizon; the call's length
    long off, n_out;      // outputs of this launch: out[off, off + n_out) (time-range shards)
    int Q, B;             // partitions; output blocks
    int nz;               // windows (forward workgroups)
    const double2* tw;    // W_F^k, k < kH
    double2* Z;           // [Q + B - 1 (+ pad)][kH] window spectra
    double* Zn;           // [..] their bin kH
    const double2* Y;     // [ys][B][kH] output spectra (bins < kH): ys partial sums over the partitions
    int ys;               // (the long-horizon MAC split over chunks of partitions, summed here)
    long ystride;
    const double* Hn;     // [Q] partition spectra at bin kH
    double* out;          // [n]
    // state upkeep, done by the inverse kernel's threads: the history after the call (the last K
    // samples of [hist | x]), the smoothers' closed form, the x history (the last O inputs)
    double* hist_next;
    const double *pg, *pin, *gin;
    double* pg_next;
    double sp_n, sg_n;
    double* xhist_next;
    int N, O;
    int upkeep;           // 0: a plain convolution (the streaming engine's response tail)
    int zero_outside;     // time-range shard: zeros outside [off, off + n_out) (hz_fb_set_time_shard_fill)
};

// u = [hist | x | 0 ...], indexed from the launch's first output block (off)
__device__ __forceinline__ double resp_u(const RespArgs& a, long m) {
    m += a.off;
    if (m < a.K) return a.hist[m];
    m -= a.K;
    return m < a.off + a.n_out ? a.x[m] : 0.0;
}

// The inverse kernel carries the band-state pass (hz_fb_state.h) as extra workgroups past its own
// (SO = the bank's order, 0: none): a CU holds one of each (<= 256 registers per wave, LDS the
// larger of the two), so the latency-bound inverse transforms run beside the state pass.
union RespLds {
    hz2k::Lds fft;
    hz_state::StateLds st;
    hz_modal::Lds2 md;
};
union ModalLds {
    hz_modal::Lds1 m1;
    hz_modal::Lds2 m2;
};
union RespFwdLds {
    hz2k::Lds fft;
    hz_modal::Lds1 m1;
    hz_modal::Lds2 m2;
};


// Z_j = the spectrum of W_j = u[jP, jP + F)
// (modal band states, hz_fb_modal.h: phase 1 and the exceptional partials as workgroups past nz)
__global__ __launch_bounds__(kThreads) void resp_fwd_kernel(RespArgs a, hz_modal::ModalArgs md) {
    __shared__ RespFwdLds u;
    if (md.on && (int)blockIdx.x >= a.nz) {
        HZ_DIAG_AT(0, 0);
        const int i = blockIdx.x - a.nz;
        if (i < md.n1) hz_modal::phase1_group(md, i, u.m1);
        else hz_modal::exc_partial(md, (i - md.n1) / md.exc_chunks, (i - md.n1) % md.exc_chunks, u.m2);
        HZ_DIAG_AT(0, 1);
        HZ_DIAG_AT(0, 2);
        HZ_DIAG_AT(0, 3);
        return;
    }
    hz2k::Lds& s = u.fft;
    const long m0 = (long)blockIdx.x * kP;
    // the pair (m, m + 1), m even, lies in one of hist / x (K and off are even): one 16-byte load
    // when that buffer is 16-byte aligned and the pair is inside the call
    const bool al = ((reinterpret_cast<uintptr_t>(a.hist) | reinterpret_cast<uintptr_t>(a.x)) & 15) == 0;
    real_window_fwd(
        s,
        [&](int mm) {
            const long m = m0 + mm + a.off;
            if (al) {
                if (m + 1 < a.K) return *reinterpret_cast<const double2*>(a.hist + m);
                if (m >= a.K && m + 1 - a.K < a.off + a.n_out) return *reinterpret_cast<const double2*>(a.x + (m - a.K));
            }
            return make_double2(resp_u(a, m0 + mm), resp_u(a, m0 + mm + 1));
        },
        a.tw, a.Z + (long)blockIdx.x * kH, a.Zn + blockIdx.x, true);
}

// Y_b[q] = sum_{p < Q} H_p[q] Z_{b+Q-1-p}[q] for b in [b0, b0 + R): thread = bin q x R output
// blocks.  The R Z values of step p sit in a register ring (element r in slot (r - p) mod R): each
// step brings one new Z value and one H value for R complex MACs.  Partitions are padded to a
// multiple of R with zero spectra (Qp), so every block of R steps loads unguarded.
// QP > 0 (Qp == QP, a compile-time count): every H and Z operand of the thread is loaded before
// the first MAC -- one memory latency per launch (a lone workgroup per CU hides none of it);
// QP == 0: any Qp, the next block's 2R loads issued before this block's MACs.
template <int R, int QP>
__global__ __launch_bounds__(256) void resp_mac_kernel(const double2* __restrict__ H, const double2* __restrict__ Z,
                                                       double2* __restrict__ Y, int Q, int Qp, int B,
                                                       hz_modal::ModalArgs md) {
    constexpr int kBinGroups = kH / 256;
    if (md.on) {   // modal band states (hz_fb_modal.h): phase 1 and / or phase 2 as extra workgroups
        __shared__ ModalLds ml;
        const int i1 = (int)blockIdx.x - md.first1;
        if (md.n1l && i1 >= 0 && i1 < md.n1l) {
            if (i1 < md.n1) hz_modal::phase1_group(md, i1, ml.m1);
            else hz_modal::exc_partial(md, (i1 - md.n1) / md.exc_chunks, (i1 - md.n1) % md.exc_chunks, ml.m2);
            return;
        }
        const int i2 = (int)blockIdx.x - md.first2;
        if (md.n2 && i2 >= 0 && i2 < md.n2) {
            if (i2 < md.n2p) hz_modal::phase2_group(md, i2, ml.m2);
            else hz_modal::exc_sum(md);
            return;
        }
    }
    const int q = (blockIdx.x % kBinGroups) * blockDim.x + threadIdx.x;   // bin
    const int b0 = (blockIdx.x / kBinGroups) * R;
    HZ_DIAG_AT(1, 0);
    double ar[R], ai[R], zr[R], zi[R];
    const long base = (long)b0 + Q - 1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        ar[r] = ai[r] = 0.0;
        const double2 z = Z[(base + r) * kH + q];
        zr[r] = z.x;
        zi[r] = z.y;
    }
    auto zrow = [&](int p) {   // Z row of step p + 1's new element; < 0 only past Q (zero H rows)
        const long zi_ = base - p - 1;
        return (zi_ > 0 ? zi_ : 0) * kH + q;
    };
    auto step = [&](int u, const double2& hc, const double2& zc) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int sl = ((r - u) % R + R) % R;
            ar[r] = fma(hc.x, zr[sl], ar[r]);
            ar[r] = fma(-hc.y, zi[sl], ar[r]);
            ai[r] = fma(hc.x, zi[sl], ai[r]);
            ai[r] = fma(hc.y, zr[sl], ai[r]);
        }
        // element 0 of step p + 1 = Z[base - p - 1] into the slot element R - 1 leaves
        const int sl = ((-(u + 1)) % R + R) % R;
        zr[sl] = zc.x;
        zi[sl] = zc.y;
    };
    if constexpr (QP > 0) {
        double2 hv[QP], zv[QP];
#pragma unroll
        for (int p = 0; p < QP; ++p) {
            hv[p] = H[(long)p * kH + q];
            zv[p] = Z[zrow(p)];
        }
#ifdef HZ_DIAG_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        HZ_DIAG_AT(1, 1);
#endif
#pragma unroll
        for (int p = 0; p < QP; ++p) step(p % R, hv[p], zv[p]);
        HZ_DIAG_AT(1, 2);
    } else {
        double2 hb[R], zb[R];
        auto fetch = [&](int p0) {
#pragma unroll
            for (int u = 0; u < R; ++u) {
                hb[u] = H[(long)(p0 + u) * kH + q];
                zb[u] = Z[zrow(p0 + u)];
            }
        };
        fetch(0);
        for (int p0 = 0; p0 < Qp; p0 += R) {
            double2 hc[R], zc[R];
#pragma unroll
            for (int u = 0; u < R; ++u) {
                hc[u] = hb[u];
                zc[u] = zb[u];
            }
            if (p0 + R < Qp) fetch(p0 + R);
#pragma unroll
            for (int u = 0; u < R; ++u) step(u, hc[u], zc[u]);
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (b0 + r < B) Y[(long)(b0 + r) * kH + q] = make_double2(ar[r], ai[r]);
    HZ_DIAG_AT(1, 3);
}

// The MAC with its operands staged in LDS: a workgroup owns 64 bins x 32 output blocks (a wave per
// 8 blocks), loads the QP partition spectra and the 32 + QP - 1 window-spectrum rows those blocks
// read once (80 KB at QP = 24), and each thread runs resp_mac_kernel's register ring (the same
// FMAs in the same order, so the same bits) from LDS.  The register-only kernel loads every H row
// once per 8 blocks and every Z row about four times: 55 MB through the L2s per C2 call, which its
// operand phase waits 3.4 us for (stamps, profiles/r5/diag); here 20 MB.
constexpr int kMacBins = 64;
// BPW output blocks per wave, 4 waves: 4 BPW blocks per workgroup
template <int QP, int BPW>
constexpr size_t mac_lds_bytes() { return sizeof(double2) * kMacBins * (QP + 4 * BPW + QP - 1); }

template <int QP, int BPW>
__global__ __launch_bounds__(256) void resp_mac_kernel_lds(const double2* __restrict__ H, const double2* __restrict__ Z,
                                                           double2* __restrict__ Y, int Q, int B) {
    constexpr int kMacBlk = 4 * BPW, kZr = kMacBlk + QP - 1, kHL = QP / 4, kZL = (kZr + 3) / 4;
    extern __shared__ double2 mac_lds[];
    double2(*hs)[kMacBins] = (double2(*)[kMacBins])mac_lds;
    double2(*zs)[kMacBins] = (double2(*)[kMacBins])(mac_lds + QP * kMacBins);
    const int t = threadIdx.x, lq = t & (kMacBins - 1), sl = t >> 6;
    const int q = (blockIdx.x % (kH / kMacBins)) * kMacBins + lq;
    const int b0 = (blockIdx.x / (kH / kMacBins)) * kMacBlk;
    // Z row of block b, partition p: b + Q - 1 - p = row_lo + (b - b0) + QP - 1 - p; rows < 0 only
    // for p >= Q (zero H rows), read as row 0
    const long row_lo = (long)b0 + Q - QP;
    double2 hv[kHL], zv[kZL];
#pragma unroll
    for (int k = 0; k < kHL; ++k) hv[k] = H[(long)(sl + 4 * k) * kH + q];
#pragma unroll
    for (int k = 0; k < kZL; ++k) {
        const int r = sl + 4 * k;
        const long row = row_lo + r;
        zv[k] = r < kZr ? Z[(row > 0 ? row : 0) * kH + q] : make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int k = 0; k < kHL; ++k) hs[sl + 4 * k][lq] = hv[k];
#pragma unroll
    for (int k = 0; k < kZL; ++k)
        if (sl + 4 * k < kZr) zs[sl + 4 * k][lq] = zv[k];
    __syncthreads();
    double ar[BPW], ai[BPW], zr[BPW], zi[BPW];
#pragma unroll
    for (int r = 0; r < BPW; ++r) {
        ar[r] = ai[r] = 0.0;
        const double2 z = zs[BPW * sl + r + QP - 1][lq];
        zr[r] = z.x;
        zi[r] = z.y;
    }
#pragma unroll
    for (int p = 0; p < QP; ++p) {
        const double2 hc = hs[p][lq];
#pragma unroll
        for (int r = 0; r < BPW; ++r) {   // resp_mac_kernel's step: the same FMA order
            ar[r] = fma(hc.x, zr[r], ar[r]);
            ar[r] = fma(-hc.y, zi[r], ar[r]);
            ai[r] = fma(hc.x, zi[r], ai[r]);
            ai[r] = fma(hc.y, zr[r], ai[r]);
        }
        if (p + 1 < QP) {   // step p + 1 reads step p's rows one block down, and one new row
#pragma unroll
            for (int r = BPW - 1; r > 0; --r) {
                zr[r] = zr[r - 1];
                zi[r] = zi[r - 1];
            }
            const double2 z = zs[BPW * sl + QP - 2 - p][lq];
            zr[0] = z.x;
            zi[0] = z.y;
        }
    }
#pragma unroll
    for (int r = 0; r < BPW; ++r) {
        const int b = b0 + BPW * sl + r;
        if (b < B) Y[(long)b * kH + q] = make_double2(ar[r], ai[r]);
    }
}

// The LDS-staged MAC for long horizons (Qp > 24 partitions, e.g. R = 0.9999: K = 507,904, Q = 248):
// the partitions in chunks of 24 -- per chunk the 24 H rows and the 24 + 31 Z rows of the
// workgroup's 32 blocks go through LDS as in resp_mac_kernel_lds<24> (the next chunk's operands
// loaded into registers while this chunk's MACs run), the accumulators carried across chunks.  The
// partitions are visited in order with the same FMAs, so the result is the register kernel's bit
// for bit.  The register kernel it replaces pulled every H row once per 8 blocks and every Z row
// ~4 times through the L2s: ~0.5 GB per R = 0.9999 call.
constexpr int kMacChunk = 24;
// BINS bins x (256 / BINS) slices of BPW blocks per workgroup: 64 x 4 x 8 = 32 blocks (the C2
// kernel's tile), 32 x 8 x 8 = 64 or 16 x 16 x 8 = 128 blocks (the default: the H rows re-read by
// 2 instead of 8 block rows, the Z rows re-read less per block; HZ_MACC_BINS=32 / 64 for A/B)
template <int BINS, int BPW>
constexpr size_t macc_lds_bytes() { return sizeof(double2) * BINS * (kMacChunk + (256 / BINS) * BPW + kMacChunk - 1); }
template <int BINS, int BPW>
__global__ __launch_bounds__(256) void resp_mac_kernel_ldsc(const double2* __restrict__ H, const double2* __restrict__ Z,
                                                            double2* __restrict__ Y, int Q, int B, int nch, int cps,
                                                            long ystride) {
    constexpr int QP = kMacChunk, SL = 256 / BINS, kMacBlk = SL * BPW, kZr = kMacBlk + QP - 1;
    constexpr int kHL = (QP + SL - 1) / SL, kZL = (kZr + SL - 1) / SL;
    extern __shared__ double2 mac_lds[];
    double2(*hs)[BINS] = (double2(*)[BINS])mac_lds;
    double2(*zs)[BINS] = (double2(*)[BINS])(mac_lds + QP * BINS);
    const int t = threadIdx.x, lq = t & (BINS - 1), sl = t / BINS;
    const int q = (blockIdx.x % (kH / BINS)) * BINS + lq;
    const int b0 = (blockIdx.x / (kH / BINS)) * kMacBlk;
    double2 hv[kHL], zv[kZL];
    auto fetch = [&](int c) {   // chunk c: partitions [24 c, 24 c + 24)
#pragma unroll
        for (int k = 0; k < kHL; ++k)
            hv[k] = sl + SL * k < QP ? H[(long)(QP * c + sl + SL * k) * kH + q] : make_double2(0.0, 0.0);
        const long row_lo = (long)b0 + Q - (long)QP * (c + 1);
#pragma unroll
        for (int k = 0; k < kZL; ++k) {
            const int r = sl + SL * k;
            const long row = row_lo + r;
            zv[k] = r < kZr ? Z[(row > 0 ? row : 0) * kH + q] : make_double2(0.0, 0.0);
        }
    };
    double ar[BPW], ai[BPW];
#pragma unroll
    for (int r = 0; r < BPW; ++r) ar[r] = ai[r] = 0.0;
    // split blockIdx.y: chunks [c0, c1) into its own partial-sum plane of Y
    const int c0 = blockIdx.y * cps, c1 = min(nch, c0 + cps);
    Y += blockIdx.y * ystride;
    if (c0 < c1) fetch(c0);
    for (int c = c0; c < c1; ++c) {
#pragma unroll
        for (int k = 0; k < kHL; ++k)
            if (sl + SL * k < QP) hs[sl + SL * k][lq] = hv[k];
#pragma unroll
        for (int k = 0; k < kZL; ++k)
            if (sl + SL * k < kZr) zs[sl + SL * k][lq] = zv[k];
        __syncthreads();
        if (c + 1 < c1) fetch(c + 1);   // in flight under this chunk's MACs
        double zr[BPW], zi[BPW];
#pragma unroll
        for (int r = 0; r < BPW; ++r) {
            const double2 z = zs[BPW * sl + r + QP - 1][lq];
            zr[r] = z.x;
            zi[r] = z.y;
        }
#pragma unroll
        for (int p = 0; p < QP; ++p) {
            const double2 hc = hs[p][lq];
#pragma unroll
            for (int r = 0; r < BPW; ++r) {
                ar[r] = fma(hc.x, zr[r], ar[r]);
                ar[r] = fma(-hc.y, zi[r], ar[r]);
                ai[r] = fma(hc.x, zi[r], ai[r]);
                ai[r] = fma(hc.y, zr[r], ai[r]);
            }
            if (p + 1 < QP) {
#pragma unroll
                for (int r = BPW - 1; r > 0; --r) {
                    zr[r] = zr[r - 1];
                    zi[r] = zi[r - 1];
                }
                const double2 z = zs[BPW * sl + QP - 2 - p][lq];
                zr[0] = z.x;
                zi[0] = z.y;
            }
        }
        __syncthreads();   // the next chunk's stores overwrite hs / zs
    }
#pragma unroll
    for (int r = 0; r < BPW; ++r) {
        const int b = b0 + BPW * sl + r;
        if (b < B) Y[(long)b * kH + q] = make_double2(ar[r], ai[r]);
    }
}
template <int BINS, int BPW>
void launch_macc_t(int Qp, int B, const double2* H, const double2* Z, double2* Y, int Q, int ns, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)resp_mac_kernel_ldsc<BINS, BPW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)macc_lds_bytes<BINS, BPW>());
        attr = true;
    }
    constexpr int blk = (256 / BINS) * BPW;
    const int nch = Qp / kMacChunk, cps = (nch + ns - 1) / ns;
    const dim3 grid((unsigned)((kH / BINS) * ((B + blk - 1) / blk)), (unsigned)ns);
    hipLaunchKernelGGL((resp_mac_kernel_ldsc<BINS, BPW>), grid, dim3(256), (macc_lds_bytes<BINS, BPW>()), s, H, Z, Y, Q, B,
                       nch, cps, (long)B * kH);
}
// The long-horizon MAC is latency-bound per chunk (each chunk's operands are fetched one chunk ahead,
// and a 10 s call gives (kH / BINS) x ceil(B / blk) = 128 workgroups whatever the tile: twice as many,
// 4 blocks per thread, measured the same 35 us), so the chunks are split over `ns` workgroup planes
// whose partial sums the inverse launch adds (HZ_MACC_SPLIT = 1 for the unsplit kernel, A/B).  The
// gain is small (the MAC at 4 planes: 32.5 us), so chunk latency is not what bounds it either
int macc_splits(int Qp) {
    static const int env = std::getenv("HZ_MACC_SPLIT") ? std::atoi(std::getenv("HZ_MACC_SPLIT")) : 0;
    const int nch = Qp / kMacChunk;
    const int ns = env > 0 ? env : 2;   // R = 0.9999, alternating: 1: 0.0645 / 0.0644, 2: 0.0632 / 0.0628, 4: 0.0640 /
                                         // 0.0639 ms per call (MAC 35.0 -> 32.5 us, the inverse's sums +1 us)
    return std::max(1, std::min(ns, nch));
}
template <int BINS>
void launch_macc(int Qp, int B, const double2* H, const double2* Z, double2* Y, int Q, int ns, hipStream_t s) {
    static const int bpw = std::getenv("HZ_MACC_BPW") ? std::atoi(std::getenv("HZ_MACC_BPW")) : 8;
    if (bpw == 4) launch_macc_t<BINS, 4>(Qp, B, H, Z, Y, Q, ns, s);
    else launch_macc_t<BINS, 8>(Qp, B, H, Z, Y, Q, ns, s);
}

// the LDS-staged MAC for Qp = 8, 16, 24 when no modal phase rides in the MAC launch (C2: 6.1
// against 7.4 us per launch, step 29.4 against 30.6 us, alternating runs on one box,
// profiles/r5/mac/summary.txt); HZ_MAC=reg selects the register-only kernel (A/B)
bool mac_lds_ok(int Qp, bool modal_in_mac) {
    static const bool reg = [] {
        const char* v = std::getenv("HZ_MAC");
        return v && std::strcmp(v, "reg") == 0;
    }();
    return !reg && !modal_in_mac && (Qp == 8 || Qp == 16 || Qp == 24 || Qp % kMacChunk == 0);
}
template <int BPW>
void launch_mac_lds_t(int Qp, int B, const double2* H, const double2* Z, double2* Y, int Q, hipStream_t s) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)resp_mac_kernel_lds<8, BPW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mac_lds_bytes<8, BPW>());
        (void)hipFuncSetAttribute((const void*)resp_mac_kernel_lds<16, BPW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mac_lds_bytes<16, BPW>());
        (void)hipFuncSetAttribute((const void*)resp_mac_kernel_lds<24, BPW>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)mac_lds_bytes<24, BPW>());
        attr = true;
    }
    const dim3 grid((unsigned)((kH / kMacBins) * ((B + 4 * BPW - 1) / (4 * BPW))));
    if (Qp > kMacChunk) {   // long horizons: partitions in chunks of 24
        // 16 bins x 128 blocks: 35.5 us per R = 0.9999 call against 37.4 (32 x 64) and 46.2 (64 x 32),
        // alternating on one box (profiles/r6/highq)
        static const int bins = std::getenv("HZ_MACC_BINS") ? std::atoi(std::getenv("HZ_MACC_BINS")) : 16;
        const int ns = macc_splits(Qp);
        if (bins == 64) launch_macc<64>(Qp, B, H, Z, Y, Q, ns, s);
        else if (bins == 16) launch_macc<16>(Qp, B, H, Z, Y, Q, ns, s);
        else launch_macc<32>(Qp, B, H, Z, Y, Q, ns, s);
        return;
    }
    if (Qp == 8) hipLaunchKernelGGL((resp_mac_kernel_lds<8, BPW>), grid, dim3(256), (mac_lds_bytes<8, BPW>()), s, H, Z, Y, Q, B);
    else if (Qp == 16) hipLaunchKernelGGL((resp_mac_kernel_lds<16, BPW>), grid, dim3(256), (mac_lds_bytes<16, BPW>()), s, H, Z, Y, Q, B);
    else hipLaunchKernelGGL((resp_mac_kernel_lds<24, BPW>), grid, dim3(256), (mac_lds_bytes<24, BPW>()), s, H, Z, Y, Q, B);
}
// HZ_MAC_BPW=4: 4 blocks per wave (16 per workgroup, twice the workgroups) -- A/B; measured
// slower: 8.25 against 6.07 us per C2 launch (profiles/r5/bpw/summary.txt)
void launch_mac_lds(int Qp, int B, const double2* H, const double2* Z, double2* Y, int Q, hipStream_t s) {
    static const int bpw = std::getenv("HZ_MAC_BPW") && std::atoi(std::getenv("HZ_MAC_BPW")) == 4 ? 4 : 8;
    if (bpw == 4) launch_mac_lds_t<4>(Qp, B, H, Z, Y, Q, s);
    else launch_mac_lds_t<8>(Qp, B, H, Z, Y, Q, s);
}

typedef void (*MacKernel)(const double2*, const double2*, double2*, int, int, int, hz_modal::ModalArgs);
MacKernel pick_mac(int Qp) {
    switch (Qp) {
    case 8: return resp_mac_kernel<kMacR, 8>;
    case 16: return resp_mac_kernel<kMacR, 16>;
    case 24: return resp_mac_kernel<kMacR, 24>;
    default: return resp_mac_kernel<kMacR, 0>;
    }
}
typedef void (*RespKernel)(RespArgs, hz_state::StateArgs, hz_modal::ModalArgs);

// history after the call, smoothers' closed form, x history; a time-range shard's zeros outside
// its range (threads of the B output-block workgroups).  A thread's first element of each is
// loaded with the transform's operands (UpkeepPre) and stored after the transform, so the tail of
// the launch waits on no load (stamps: the store phase was 1.3 us with the loads issued there)
struct UpkeepPre {
    double h = 0.0, p0 = 0.0, g0 = 0.0, pb = 0.0, gb = 0.0, xh = 0.0;
};
__device__ __forceinline__ UpkeepPre resp_upkeep_pre(const RespArgs& a, long b) {
    UpkeepPre u;
    const long g = b * blockDim.x + threadIdx.x;
    if (g < a.K) {
        const long m = a.n + g;
        u.h = m < a.K ? a.hist[m] : a.x[m - a.K];
    }
    if (g < a.N) {
        u.p0 = a.pg[2 * g];
        u.g0 = a.pg[2 * g + 1];
        u.pb = a.pin[g];
        u.gb = a.gin[g];
    }
    if (g < a.O) u.xh = a.x[a.n - 1 - g];
    return u;
}
__device__ __forceinline__ void resp_upkeep(const RespArgs& a, long b, const UpkeepPre& u) {
    const int t = threadIdx.x;
    const long g = b * blockDim.x + t, stride = (long)a.B * blockDim.x;
    // a time-range shard leaves zeros outside its range (the ranks' outputs sum to the call's), or
    // nothing there (disjoint shares)
    if (a.zero_outside)
        for (long i = g; i < a.n - a.n_out; i += stride) a.out[i < a.off ? i : i + a.n_out] = 0.0;
    if (g < a.K) a.hist_next[g] = u.h;
    for (long i = g + stride; i < a.K; i += stride) {
        const long m = a.n + i;
        a.hist_next[i] = m < a.K ? a.hist[m] : a.x[m - a.K];
    }
    if (g < a.N) {
        a.pg_next[2 * g] = u.pb + a.sp_n * (u.p0 - u.pb);
        a.pg_next[2 * g + 1] = u.gb + a.sg_n * (u.g0 - u.gb);
    }
    for (long n = g + stride; n < a.N; n += stride) {
        const double P0 = a.pg[2 * n], G0 = a.pg[2 * n + 1], pb = a.pin[n], gb = a.gin[n];
        a.pg_next[2 * n] = pb + a.sp_n * (P0 - pb);
        a.pg_next[2 * n + 1] = gb + a.sg_n * (G0 - gb);
    }
    if (g < a.O) a.xhist_next[g] = u.xh;
}

// output block b: the merge of Y_b into Zh' = E' + i O' (E' = Y[k] + conj Y[kH-k],
// O' = (Y[k] - conj Y[kH-k]) W^-k; Zh'[kH-k] = conj E' + i conj O'), the inverse 2048-point FFT,
// out[bP + 2r (+1)] = Re (Im) z[kH/2 + r] (the last P samples of the window's circular
// convolution) straight from the last pass's registers
template <int SO>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void resp_inv_kernel(
    RespArgs a, hz_state::StateArgs st, hz_modal::ModalArgs md) {
    __shared__ RespLds u;
    if constexpr (SO == 0) {   // modal band states, phase 2 (hz_fb_modal.h): workgroups [first2, first2 + n2)
        const int i = (int)blockIdx.x - md.first2;
        if (md.on && i >= 0 && i < md.n2) {
            HZ_DIAG_AT(2, 0);
            if (i < md.n2p) hz_modal::phase2_group(md, i, u.md);
            else hz_modal::exc_sum(md);
            HZ_DIAG_AT(2, 1);
            HZ_DIAG_AT(2, 2);
            HZ_DIAG_AT(2, 3);
            return;
        }
    }
    if constexpr (SO > 0) {
        if ((int)blockIdx.x >= a.B) {
            const int i = blockIdx.x - a.B;
            hz_state::state_group<SO>(st, i % st.G, i / st.G, u.st);
            return;
        }
    }
    hz2k::Lds& s = u.fft;
    const int t = threadIdx.x;
    const long b = (long)blockIdx.x - ((SO == 0 && md.on && md.first2 == 0) ? md.n2 : 0);
    if (SO == 0) HZ_DIAG_AT(2, 0);
#ifdef HZ_DIAG_STAMPS
    long long* stp = SO > 0 && st.stamps ? st.stamps + ((long)st.G * st.nseg + b) * 4 : nullptr;
    if (stp && t == 0) {
        stp[0] = __builtin_amdgcn_s_memrealtime();
        stp[3] = ((long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) | __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
#endif
    const double2* y = a.Y + b * kH;
    double2 ya[4], yb[4], w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = t + i * kThreads;
        ya[i] = y[k];
        yb[i] = y[(kH - k) & (kH - 1)];   // k = 0: replaced by (Y_kH, 0) below
        w[i] = a.tw[k];
    }
    double2 ym = y[kH / 2];
    for (int sp = 1; sp < a.ys; ++sp) {   // the split MAC's partial sums, in split order
        const double2* ys = y + sp * a.ystride;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int k = t + i * kThreads;
            const double2 u = ys[k], v = ys[(kH - k) & (kH - 1)];
            ya[i] = make_double2(ya[i].x + u.x, ya[i].y + u.y);
            yb[i] = make_double2(yb[i].x + v.x, yb[i].y + v.y);
        }
        const double2 um = ys[kH / 2];
        ym = make_double2(ym.x + um.x, ym.y + um.y);
    }
    hz2k::InvTw it;
    it.load(a.tw);
    const UpkeepPre up = a.upkeep ? resp_upkeep_pre(a, b) : UpkeepPre();
    // bin kH (real): sum_p Hn[p] Zn[b + Q - 1 - p], wave 0 in a fixed order
    double yn = 0.0;
    if (t < 64) {
        for (int p = t; p < a.Q; p += 64) yn = fma(a.Hn[p], a.Zn[b + a.Q - 1 - p], yn);
#pragma unroll
        for (int o = 32; o; o >>= 1) yn += __shfl_xor(yn, o);
    }
    if (t == 0) yb[0] = make_double2(yn, 0.0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = t + i * kThreads, kb = (kH - k) & (kH - 1);
        const double er = ya[i].x + yb[i].x, ei = ya[i].y - yb[i].y;
        const double dr = ya[i].x - yb[i].x, di = ya[i].y + yb[i].y;
        const double orr = dr * w[i].x + di * w[i].y, oi = di * w[i].x - dr * w[i].y;
        s.z[hz2k::ix(hz::bitrev(k, kLgH))] = make_double2(er - oi, ei + orr);
        if (k) s.z[hz2k::ix(hz::bitrev(kb, kLgH))] = make_double2(er + oi, orr - ei);
    }
    if (t == 0) {   // Zh'[kH/2] = 2 conj Y[kH/2] (bit-reversed position 1)
        s.z[hz2k::ix(1)] = make_double2(2.0 * ym.x, -2.0 * ym.y);
    }
    double vr[kPT], vi[kPT];
    if (SO == 0) HZ_DIAG_AT(2, 1);
    hz2k::inv(s, vr, vi, it);
    if (SO == 0) HZ_DIAG_AT(2, 2);
    // z[kH/2 + r], r = t + 256 (i - 4): output samples bP + 2r, bP + 2r + 1 (one 16-byte store
    // when the output is 16-byte aligned)
    const bool oal = (reinterpret_cast<uintptr_t>(a.out + a.off) & 15) == 0;
#pragma unroll
    for (int i = kPT / 2; i < kPT; ++i) {
        const long t0 = b * kP + 2 * (t + (long)(i - kPT / 2) * kThreads);
        if (oal && t0 + 1 < a.n_out) {
            *reinterpret_cast<double2*>(a.out + a.off + t0) = make_double2(vr[i], vi[i]);
        } else {
            if (t0 < a.n_out) a.out[a.off + t0] = vr[i];
            if (t0 + 1 < a.n_out) a.out[a.off + t0 + 1] = vi[i];
        }
    }
    if (a.upkeep) resp_upkeep(a, b, up);
    if (SO == 0) HZ_DIAG_AT(2, 3);
#ifdef HZ_DIAG_STAMPS
    if (stp && t == 0) stp[1] = stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
}

// column-split path: the inverse columns of the range's blocks (hz_fb_col.h).  (The band-state
// pass stays in the combine kernel: this kernel's 136 KB of LDS would leave no room beside it.)
template <int QP>
__global__ __launch_bounds__(hz_col::kColThreads) void resp_col_kernel(hz_col::ColArgs a) {
    __shared__ hz_col::ColLds<QP> u;
    // ranges of the same unit index spread over the XCDs, all units of a range on one XCD (NR a
    // multiple of 8): a range's samples are read into one L2
    hz_col::col_group<QP>(a, (int)blockIdx.x / a.NR, (int)blockIdx.x % a.NR, u);
}

union CombLdsU {
    hz_col::CombLds c;
    hz_state::StateLds st;
};

// column-split path: one workgroup per output block (the combine + the upkeep), the band-state
// pass as extra workgroups past them (SO = the bank's order, 0: none)
template <int SO>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void resp_comb_kernel(
    RespArgs a, const double2* __restrict__ T, const unsigned char* __restrict__ cmap, const double2* __restrict__ tw4k,
    hz_state::StateArgs st) {
    __shared__ CombLdsU u;
    if constexpr (SO > 0) {
        if ((int)blockIdx.x >= a.B) {
            const int i = blockIdx.x - a.B;
            hz_state::state_group<SO>(st, i % st.G, i / st.G, u.st);
            return;
        }
    }
    const long b = blockIdx.x;
    const UpkeepPre up = resp_upkeep_pre(a, b);
    hz_col::comb_block(T, cmap, tw4k, b, u.c, a.out + a.off, a.n_out);
    resp_upkeep(a, b, up);
}


// history after a call: the last K samples of [hist | x]
__global__ __launch_bounds__(256) void resp_hist_kernel(const double* __restrict__ hist, const double* __restrict__ x,
                                                        long K, long n, double* __restrict__ hist_next) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K) return;
    const long m = n + i;
    hist_next[i] = m < K ? hist[m] : x[m - K];
}

typedef void (*RespHKernel)(const double*, const double*, const double*, const double*, int, long, double*);
RespHKernel pick_h(int O) {
    switch (O) {
    case 1: return resp_h_kernel<1>;
    case 2: return resp_h_kernel<2>;
    case 3: return resp_h_kernel<3>;
    default: return resp_h_kernel<4>;
    }
}

int resp_alloc(double** p, size_t* cap, size_t need) {
    if (need <= *cap) return HZ_OK;
    if (*p) HZ_TRY_HIP(hipFree(*p));
    *p = nullptr;
    HZ_TRY_HIP(hipMalloc(p, need * sizeof(double)));
    *cap = need;
    return HZ_OK;
}

// partitions padded with zero spectra: to the MAC's register window (8), or to whole chunks of the
// chunked LDS MAC (24) past 24
int q_padded(int Q) { return Q > 24 ? (Q + 23) / 24 * 24 : (Q + kMacR - 1) / kMacR * kMacR; }

// partition counts the column-split kernel is built for (its LDS holds kWB + Q window rows of four
// columns: Q <= 24 is 136 KB)
bool col_q_ok(int Q) { return Q == 8 || Q == 16 || Q == 24; }
typedef void (*ColKernel)(hz_col::ColArgs);
ColKernel pick_col(int Q) {
    return Q == 8 ? resp_col_kernel<8> : Q == 16 ? resp_col_kernel<16> : resp_col_kernel<24>;
}

// per-bank setup: horizon, history buffers, twiddles
int resp_setup(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    if (R.K == -2) {
        // ||M^K|| < 2^-53: older inputs reach a band state below one unit in the last place of
        // it, and the bank response's tail below 2^-53 of its l1 norm; then a whole number of the
        // chunk-128 state kernel's 8192-sample tiles
        R.K = hz_fbi::fb_horizon(h, -53);
        if (R.K >= 0) R.K = std::max<long>(8192, (R.K + 8191) / 8192 * 8192);
        R.h_valid = false;
        R.run = 0;
    }
    if (R.K <= 0) return HZ_OK;
    const size_t nz = std::max<size_t>((size_t)h->N * h->order, hz_fbi::kMaxOrder);
    if (nz > R.zero_cap) {
        HZ_TRY(resp_alloc(&R.d_zero, &R.zero_cap, nz));
        HZ_TRY_HIP(hipMemset(R.d_zero, 0, sizeof(double) * nz));
    }
    HZ_TRY(resp_alloc(&R.d_hist[0], &R.hist_cap0, (size_t)R.K));
    HZ_TRY(resp_alloc(&R.d_hist[1], &R.hist_cap1, (size_t)R.K));
    if (!R.d_tw4k) {   // column path: W_4096^k, k < 4096, in long double; the combine's column map
        std::vector<double2> tw(kF);
        const long double pi = acosl(-1.0L);
        for (int k = 0; k < kF; ++k) {
            const long double ang = -2.0L * pi * k / kF;
            tw[k] = make_double2((double)cosl(ang), (double)sinl(ang));
        }
        HZ_TRY_HIP(hipMalloc((void**)&R.d_tw4k, sizeof(double2) * kF));
        HZ_TRY_HIP(hipMemcpy(R.d_tw4k, tw.data(), sizeof(double2) * kF, hipMemcpyHostToDevice));
        unsigned char cm[64];
        hz_col::col_map(cm);
        HZ_TRY_HIP(hipMalloc((void**)&R.d_cmap, sizeof(cm)));
        HZ_TRY_HIP(hipMemcpy(R.d_cmap, cm, sizeof(cm), hipMemcpyHostToDevice));
    }
    if (!R.d_tw) {   // W_F^k, k < kH, in long double
        std::vector<double2> tw(kH);
        const long double pi = acosl(-1.0L);
        for (int k = 0; k < kH; ++k) {
            const long double ang = -2.0L * pi * k / kF;
            tw[k] = make_double2((double)cosl(ang), (double)sinl(ang));
        }
        HZ_TRY_HIP(hipMalloc((void**)&R.d_tw, sizeof(double2) * tw.size()));
        HZ_TRY_HIP(hipMemcpy(R.d_tw, tw.data(), sizeof(double2) * tw.size(), hipMemcpyHostToDevice));
    }
    return HZ_OK;
}

// h and its partition spectra for the current coefficients / targets
int modal_prepare(hz_fb* h);

int resp_build_h(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    if (R.h_valid) return HZ_OK;
    const int O = h->order, N = h->N;
    const long K = R.K;
    const int G = (N + 63) / 64;
    const int Q = (int)(K / kP), Qp = q_padded(Q);   // zero spectra past Q (the MAC's unguarded blocks)
    HZ_TRY(resp_alloc(&R.d_coef, &R.coef_cap, (size_t)N * (2 * O + 1)));
    HZ_TRY_HIP(hipMemcpyAsync(R.d_coef, h->F.data(), sizeof(double) * N * (O + 1), hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipMemcpyAsync(R.d_coef + (size_t)N * (O + 1), h->B.data(), sizeof(double) * N * O,
                              hipMemcpyHostToDevice, h->stream));
    HZ_TRY(resp_alloc(&R.d_hpart, &R.hpart_cap, (size_t)G * K));
    HZ_TRY(resp_alloc(&R.d_h, &R.h_cap, (size_t)K));
    HZ_TRY(resp_alloc(&R.d_H, &R.H_cap, (size_t)Qp * (2 * kH + 1)));   // [Qp][kH] complex, then [Qp] bin kH
    HZ_TRY_HIP(hipMemsetAsync(R.d_H, 0, sizeof(double) * (size_t)Qp * (2 * kH + 1), h->stream));
    hipLaunchKernelGGL(pick_h(O), dim3(G), dim3(64), 0, h->stream, (const double*)R.d_coef,
                       (const double*)(R.d_coef + (size_t)N * (O + 1)), (const double*)h->d_pin,
                       (const double*)h->d_gin, N, K, R.d_hpart);
    HZ_TRY_HIP(hipGetLastError());
    hipLaunchKernelGGL(resp_hsum_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, h->stream,
                       (const double*)R.d_hpart, G, K, R.d_h);
    HZ_TRY_HIP(hipGetLastError());
    if (R.over_valid)   // the whole bank's response (time-range shards)
        HZ_TRY_HIP(hipMemcpyAsync(R.d_h, R.h_over.data(), sizeof(double) * K, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(resp_hspec_kernel, dim3((unsigned)Q), dim3(kThreads), 0, h->stream, (const double*)R.d_h, K,
                       (const double2*)R.d_tw, (double2*)R.d_H, R.d_H + (size_t)Qp * 2 * kH);
    HZ_TRY_HIP(hipGetLastError());
    if (col_q_ok(Q)) {   // the column path's partition spectra, lane order
        HZ_TRY(resp_alloc(&R.d_Hc, &R.Hc_cap, (size_t)hz_col::kSlots * Q * 64 * 2));
        hipLaunchKernelGGL(hz_col::resp_hcol_kernel, dim3(hz_col::kSlots, (unsigned)Q), dim3(64), 0, h->stream,
                           (const double2*)R.d_H, (const double*)(R.d_H + (size_t)Qp * 2 * kH), Q, (double2*)R.d_Hc);
        HZ_TRY_HIP(hipGetLastError());
    }
    HZ_TRY(hz_fbi::fb_state_prepare(h));   // the state pass's records and operands, for LAZY too
    HZ_TRY(modal_prepare(h));               // banks on one pole circle (hz_fb_modal.h)
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // pageable coefficient sources
    R.h_valid = true;
    ++R.h_gen;
    return HZ_OK;
}

// zero-start band states over the history's K samples -> ystate (the end state of the last
// stationary call: after it (EAGER) or when needed (LAZY))
int resp_states(hz_fb* h, double* ystate) {
    hz_fb::Resp& R = h->resp;
    return hz_fbi::fb_state_window(h, R.d_hist[R.hcur], R.K, ystate, h->stream);
}

// ---- modal band states (hz_fb_modal.h) -----------------------------------------------------
// Does the bank qualify, and its tables (with h, per coefficient / target change): order 2, every
// band's poles complex on one circle at angles on the 2 pi / 8192 grid up to |c| K <= 1e-6 (c =
// log(p / p_g), long double), at most kMaxExc bands with (nearly) coincident poles -- those get their
// long-double responses for the direct sums.
int modal_prepare(hz_fb* h) {
    using namespace hz_modal;
    hz_fb::Resp& R = h->resp;
    R.modal_ok = false;
    const long K = R.K;
    const int N = h->N;
    // (time-range shards qualify too: every rank has the whole call's input, so its own bands'
    // states over the call's last K inputs come out of the same fold and DFT)
    if (h->order != 2 || K < kL || K % kL != 0 || N <= 0) return HZ_OK;
    const long double pi = 3.141592653589793238462643383279502884L;
    std::vector<BandPar> par((size_t)N);
    std::vector<int> exc;
    std::vector<long> mm((size_t)N, -1);
    std::vector<long double> Rn((size_t)N), ph((size_t)N);
    long double Rg = -1;
    for (int n = 0; n < N; ++n) {
        const long double a1 = h->B[2 * (size_t)n], a2 = h->B[2 * (size_t)n + 1];
        const long double disc = a2 - a1 * a1 / 4;   // Im(p)^2
        const long double im = disc > 0 ? sqrtl(disc) : 0.0L;
        if (a2 <= 0 || im <= 1e-6L * sqrtl(a2)) {
            exc.push_back(n);
            continue;
        }
        Rn[n] = sqrtl(a2);
        ph[n] = atan2l(im, -a1 / 2);
        if (Rg < 0) Rg = Rn[n];
        const double pin = h->pin[n];
        BandPar& P = par[n];
        P.pr = (double)(-a1 / 2);
        P.pi = (double)im;
        P.inv_im = (double)(1.0L / im);
        P.b0 = pin * h->F[3 * (size_t)n];
        P.b1 = pin * h->F[3 * (size_t)n + 1];
        P.b2 = pin * h->F[3 * (size_t)n + 2];
    }
    if ((int)exc.size() > kMaxExc || Rg < 0) return HZ_OK;
    constexpr int kW2 = kPhase2;   // phase-2 bin groups: w = 4 k1 + k2 / 16 (k2 < 64: m < L / 2)
    std::vector<int> ints(kW2 + 1 + 2 * (size_t)N + kMaxExc, 0);
    std::vector<std::vector<std::pair<int, int>>> bucket(kW2);
    for (int n = 0; n < N; ++n) {
        if (Rn[n] == 0) continue;   // exceptional
        const long m = std::lround((double)(ph[n] * kL / (2 * pi)));
        if (m <= 0 || m >= kL / 2) return HZ_OK;
        const long double cr = logl(Rn[n] / Rg), ci = ph[n] - 2 * pi * m / kL;
        if (sqrtl(cr * cr + ci * ci) * K > 1e-6L) return HZ_OK;
        par[n].cr = (double)cr;
        par[n].ci = (double)ci;
        bucket[(m & 63) * kParts + (int)((m >> 6) / 16)].push_back({n, (int)(m >> 6)});
    }
    int at = 0;
    for (int w = 0; w < kW2; ++w) {
        ints[w] = at;
        for (auto& bk : bucket[w]) {
            ints[kW2 + 1 + 2 * at] = bk.first;
            ints[kW2 + 1 + 2 * at + 1] = bk.second;
            ++at;
        }
    }
    ints[kW2] = at;
    for (size_t e = 0; e < exc.size(); ++e) ints[kW2 + 1 + 2 * (size_t)N + e] = exc[e];
    // tables: R_g^r, R_g^(L s), e^(2 pi i q / L)
    const int S = (int)(K / kL);
    std::vector<double> tab((size_t)kL + S + 2 * (size_t)kL);
    for (int r = 0; r < kL; ++r) tab[r] = (double)powl(Rg, (long double)r);
    for (int q = 0; q < S; ++q) tab[kL + q] = (double)powl(Rg, (long double)kL * q);
    for (int q = 0; q < kL; ++q) {
        tab[kL + S + 2 * (size_t)q] = (double)cosl(2 * pi * q / kL);
        tab[kL + S + 2 * (size_t)q + 1] = (double)sinl(2 * pi * q / kL);
    }
    // exceptional bands: their zero-start responses r[tau], tau <= K (pin included), long double
    const int chunks = (int)((K + kExcChunk - 1) / kExcChunk);
    std::vector<double> er(exc.size() * (size_t)(K + 1));
    for (size_t e = 0; e < exc.size(); ++e) {
        const int n = exc[e];
        const long double f0 = h->F[3 * (size_t)n], f1 = h->F[3 * (size_t)n + 1], f2 = h->F[3 * (size_t)n + 2];
        const long double a1 = h->B[2 * (size_t)n], a2 = h->B[2 * (size_t)n + 1], pin = h->pin[n];
        long double y1 = 0, y2 = 0;
        for (long t = 0; t <= K; ++t) {
            const long double ff = t == 0 ? f0 : t == 1 ? f1 : t == 2 ? f2 : 0.0L;
            const long double y = pin * ff - (a1 * y1 + a2 * y2);
            y2 = y1;
            y1 = y;
            er[e * (size_t)(K + 1) + t] = (double)y;
        }
    }
    HZ_TRY(resp_alloc(&R.d_mpar, &R.mpar_cap, (size_t)N * sizeof(BandPar) / sizeof(double)));
    HZ_TRY(resp_alloc(&R.d_mtab, &R.mtab_cap, tab.size()));
    HZ_TRY(resp_alloc(&R.d_mA, &R.mA_cap, 2 * 2 * (size_t)kR2 * kR1));
    HZ_TRY(resp_alloc(&R.d_mexc, &R.mexc_cap, er.size() + exc.size() * (size_t)chunks * 4 + 1));
    if (ints.size() > R.mint_cap) {
        if (R.d_mint) HZ_TRY_HIP(hipFree(R.d_mint));
        R.d_mint = nullptr;
        HZ_TRY_HIP(hipMalloc(&R.d_mint, sizeof(int) * ints.size()));
        R.mint_cap = ints.size();
    }
    HZ_TRY_HIP(hipMemcpyAsync(R.d_mpar, par.data(), sizeof(BandPar) * N, hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipMemcpyAsync(R.d_mtab, tab.data(), sizeof(double) * tab.size(), hipMemcpyHostToDevice, h->stream));
    if (!er.empty())
        HZ_TRY_HIP(hipMemcpyAsync(R.d_mexc, er.data(), sizeof(double) * er.size(), hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipMemcpyAsync(R.d_mint, ints.data(), sizeof(int) * ints.size(), hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // the host tables above are locals
    R.mexc_n = (int)exc.size();
    R.mexc_chunks = chunks;
    R.mS = S;
    R.modal_ok = true;
    return HZ_OK;
}

// the window of the call's last K inputs: [history n.. | call] for calls n < K, else the call's tail
void modal_args(hz_fb* h, const double* hist, const double* x, long n, double* out, hz_modal::ModalArgs* a) {
    using namespace hz_modal;
    hz_fb::Resp& R = h->resp;
    const long K = R.K;
    *a = ModalArgs();
    a->on = 1;
    if (n >= K) {
        a->xw = x + (n - K);
        a->xw2 = x + (n - K);
        a->split = 0;
    } else {
        a->xw = hist + n;
        a->xw2 = x;
        a->split = K - n;
    }
    a->K = K;
    a->S = R.mS;
    a->wR = R.d_mtab;
    a->RL = R.d_mtab + kL;
    a->tw = (const double2*)(R.d_mtab + kL + R.mS);
    a->A = (double2*)R.d_mA;
    a->par = (const BandPar*)R.d_mpar;
    a->csr_ptr = R.d_mint;
    a->csr = (const int2*)(R.d_mint + kPhase2 + 1);
    a->nexc = R.mexc_n;
    a->exc_band = R.d_mint + kPhase2 + 1 + 2 * (size_t)h->N;
    a->exc_r = R.d_mexc;
    a->exc_part = R.d_mexc + (size_t)R.mexc_n * (K + 1);
    a->exc_chunks = R.mexc_chunks;
    a->out = out;
    // (A/B) residues per phase-1 workgroup, columns per phase-2 workgroup
    static const int per1 = std::getenv("HZ_MODAL_R1PER") ? std::atoi(std::getenv("HZ_MODAL_R1PER")) : 1;
    static const int per2 = std::getenv("HZ_MODAL_K1PER") ? std::atoi(std::getenv("HZ_MODAL_K1PER")) : 1;
    a->per1 = (per1 > 0 && kR1 % per1 == 0) ? per1 : 1;
    a->per2 = (per2 > 0 && kPhase2 % per2 == 0) ? per2 : 1;
    a->n1 = kR1 / a->per1;
    a->n2p = kPhase2 / a->per2;
}

long resp_min_call(const hz_fb* h) { return h->resp.min_call > 0 ? h->resp.min_call : kMinCall; }

}  // namespace

namespace hz_fbi {

void fb_resp_init(hz_fb* h) { h->resp.mode = HZ_FB_RESP_EAGER; }

void fb_resp_invalidate(hz_fb* h, bool coefficients) {
    fb_stream_dclear(h);
    if (coefficients) h->resp.st.rband_valid = false;
    h->resp.run = 0;
    h->resp.h_valid = false;
    h->resp.over_valid = false;
    h->resp.armed = false;
    if (coefficients) h->resp.K = -2;
}

void fb_resp_setter(hz_fb* h) {
    if (h->resp.over_valid) h->resp.h_valid = false;   // back to this shard's own response
    h->resp.over_valid = false;
    h->resp.armed = false;
}

bool fb_resp_time_sharded(const hz_fb* h) { return h->resp.over_valid && h->resp.shard_world > 1; }

// the cost model alone: would a call of n samples run stationary (given the history)?
static bool resp_worth(const hz_fb* h, long n) {
    const hz_fb::Resp& R = h->resp;
    const long per = R.bands_per_sample >= 0 ? R.bands_per_sample : kBandsPerSample;
    // time-range shards cost the whole bank's convolution (the choice itself is armed by the
    // caller on every rank, hz_fb_arm_time_shard)
    const double bands = R.over_valid ? (double)h->N_total : (double)h->N;
    return bands * n >= (double)per * (double)(R.K + n);
}

bool fb_resp_eligible(hz_fb* h, long n, bool conv) {
    hz_fb::Resp& R = h->resp;
    if (R.mode == HZ_FB_RESP_OFF || !conv || h->order == 0 || h->dist_id != HZ_DIST_NONE ||
        h->path_mode != HZ_FB_PATH_AUTO || n < resp_min_call(h))
        return false;
    if (R.K == -2 && resp_setup(h) != HZ_OK) return false;
    if (R.K <= 0 || R.run < R.K) return false;
    // the bank engines cost ~N per sample, this one ~(K + n) / n (Q MACs + two FFT passes per
    // sample): measured crossover near 300 band-equivalents per sample of history + call
    return resp_worth(h, n);
}

int fb_resp_setup(hz_fb* h) { return resp_setup(h); }

int fb_resp_build(hz_fb* h) {
    HZ_TRY(resp_setup(h));
    return resp_build_h(h);
}

int fb_resp_materialize(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    if (!R.implicit) return HZ_OK;
    if (R.st.line_hist)   // streamed calls: the history is in the ring
        HZ_TRY(fb_stream_materialize(h));
    else
        HZ_TRY(resp_states(h, h->d_ystate[h->scur]));
    R.implicit = false;
    return HZ_OK;
}

// after a call on any engine: the history keeps the last K inputs while the bank stays converged
int fb_resp_track(hz_fb* h, const double* d_in, long n, bool conv) {
    hz_fb::Resp& R = h->resp;
    // short calls: 1024-sample blocks the streaming engine could take keep the history in its
    // ring (hz_fb_stream.hip); any other short call restarts the count
    if (n < resp_min_call(h)) return fb_stream_track(h, d_in, n, conv);
    // (handles pinned to the general engine never run stationary: no history upkeep; a
    // distortion functor keeps it, the engine resumes when the functor is cleared)
    if (R.mode == HZ_FB_RESP_OFF || !conv || h->order == 0 || h->path_mode != HZ_FB_PATH_AUTO) {
        R.run = 0;
        R.st.fdl_valid = false;
        fb_stream_dclear(h);
        return HZ_OK;
    }
    HZ_TRY(fb_stream_to_hist(h));   // after streamed calls
    if (R.K == -2) HZ_TRY(resp_setup(h));
    // no history for banks / call lengths the engine would not take (small banks keep their
    // per-band calls free of the upkeep launch)
    if (R.K <= 0 || !resp_worth(h, n)) {
        R.run = 0;
        return HZ_OK;
    }
    HZ_TRY(resp_setup(h));
    hipLaunchKernelGGL(resp_hist_kernel, dim3((unsigned)((R.K + 255) / 256)), dim3(256), 0, h->stream,
                       (const double*)R.d_hist[R.hcur], d_in, R.K, n, R.d_hist[R.hcur ^ 1]);
    HZ_TRY_HIP(hipGetLastError());
    R.hcur ^= 1;
    R.run = std::min(R.run + n, 1L << 60);
    return HZ_OK;
}

// a stationary call (fb_resp_eligible): output, history, end state
int fb_launch_resp(hz_fb* h, const double* d_in, double* d_out, long n) {
    hz_fb::Resp& R = h->resp;
    HZ_TRY(resp_setup(h));
    HZ_TRY(fb_stream_to_hist(h));   // after streamed calls: the history back in d_hist
    HZ_TRY(resp_build_h(h));
    const long K = R.K;
    const int Q = (int)(K / kP), Qp = q_padded(Q);
    // time-range shard (hz_fb_set_time_shard, with the whole bank's response): this rank's run of
    // whole output blocks
    long off = 0, n_out = n;
    if (R.shard_world > 1 && R.over_valid) {
        const long Ball = (n + kP - 1) / kP;
        const long lo = Ball * R.shard_rank / R.shard_world, hi = Ball * (R.shard_rank + 1) / R.shard_world;
        off = std::min(n, lo * kP);
        n_out = std::min(n, hi * kP) - off;
    }
    const int B = (int)std::max<long>(1, (n_out + kP - 1) / kP);
    const int nz = Q + B - 1;
    // rows the MAC may read: its last register window (B padded to kMacR output blocks, Qp
    // partitions); rows past nz are never stored, only multiplied into discarded outputs
    const int zrows = (B + 64 - 1) / 64 * 64 + Qp;
    if ((size_t)zrows * (2 * kH + 1) > R.Z_cap) {
        HZ_TRY(resp_alloc(&R.d_Z, &R.Z_cap, (size_t)zrows * (2 * kH + 1)));
        HZ_TRY_HIP(hipMemsetAsync(R.d_Z, 0, sizeof(double) * R.Z_cap, h->stream));
    }
    const size_t zn_at = (size_t)zrows * 2 * kH;   // [zrows] bin kH after the rows
    const int ys = (mac_lds_ok(Qp, false) && Qp > kMacChunk) ? macc_splits(Qp) : 1;   // (launch_mac_lds's split)
    HZ_TRY(resp_alloc(&R.d_Y, &R.Y_cap, (size_t)ys * B * kH * 2));
    hipEvent_t* e = nullptr;
    if (h->prof) {
        HZ_TRY(fb_prof_events(h, &e));
        HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        h->ev_skip[(e - h->ev.data()) / 5] |= 2;   // no segment phase
    }
    RespArgs a;
    a.hist = R.d_hist[R.hcur];
    a.x = d_in;
    a.K = K;
    a.n = n;
    a.off = off;
    a.n_out = n_out;
    a.Q = Q;
    a.B = B;
    a.tw = (const double2*)R.d_tw;
    a.Z = (double2*)R.d_Z;
    a.Zn = R.d_Z + zn_at;
    a.Y = (const double2*)R.d_Y;
    a.ys = ys;
    a.ystride = (long)B * kH;
    a.Hn = R.d_H + (size_t)Qp * 2 * kH;
    a.out = d_out;
    a.hist_next = R.d_hist[R.hcur ^ 1];
    a.pg = h->d_pg[h->scur];
    a.pg_next = h->d_pg[h->scur ^ 1];
    a.pin = h->d_pin;
    a.gin = h->d_gin;
    a.sp_n = (double)powl((long double)h->sp, (long double)n);
    a.sg_n = (double)powl((long double)h->sg, (long double)n);
    a.xhist_next = h->d_xhist[h->xcur ^ 1];
    a.N = h->N;
    a.O = h->order;
    a.nz = nz;
    a.upkeep = 1;
    a.zero_outside = R.shard_zero ? 1 : 0;
    // EAGER, n >= K: the band states after the call are the zero-start states over the call's last
    // K samples, independent of the convolution: the state pass runs as extra workgroups of the
    // inverse kernel (orders <= 2: 256 registers; prefetching its operands into the XCDs' L2 from the
    // MAC kernel was measured: no gain)
    const bool lazy = R.mode == HZ_FB_RESP_LAZY;
    const bool col = R.col_on && col_q_ok(Q);
    // banks on one pole circle: the modal states (hz_fb_modal.h) instead of the MFMA pass, phase 1
    // in the forward kernel, phase 2 in the inverse kernel
    // (calls shorter than K too: the window is the history's tail and the call, hz_fb_modal.h win())
    const bool modal = !lazy && n >= 3 && R.modal_on && R.modal_ok && !col;
    const bool chained = !lazy && n >= K && h->order <= 2 && !modal;
    const bool inside = chained || modal;   // the states come out of the transform kernels
    hz_state::StateArgs st = hz_state::StateArgs();
    if (chained) HZ_TRY(fb_state_chained(h, d_in + (n - K), K, h->d_ystate[h->scur ^ 1], &st));
    hz_modal::ModalArgs md = hz_modal::ModalArgs();
    if (modal) modal_args(h, R.d_hist[R.hcur], d_in, n, h->d_ystate[h->scur ^ 1], &md);
    const int so = chained ? h->order : 0;
    const int nmac = (kH / 256) * ((B + kMacR - 1) / kMacR);
    int dg_fx = 0, dg_ix = 0, dg_i0 = 0, dg_n1 = 0;   // (diagnostic stamps) modal workgroups per launch
    (void)dg_fx; (void)dg_ix; (void)dg_i0; (void)dg_n1;
    R.last_engine = col ? 1 : modal ? 2 : 0;
    R.modal_last = modal;
    if (col) {
        // column-split path (hz_fb_col.h): window spectra never leave the column kernel; the
        // combine kernel carries the band-state pass
        const int NR = (B + hz_col::kWB - 1) / hz_col::kWB;
        HZ_TRY(resp_alloc(&R.d_T, &R.T_cap, (size_t)B * hz_col::kSlots * 64 * 2));
        hz_col::ColArgs ca;
        ca.hist = a.hist;
        ca.x = a.x;
        ca.K = K;
        ca.off = off;
        ca.n_out = n_out;
        ca.Q = Q;
        ca.B = B;
        ca.NR = NR;
        ca.tw4k = (const double2*)R.d_tw4k;
        ca.Hc = (const double2*)R.d_Hc;
        ca.T = (double2*)R.d_T;
        hipLaunchKernelGGL(pick_col(Q), dim3((unsigned)(hz_col::kUnits * NR)), dim3(hz_col::kColThreads), 0, h->stream, ca);
        HZ_TRY_HIP(hipGetLastError());
        if (e && inside) {
            HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
            h->ev_skip[(e - h->ev.data()) / 5] |= 8;
        }
        auto kc = so == 1 ? resp_comb_kernel<1> : so == 2 ? resp_comb_kernel<2> : resp_comb_kernel<0>;
        hipLaunchKernelGGL(kc, dim3((unsigned)(B + (chained ? st.G * st.nseg : 0))), dim3(kThreads), 0, h->stream, a,
                           (const double2*)R.d_T, (const unsigned char*)R.d_cmap, (const double2*)R.d_tw4k, st);
        HZ_TRY_HIP(hipGetLastError());
    } else {
        // (HZ_MODAL_DIAG, timing diagnostics only -- wrong states: 1 no phase-1 / exceptional
        // workgroups, 2 no phase 2, 3 no exceptional partials)
        static const int diag = std::getenv("HZ_MODAL_DIAG") ? std::atoi(std::getenv("HZ_MODAL_DIAG")) : 0;
        const int nm1 = !modal || diag == 1 ? 0 : diag == 3 ? md.n1 : md.n1 + md.nexc * md.exc_chunks;
        // phase 1: extra workgroups of the forward kernel (HZ_MODAL_P1=mac: of the MAC kernel -- A/B)
        static const char* p1env = std::getenv("HZ_MODAL_P1");
        static const bool p1mac = p1env && std::string(p1env) == "mac";
        // profiling with hz_fb_profile(h, rep > 1): each (idempotent) kernel of the modal path launched rep
        // times between its events
        const int rep = e && modal ? h->prof_rep : 1;
        if (e) h->ev_rep[(e - h->ev.data()) / 5] = (unsigned char)rep;
        for (int r = 0; r < rep; ++r)
            hipLaunchKernelGGL(resp_fwd_kernel, dim3((unsigned)(nz + (p1mac ? 0 : nm1))), dim3(kThreads), 0,
                               h->stream, a, md);
        HZ_TRY_HIP(hipGetLastError());
        if (e && inside) {   // profiling: e0..e1 forward, e1..e2 MAC, e2..e4 inverse with the band states
            HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
            h->ev_skip[(e - h->ev.data()) / 5] &= (unsigned char)~2;
        }
        // phase 2: extra workgroups of the inverse kernel after its transforms (HZ_MODAL_P2 =
        // inv_first: before them; mac: beside the MAC -- A/B)
        static const char* p2env = std::getenv("HZ_MODAL_P2");
        static const int p2 = !p2env ? 1 : std::string(p2env) == "mac" ? 0 : std::string(p2env) == "inv_first" ? 2 : 1;
        const int nm2 = !modal || diag == 2 ? 0 : md.n2p + (md.nexc ? 1 : 0);
        hz_modal::ModalArgs mdm = md, mdi = md;
        mdm.on = modal && (p2 == 0 || p1mac);
        mdm.first2 = nmac;
        mdm.n2 = p2 == 0 ? nm2 : 0;
        mdm.first1 = nmac + mdm.n2;
        mdm.n1l = modal && p1mac ? nm1 : 0;
        mdi.on = modal && p2 != 0;
        mdi.first2 = p2 == 2 ? 0 : B;
        mdi.n2 = nm2;
        a.ys = (mac_lds_ok(Qp, mdm.on) && Qp > kMacChunk) ? macc_splits(Qp) : 1;   // launch_mac_lds's planes
        for (int r = 0; r < rep; ++r) {
            if (mac_lds_ok(Qp, mdm.on))
                launch_mac_lds(Qp, B, (const double2*)R.d_H, (const double2*)R.d_Z, (double2*)R.d_Y, Q, h->stream);
            else
                hipLaunchKernelGGL(pick_mac(Qp), dim3((unsigned)(nmac + (mdm.on ? mdm.n2 + mdm.n1l : 0))), dim3(256), 0,
                                   h->stream, (const double2*)R.d_H, (const double2*)R.d_Z, (double2*)R.d_Y, Q, Qp, B, mdm);
        }
        HZ_TRY_HIP(hipGetLastError());
        if (e && inside) {
            HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
            h->ev_skip[(e - h->ev.data()) / 5] |= 8;
        }
        dg_fx = p1mac ? 0 : nm1;
        dg_n1 = md.n1;
        dg_ix = mdi.on ? nm2 : 0;
        dg_i0 = mdi.first2;
        RespKernel ki = so == 1 ? resp_inv_kernel<1> : so == 2 ? resp_inv_kernel<2> : resp_inv_kernel<0>;
        for (int r = 0; r < rep; ++r)
            hipLaunchKernelGGL(ki, dim3((unsigned)(B + (chained ? st.G * st.nseg : 0) + (mdi.on ? nm2 : 0))),
                               dim3(kThreads), 0, h->stream, a, st, mdi);
        HZ_TRY_HIP(hipGetLastError());
    }
    if (chained) HZ_TRY(fb_state_combine(h, st, h->stream));   // pieces of a small bank
#ifdef HZ_DIAG_STAMPS
    if (col && R.calls == 30) {
        static long long cv[1024][5];
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        if (hipMemcpyFromSymbol(cv, HIP_SYMBOL(hz_col::g_cdiag), sizeof(cv)) == hipSuccess) {
            const int n = std::min(1024, hz_col::kUnits * ((B + hz_col::kWB - 1) / hz_col::kWB));
            long long t0 = cv[0][0];
            for (int i = 0; i < n; ++i) t0 = std::min(t0, cv[i][0]);
            double ph[4] = {0, 0, 0, 0}, smax = 0, emax = 0;
            int full = 0;
            for (int i = 0; i < n; ++i) {
                smax = std::max(smax, (cv[i][0] - t0) * 0.01);
                emax = std::max(emax, (cv[i][4] - t0) * 0.01);
                if (cv[i][4] > cv[i][0]) {
                    ++full;
                    for (int j = 0; j < 4; ++j) ph[j] += (cv[i][j + 1] - cv[i][j]) * 0.01;
                }
            }
            std::fprintf(stderr, "[col stamps] %d workgroups: mean stage1 %.2f us, stage3 %.2f us, MAC %.2f us, "
                         "inverse %.2f us; starts up to %.2f us, last end %.2f us\n", n, ph[0] / full, ph[1] / full,
                         ph[2] / full, ph[3] / full, smax, emax);
        }
    }
    if ((chained || modal) && R.calls == 30) {
        if (chained) fb_state_stamps_dump(st, B, R.calls);
        static long long hv[3][1024][4];
        if (hipMemcpyFromSymbol(hv, HIP_SYMBOL(g_diag), sizeof(hv)) == hipSuccess) {
            // workgroups [0, main) run the kernel's own part, the rest (up to 1024) the modal phases
            const int tot[3] = {std::min((int)nz + dg_fx, 1024), std::min(nmac, 1024), std::min((int)B + dg_ix, 1024)};
            for (int k = 0; k < 3; ++k) {
                long long t0 = hv[k][0][0];
                for (int i = 0; i < tot[k]; ++i) t0 = std::min(t0, hv[k][i][0]);
                double ph[3] = {0, 0, 0}, emain = 0, eextra = 0, smax = 0;
                int nmain = 0, nextra = 0;
                for (int i = 0; i < tot[k]; ++i) {
                    const bool extra = k == 0 ? i >= nz : k == 2 ? (dg_i0 == 0 ? i < dg_ix : i >= B) : false;
                    const double e = (hv[k][i][3] - t0) * 0.01;
                    smax = std::max(smax, (hv[k][i][0] - t0) * 0.01);
                    if (extra) {
                        ++nextra;
                        eextra = std::max(eextra, e);
                    } else {
                        ++nmain;
                        emain = std::max(emain, e);
                        for (int j = 0; j < 3; ++j) ph[j] += (hv[k][i][j + 1] - hv[k][i][j]) * 0.01;
                    }
                }
                if (k == 0 && dg_fx > dg_n1) {   // phase-1 residues vs the exceptional bands' partials
                    double e1 = 0, ex = 0;
                    for (int i = nz; i < tot[0]; ++i) {
                        const double e = (hv[0][i][3] - t0) * 0.01;
                        if (i < nz + dg_n1) e1 = std::max(e1, e);
                        else ex = std::max(ex, e);
                    }
                    std::fprintf(stderr, "[fwd stamps] phase-1 workgroups (%d) last end %.2f us, exceptional partials (%d) last end %.2f us\n",
                                 dg_n1, e1, dg_fx - dg_n1, ex);
                }
                std::fprintf(stderr, "[%s stamps] %d workgroups: mean operands %.2f us, compute %.2f us, stores %.2f us; "
                             "starts up to %.2f us, last end %.2f us; %d modal workgroups, last end %.2f us\n",
                             k == 0 ? "fwd" : k == 1 ? "mac" : "inv", nmain, ph[0] / std::max(nmain, 1),
                             ph[1] / std::max(nmain, 1), ph[2] / std::max(nmain, 1), smax, emain, nextra, eextra);
            }
        }
    }
#endif
    if (e && inside) HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
    if (e && !inside) HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
    R.hcur ^= 1;   // the inverse kernel wrote the history after the call
    R.run = std::min(R.run + n, 1L << 60);
    // end state: the band states over the new history (EAGER: computed inside the transform
    // kernels, or after them when n < K / order > 2) or when needed (LAZY); the smoothers and x
    // history were written by the inverse kernel (profiling events 3 / 4 bracket the state pass;
    // chained: the three kernels)
    if (lazy) {
        R.implicit = true;
        if (e) HZ_TRY_HIP(hipEventRecord(e[3], h->stream));
        if (e) HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
    } else if (inside) {
        R.implicit = false;
    } else {
        if (e) HZ_TRY_HIP(hipEventRecord(e[3], h->stream));
        HZ_TRY(resp_states(h, h->d_ystate[h->scur ^ 1]));
        if (e) HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
        R.implicit = false;
    }
    h->scur ^= 1;
    h->xcur ^= 1;
    h->prof_launches += h->prof ? 1 : 0;
    ++R.calls;
    fb_mirror_advance(h, n);
    return HZ_OK;
}

int fb_resp_tail_spectra(hz_fb* h, long K1) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    const long Kt = R.K - K1;
    const int Q = (int)(Kt / kP), Qp = q_padded(Q);
    HZ_TRY(resp_alloc(&S.d_tH, &S.tH_cap, (size_t)Qp * (2 * kH + 1)));
    HZ_TRY_HIP(hipMemsetAsync(S.d_tH, 0, sizeof(double) * (size_t)Qp * (2 * kH + 1), h->stream));
    hipLaunchKernelGGL(resp_hspec_kernel, dim3((unsigned)Q), dim3(kThreads), 0, h->stream, (const double*)(R.d_h + K1),
                       Kt, (const double2*)R.d_tw, (double2*)S.d_tH, S.d_tH + (size_t)Qp * 2 * kH);
    HZ_TRY_HIP(hipGetLastError());
    S.tQ = Q;
    return HZ_OK;
}

int fb_resp_tail_conv(hz_fb* h, const double* u, long n, double* out, hipStream_t st) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    const int Q = S.tQ, Qp = q_padded(Q);
    const long Kt = (long)Q * kP;
    const int B = (int)((n + kP - 1) / kP), nz = Q + B - 1;
    const int zrows = (B + 64 - 1) / 64 * 64 + Qp;
    if ((size_t)zrows * (2 * kH + 1) > S.tZ_cap) {
        HZ_TRY(resp_alloc(&S.d_tZ, &S.tZ_cap, (size_t)zrows * (2 * kH + 1)));
        HZ_TRY_HIP(hipMemsetAsync(S.d_tZ, 0, sizeof(double) * S.tZ_cap, st));
    }
    HZ_TRY(resp_alloc(&S.d_tY, &S.tY_cap, (size_t)B * kH * 2));
    RespArgs a{};
    a.hist = u;
    a.x = u + Kt;
    a.K = Kt;
    a.n = n;
    a.off = 0;
    a.n_out = n;
    a.Q = Q;
    a.B = B;
    a.nz = nz;
    a.tw = (const double2*)R.d_tw;
    a.Z = (double2*)S.d_tZ;
    a.Zn = S.d_tZ + (size_t)zrows * 2 * kH;
    a.Y = (const double2*)S.d_tY;
    a.ys = 1;
    a.Hn = S.d_tH + (size_t)Qp * 2 * kH;
    a.out = out;
    a.upkeep = 0;
    a.zero_outside = 0;
    hipLaunchKernelGGL(resp_fwd_kernel, dim3((unsigned)nz), dim3(kThreads), 0, st, a, hz_modal::ModalArgs());
    HZ_TRY_HIP(hipGetLastError());
    const int nmac = (kH / 256) * ((B + kMacR - 1) / kMacR);
    hipLaunchKernelGGL(pick_mac(Qp), dim3((unsigned)nmac), dim3(256), 0, st, (const double2*)S.d_tH,
                       (const double2*)S.d_tZ, (double2*)S.d_tY, Q, Qp, B, hz_modal::ModalArgs());
    HZ_TRY_HIP(hipGetLastError());
    hipLaunchKernelGGL(resp_inv_kernel<0>, dim3((unsigned)B), dim3(kThreads), 0, st, a, hz_state::StateArgs(),
                       hz_modal::ModalArgs());
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

void fb_resp_free(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    for (double* p : {R.d_hist[0], R.d_hist[1], R.d_h, R.d_hpart, R.d_coef, R.d_zero, R.d_H, R.d_Z, R.d_Y, R.d_tw,
                      R.d_spart, R.d_sop, R.d_tw4k, R.d_Hc, R.d_T, R.d_mpar, R.d_mtab, R.d_mA, R.d_mexc})
        if (p) (void)hipFree(p);
    if (R.d_cmap) (void)hipFree(R.d_cmap);
    if (R.d_scount) (void)hipFree(R.d_scount);
    if (R.d_mint) (void)hipFree(R.d_mint);
    fb_stream_free(h);
    const bool col_on = R.col_on, modal_on = R.modal_on;
    R = hz_fb::Resp();
    R.col_on = col_on;
    R.modal_on = modal_on;
}

}  // namespace hz_fbi

extern "C" {

int hz_fb_set_response(hz_fb* h, int mode) {
    if (!h || mode < HZ_FB_RESP_OFF || mode > HZ_FB_RESP_LAZY) {
        hz::set_error("hz_fb_set_response: mode must be HZ_FB_RESP_OFF, _EAGER or _LAZY");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    HZ_TRY(hz_fbi::fb_resp_materialize(h));
    h->resp.mode = mode;
    h->resp.armed = false;   // a time-sharded handle re-arms (on every rank) for the new mode
    if (mode == HZ_FB_RESP_OFF) h->resp.run = 0;
    return HZ_OK;
}

int hz_fb_set_bank_response(hz_fb* h, const double* resp, long count) {
    if (!h || (count > 0 && !resp) || count < 0) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->device));
    HZ_TRY(hz_fbi::fb_upload_staged(h));
    if (count == 0) {
        h->resp.over_valid = false;
        h->resp.h_valid = false;
        h->resp.armed = false;
        return HZ_OK;
    }
    HZ_TRY(resp_setup(h));
    if (h->resp.K <= 0 || count < h->resp.K || count % 8192 != 0 || count > (1L << 19)) {
        hz::set_error("hz_fb_set_bank_response: %ld values (a multiple of 8192, at least this shard's "
                      "horizon %ld)", count, h->resp.K);
        return HZ_E_INVALID;
    }
    if (count > h->resp.K) {   // the bank's horizon (another shard's bands ring longer): a longer history
        h->resp.K = count;
        HZ_TRY(resp_setup(h));
    }
    // every rank restarts its history count here, whatever its own horizon was, so the ranks'
    // readiness (hz_fb_stationary_ready) evolves alike from this call on
    h->resp.run = 0;
    h->resp.h_over.assign(resp, resp + count);
    h->resp.over_valid = true;
    h->resp.h_valid = false;
    h->resp.armed = false;
    return HZ_OK;
}

int hz_fb_set_time_shard(hz_fb* h, int rank, int world) {
    if (!h || world < 1 || rank < 0 || rank >= world) return HZ_E_INVALID;
    h->resp.shard_rank = rank;
    h->resp.shard_world = world;
    h->resp.armed = false;
    return HZ_OK;
}

int hz_fb_set_time_shard_fill(hz_fb* h, int zero_outside) {
    if (!h) return HZ_E_INVALID;
    h->resp.shard_zero = zero_outside != 0;
    return HZ_OK;
}

int hz_fb_stationary_ready(hz_fb* h, long n, int* ready) {
    if (!h || !ready || n < 0) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->device));
    const bool conv = h->order > 0 && n >= 16 && hz_fbi::fb_converged(h);
    *ready = hz_fbi::fb_resp_eligible(h, n, conv) ? 1 : 0;
    return HZ_OK;
}

int hz_fb_arm_time_shard(hz_fb* h, int armed) {
    if (!h) return HZ_E_INVALID;
    if (armed && !hz_fbi::fb_resp_time_sharded(h)) {
        hz::set_error("hz_fb_arm_time_shard: no time shard set (hz_fb_set_bank_response + hz_fb_set_time_shard)");
        return HZ_E_STATE;
    }
    h->resp.armed = armed != 0;
    return HZ_OK;
}

int hz_fb_tune_response_engine(hz_fb* h, int column_split) {
    if (!h) return HZ_E_INVALID;
    const bool on = column_split != 0;
    h->resp.col_on = on;
    return HZ_OK;
}

int hz_fb_tune_modal(hz_fb* h, int on) {
    if (!h) return HZ_E_INVALID;
    h->resp.modal_on = on != 0;
    return HZ_OK;
}

int hz_fb_modal_info(hz_fb* h, int* on, int* qualifies, int* exceptional, int* last_call) {
    if (!h) return HZ_E_INVALID;
    if (on) *on = h->resp.modal_on ? 1 : 0;
    if (qualifies) *qualifies = h->resp.modal_ok ? 1 : 0;
    if (exceptional) *exceptional = h->resp.modal_ok ? h->resp.mexc_n : -1;
    if (last_call) *last_call = h->resp.modal_last ? 1 : 0;
    return HZ_OK;
}

int hz_fb_response_engine(hz_fb* h, int* column_split_on, int* last_call_column_split) {
    if (!h) return HZ_E_INVALID;
    if (column_split_on) *column_split_on = h->resp.col_on ? 1 : 0;
    if (last_call_column_split) *last_call_column_split = h->resp.last_engine;
    return HZ_OK;
}

int hz_fb_tune_response(hz_fb* h, long min_call, long bands_per_sample) {
    if (!h || min_call < 0 || bands_per_sample < 0) return HZ_E_INVALID;
    h->resp.min_call = min_call;                                   // 0: 16384
    h->resp.bands_per_sample = bands_per_sample ? bands_per_sample : -1;   // 0: 256 (HZ_FB_RESP_BANDS)
    return HZ_OK;
}

int hz_fb_time_shard_info(hz_fb* h, int* active, long* first, long* count, long n) {
    if (!h) return HZ_E_INVALID;
    const hz_fb::Resp& R = h->resp;
    const bool on = R.shard_world > 1 && R.over_valid;
    long lo = 0, cnt = n;
    if (on) {
        const long Ball = (n + kP - 1) / kP;
        lo = std::min(n, Ball * R.shard_rank / R.shard_world * kP);
        cnt = std::min(n, Ball * (R.shard_rank + 1) / R.shard_world * kP) - lo;
    }
    if (active) *active = on ? 1 : 0;
    if (first) *first = lo;
    if (count) *count = cnt;
    return HZ_OK;
}

int hz_fb_response_info(hz_fb* h, long* horizon, long* run, int* implicit_state, long* calls) {
    if (!h) return HZ_E_INVALID;
    if (horizon) *horizon = h->resp.K;
    if (run) *run = h->resp.run;
    if (implicit_state) *implicit_state = h->resp.implicit ? 1 : 0;
    if (calls) *calls = h->resp.calls;
    return HZ_OK;
}

int hz_fb_get_response(hz_fb* h, double* out, long count) {
    if (!h || !out || count < 0) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->device));
    HZ_TRY(hz_fbi::fb_upload_staged(h));
    if (h->order == 0) {
        hz::set_error("hz_fb_get_response: order 0 bank");
        return HZ_E_INVALID;
    }
    HZ_TRY(resp_setup(h));
    if (h->resp.K <= 0) {
        hz::set_error("hz_fb_get_response: no finite horizon (some band needs more than 2^18 samples)");
        return HZ_E_UNSUPPORTED;
    }
    HZ_TRY(resp_build_h(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    const long c = std::min(count, h->resp.K);
    HZ_TRY_HIP(hipMemcpy(out, h->resp.d_h, sizeof(double) * c, hipMemcpyDeviceToHost));
    for (long i = c; i < count; ++i) out[i] = 0.0;
    return HZ_OK;
}

}  // extern "C"
