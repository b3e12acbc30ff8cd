// hz_stft.hip -- Fourier / StaticSTFT overlap-add engines and Cosine (DCT) for MI355X.
//
// Replaces src/fourier.h:50-194 (Fourier, halfhann windows, processor callback),
// src/staticSTFT.h:10-177 (hann windows, built-in gate) and src/fourier.h:197-234 (Cosine).
//
// The reference runs a per-sample state machine over 2*laps slots (write() then read()
// per sample).  Its schedule has a closed form: frame f = c*2*laps + i of
// slot i covers input [s, s+N-1], s = stride*i + c*(2N-1), and emits its IFFT sample k,
// weighted by w(k/N), at t = s+N-1+k; frames are ordered by completion time, so the
// frames completing inside a block are a contiguous range [f_lo, f_hi).  A block is:
//   1. stage the block's input behind the previous N-1 samples (history);
//   2. one workgroup per completing frame: window -> FFT -> processor -> IFFT entirely in
//      LDS (bit-reversed spectrum between the two transforms, hz_fft.h), frame output to a
//      ring of R frame buffers in HBM;
//   3. overlap-add: one thread per output sample sums the (<= 2 laps) reading slots in slot
//      order, in double-double (the reference accumulates in long double), and divides by
//      the int N*laps/2.
// Processors: identity, the StaticSTFT gate (staticSTFT.h:99-128), the spectral.cpp 625
// gate (tests/spectral.cpp:32-72), the Hilbert half-band (tests/SFML/hilbert.cpp:37-49) as
// device code; any other host function pointer runs per frame, in frame order, on the host
// between a forward-only and an inverse-only kernel, with each slot's `out` buffer kept
// between frames as in the reference (fourier.h:57-59).
//
// Cosine: REDFT10 (DCT-II) and REDFT01 (DCT-III) through one complex FFT of length N
// (Makhoul's even/odd reordering), in LDS, batched one transform per workgroup.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "hz_common.h"
#include "hz_fft.h"

// Experiment builds only (-DHZ_STFT_ABLATE=mask; wrong results): 1 skip the processor,
// 2 skip the inverse FFT, 4 skip the forward FFT, 8 skip the ring store, 16 twiddles = tw[0].
#ifndef HZ_STFT_ABLATE
#define HZ_STFT_ABLATE 0
#endif

namespace {

constexpr int kThreads = 1024;       // DCT workgroups: one radix-4 butterfly per thread at N = 4096
constexpr int kFrameThreads = 512;   // STFT frame workgroups (N/8 threads at N = 4096, N/16 at 8192)
constexpr int kMaxN = 8192;          // complex FP64 frame fully resident in LDS (128 KB)
constexpr long kChunkMax = 1L << 20;          // samples per internal block: one frame launch each
constexpr size_t kRingBytes = 128u << 20;     // frame-ring budget that caps the block below kChunkMax

struct StftArgs {
    const double* hr;     // history: hr[k] = Re input at time T0 - (N-1) + k, k < N-1
    const double* hi;     // its Im plane; null when every sample this launch reads is real
    const double* inr;    // this block's input (caller memory): time T0 + k
    const double* ini;    // its Im part (may be null: real input)
    double* fo;           // frame-output ring, planar: Re [R][N] then Im [R][N]
    double2* spec;        // host-processor path: spectra [frames][N] (natural order)
    const double* win;    // [N]
    const double2* tw;    // [N/2]  e^{-2 pi i k/N}
    long f_lo, T0;
    int N, lg, laps, stride, R;
    double p0, p1;
    // time-range shards: the launch's frames are this rank's runs of sh_block frames, the
    // first run (index sh_q0) entered sh_off frames in; sh_world <= 1: f_lo, f_lo + 1, ...
    long sh_q0, sh_block;
    int sh_off, sh_world;
    // unsharded launches (stft_pair4096_kernel): frame f_lo + i starts at position
    // u0 + c (2N - 1) + stride r, (c, r) = (i0 + i) divmod 2 laps, and fills ring row (r0 + i) mod R
    // -- the 64-bit divides of frame_at / frame_start / f % R done once on the host
    long u0;
    int i0, r0;
};

// the launch's i-th frame (one 64-bit divide per workgroup when sharded)
__device__ __forceinline__ long frame_at(const StftArgs& a, long i) {
    if (a.sh_world <= 1) return a.f_lo + i;
    const long p = i + a.sh_off, k = p / a.sh_block;
    return (a.sh_q0 + k * a.sh_world) * a.sh_block + (p - k * a.sh_block);
}

__host__ __device__ __forceinline__ long frame_start(long f, int laps, int stride, int N) {
    const long c = f / (2 * laps);
    const int i = (int)(f - c * 2 * laps);
    return (long)stride * i + c * (2L * N - 1);
}

// block-wide sum (wave64 shuffles + LDS across waves); all threads get the result
__device__ __forceinline__ double block_sum(double v, double* scratch) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) scratch[wave] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += scratch[w];
    return s;
}

__device__ __forceinline__ void block_sum_dd(double& hi, double& lo, double* scratch) {
    for (int o = 32; o > 0; o >>= 1) {
        const double oh = __shfl_xor(hi, o, 64), ol = __shfl_xor(lo, o, 64);
        hz::dd_add(hi, lo, oh);
        hz::dd_add(hi, lo, ol);
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0) {
        scratch[2 * wave] = hi;
        scratch[2 * wave + 1] = lo;
    }
    __syncthreads();
    double h = 0.0, l = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        hz::dd_add(h, l, scratch[2 * w]);
        hz::dd_add(h, l, scratch[2 * w + 1]);
    }
    hi = h;
    lo = l;
}

// Device processors on one group of spectrum slots held in registers: slots e0 + j
// (bit-reversed order, bin k = bitrev(e0 + j)); `act` false for threads without a group.
// Every thread calls this (the gates reduce over the whole frame).
template <int PROC, int M>
__device__ __forceinline__ void apply_proc(double* xr, double* xi, bool act, int e0, int N, double p0, double p1,
                                           double* scratch) {
#pragma clang fp contract(off)
    if constexpr (PROC == HZ_PROC_STATIC_GATE) {   // staticSTFT.h:99-128
        const double inv_n = 1.0 / N;   // exact (N = 2^lg): same as the reference's / N
        double part = 0.0;
        if (act)
#pragma unroll
            for (int j = 0; j < M; ++j) part += sqrt(xr[j] * xr[j] + xi[j] * xi[j]) * inv_n;
        const double average = block_sum(part, scratch);
        const double thr = p0 * average * average;
        if (act)
#pragma unroll
            for (int j = 0; j < M; ++j)
                if (xr[j] * xr[j] + xi[j] * xi[j] < thr) {
                    xr[j] = xr[j] * p1;
                    xi[j] = xi[j] * p1;
                }
    } else if constexpr (PROC == HZ_PROC_GATE_KEEP) {   // tests/spectral.cpp:32-72
        double hi = 0.0, lo = 0.0;
        if (act)
#pragma unroll
            for (int j = 0; j < M; ++j) hz::dd_add(hi, lo, hypot(xr[j], xi[j]));
        block_sum_dd(hi, lo, scratch);
        // average = sum / N (long double in the reference); thr = p0 * average^2
        const double q = hi / N;
        const double avg = q + (fma(-q, (double)N, hi) + lo) / N;
        const double thr = p0 * avg * avg;
        if (act)
#pragma unroll
            for (int j = 0; j < M; ++j)
                if (!(xr[j] * xr[j] + xi[j] * xi[j] > thr)) {
                    xr[j] = 0.0;
                    xi[j] = 0.0;
                }
    } else if constexpr (PROC == HZ_PROC_HILBERT) {   // bins k < N/2 kept: even slots
        if (act)
#pragma unroll
            for (int j = 0; j < M; ++j)
                if ((e0 + j) & 1) {
                    xr[j] = 0.0;
                    xi[j] = 0.0;
                }
    }
    (void)e0;
}

// The fused middle of a frame: last forward pass, processor, first inverse pass, all on the
// same contiguous group {b 2^R + j} in registers (one group per thread)
template <int R, int PROC>
__device__ __forceinline__ void frame_middle(double* re, double* im, int lg, double p0, double p1, double* scratch,
                                             const double2* T) {
    constexpr int M = 1 << R;
    const int b = threadIdx.x, e0 = b << R;
    const bool act = b < (1 << (lg - R));
    double xr[M], xi[M];
    if (act) {
#pragma unroll
        for (int j = 0; j < M; ++j) {
            xr[j] = re[hz::pad16(e0 + j)];
            xi[j] = im[hz::pad16(e0 + j)];
        }
        if constexpr (!(HZ_STFT_ABLATE & 4)) hz::dif_regs<R, false>(xr, xi, lg, R - 1, 0, T);
    }
    if constexpr (!(HZ_STFT_ABLATE & 1)) apply_proc<PROC, M>(xr, xi, act, e0, 1 << lg, p0, p1, scratch);
    if (act) {
        if constexpr (!(HZ_STFT_ABLATE & 2)) hz::dit_regs<R, false>(xr, xi, lg, 0, 0, T);
#pragma unroll
        for (int j = 0; j < M; ++j) {
            re[hz::pad16(e0 + j)] = xr[j];
            im[hz::pad16(e0 + j)] = xi[j];
        }
    }
}

// stages per LDS pass: radix 8 up to N = 4096 (512 threads, 8 waves per frame), radix 16 above
#ifndef HZ_STFT_R4_ABOVE
#define HZ_STFT_R4_ABOVE 4096
#endif
inline int frame_rmax(int N) { return N > HZ_STFT_R4_ABOVE ? 4 : 3; }

// XCD-aware frame order: workgroups go round-robin over the 8 XCDs, so give each XCD a
// contiguous run of frames -- overlapping frames then share input lines in that XCD's L2
__device__ __forceinline__ int frame_of_block(int b, int nf) {
    const int x = b & 7, q = nf >> 3, r = nf & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// threads per frame workgroup: one radix-2^rmax group per thread, at least one wave
inline int frame_threads(int N) {
    const int t = N >> frame_rmax(N);
    return t < 64 ? 64 : (t > kFrameThreads ? kFrameThreads : t);
}

// dynamic LDS of a frame workgroup: padded re/im, the block-sum scratch, the compact twiddles
inline size_t frame_lds(int N) {
    int lg = 0;
    while ((1 << lg) < N) ++lg;
    return sizeof(double) * (2 * (size_t)hz::padded_len(N) + 2 * (size_t)(frame_threads(N) / 64)) +
           sizeof(double2) * (size_t)hz::twc_len(lg);
}

// One workgroup per frame; the frame stays in LDS from the window to the overlap-add ring.
// MODE 0: fused (window, FFT, device processor, IFFT -> ring)
// MODE 1: forward only (window, FFT -> spec, natural order)
// MODE 2: inverse only (spec -> IFFT -> ring)
template <int PROC, int MODE, int RMAX>
__global__ __launch_bounds__(kFrameThreads) void stft_frame_kernel(StftArgs a) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int N = a.N, lg = a.lg;
    double* re = lds;
    double* im = lds + hz::padded_len(N);
    double* scratch = im + hz::padded_len(N);
    double2* T = (double2*)(scratch + 2 * (blockDim.x >> 6));
    for (int k = threadIdx.x; k < hz::twc_len(lg); k += blockDim.x) T[k] = a.tw[k];
    const int fl = frame_of_block(blockIdx.x, gridDim.x);   // frame within the launch
    const long f = frame_at(a, fl);
    if constexpr (MODE != 2) {
        const long off = frame_start(f, a.laps, a.stride, N) - a.T0 + (N - 1);
        constexpr int PB = 8;   // batches of 8 samples per thread, loads before stores
        for (int k0 = threadIdx.x; k0 < N; k0 += PB * blockDim.x) {
            double vr[PB], vi[PB], w[PB];
#pragma unroll
            for (int i = 0; i < PB; ++i) {
                const int k = k0 + i * blockDim.x;
                const long u = off + k;   // position in [history (N-1) | block input]
                vr[i] = vi[i] = w[i] = 0.0;
                if (k < N) {
                    if (u < N - 1) {
                        vr[i] = a.hr[u];
                        if (a.hi) vi[i] = a.hi[u];
                    } else {
                        vr[i] = a.inr[u - (N - 1)];
                        if (a.hi && a.ini) vi[i] = a.ini[u - (N - 1)];
                    }
                    w[i] = a.win[k];
                }
            }
#pragma unroll
            for (int i = 0; i < PB; ++i) {
                const int k = k0 + i * blockDim.x;
                if (k < N) {
                    const int e = hz::pad16(k);
                    re[e] = w[i] * vr[i];   // fourier.h:110-112: window * real, window * imag
                    im[e] = w[i] * vi[i];
                }
            }
        }
    } else {
        const double2* sp = a.spec + (long)fl * N;
        for (int p = threadIdx.x; p < N; p += blockDim.x) {
            const double2 v = sp[hz::bitrev(p, lg)];
            const int e = hz::pad16(p);
            re[e] = v.x;
            im[e] = v.y;
        }
    }
    __syncthreads();
    if constexpr (MODE == 1) {
        hz::fft_fwd_lead<RMAX>(re, im, lg, T, true);
        double2* sp = a.spec + (long)fl * N;
        for (int p = threadIdx.x; p < N; p += blockDim.x) {
            const int e = hz::pad16(p);
            sp[hz::bitrev(p, lg)] = make_double2(re[e], im[e]);
        }
        return;
    } else if constexpr (MODE == 2) {
        hz::fft_inv_tail<RMAX>(re, im, lg, T, true);
    } else {
        if constexpr (!(HZ_STFT_ABLATE & 4)) hz::fft_fwd_lead<RMAX>(re, im, lg, T, false);
        switch (hz::fft_rlast<RMAX>(lg)) {
        case 4: if constexpr (RMAX >= 4) frame_middle<4, PROC>(re, im, lg, a.p0, a.p1, scratch, T); break;
        case 3: frame_middle<3, PROC>(re, im, lg, a.p0, a.p1, scratch, T); break;
        default: frame_middle<2, PROC>(re, im, lg, a.p0, a.p1, scratch, T); break;   // N = 4
        }
        __syncthreads();
        if constexpr (!(HZ_STFT_ABLATE & 2)) hz::fft_inv_tail<RMAX>(re, im, lg, T, false);
    }
    double* out = a.fo + (f % a.R) * N;
    const long plane = (long)a.R * N;
    if constexpr ((HZ_STFT_ABLATE & 8) != 0) return;
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        const int e = hz::pad16(k);
        out[k] = re[e];
        out[plane + k] = im[e];
    }
}

// Two real frames per complex transform (real input, symmetric gates).  While every sample a
// launch reads is real (StftArgs::hi == nullptr) and the processor is a magnitude gate (its
// keep/scale decision is the same for bins k and N - k of a real frame), frames f and f + 1
// share one FFT pair: z = w x_f + i w x_{f+1}, Z = FFT(z), then per bin pair (k, N - k)
//     X_f = (Z_k + conj Z_{N-k}) / 2,   X_{f+1} = (Z_k - conj Z_{N-k}) / 2i,
// each frame's gate on its own spectrum (its own average), Y = Y_f + i Y_{f+1} (both Hermitian),
// and one inverse FFT gives y_f + i y_{f+1}.  Half the FFT work per frame; the Im output of a
// real frame is written as 0 (the reference's complex transform leaves ~1e-17 there).
// bin pairs per thread: ceil((N/2 + 1) / threads), threads = N/8 (radix 8) or N/16 (radix 16)
template <int RMAX>
__host__ __device__ constexpr int pair_items() { return RMAX == 3 ? 5 : 9; }

template <int PROC, int kPairItems>
__device__ __forceinline__ void pair_gate(double* re, double* im, int lg, double p0, double p1, double* scratch) {
#pragma clang fp contract(off)
    const int N = 1 << lg, H = N >> 1;
    double ar[kPairItems], ai[kPairItems], br[kPairItems], bi[kPairItems];
    double pa = 0.0, pb = 0.0, la = 0.0, lb = 0.0;   // magnitude sums (GATE_KEEP: double-double)
#pragma unroll
    for (int i = 0; i < kPairItems; ++i) {
        const int k = threadIdx.x + i * blockDim.x;
        ar[i] = ai[i] = br[i] = bi[i] = 0.0;
        if (k <= H) {
            const int m = (N - k) & (N - 1);
            const int ek = hz::pad16(hz::bitrev(k, lg)), em = hz::pad16(hz::bitrev(m, lg));
            const double zr = re[ek], zi = im[ek], wr = re[em], wi = im[em];
            ar[i] = (zr + wr) * 0.5;   // X_f
            ai[i] = (zi - wi) * 0.5;
            br[i] = (zi + wi) * 0.5;   // X_{f+1}
            bi[i] = (wr - zr) * 0.5;
            const double c = (k == 0 || k == H) ? 1.0 : 2.0;   // bins k and N - k
            if constexpr (PROC == HZ_PROC_STATIC_GATE) {
                pa += c * (sqrt(ar[i] * ar[i] + ai[i] * ai[i]) / N);
                pb += c * (sqrt(br[i] * br[i] + bi[i] * bi[i]) / N);
            } else {
                const double ha = hypot(ar[i], ai[i]), hb = hypot(br[i], bi[i]);
                hz::dd_add(pa, la, ha);
                hz::dd_add(pb, lb, hb);
                if (c == 2.0) {
                    hz::dd_add(pa, la, ha);
                    hz::dd_add(pb, lb, hb);
                }
            }
        }
    }
    double thra, thrb;
    if constexpr (PROC == HZ_PROC_STATIC_GATE) {   // staticSTFT.h:99-128
        const double avga = block_sum(pa, scratch), avgb = block_sum(pb, scratch);
        thra = p0 * avga * avga;
        thrb = p0 * avgb * avgb;
    } else {   // tests/spectral.cpp:32-72 (sum / N in long double)
        block_sum_dd(pa, la, scratch);
        block_sum_dd(pb, lb, scratch);
        const double qa = pa / N, qb = pb / N;
        const double avga = qa + (fma(-qa, (double)N, pa) + la) / N;
        const double avgb = qb + (fma(-qb, (double)N, pb) + lb) / N;
        thra = p0 * avga * avga;
        thrb = p0 * avgb * avgb;
    }
#pragma unroll
    for (int i = 0; i < kPairItems; ++i) {
        const int k = threadIdx.x + i * blockDim.x;
        if (k > H) continue;
        double xr = ar[i], xi = ai[i], yr = br[i], yi = bi[i];
        if constexpr (PROC == HZ_PROC_STATIC_GATE) {
            if (xr * xr + xi * xi < thra) {
                xr = xr * p1;
                xi = xi * p1;
            }
            if (yr * yr + yi * yi < thrb) {
                yr = yr * p1;
                yi = yi * p1;
            }
        } else {
            if (!(xr * xr + xi * xi > thra)) xr = xi = 0.0;
            if (!(yr * yr + yi * yi > thrb)) yr = yi = 0.0;
        }
        const int m = (N - k) & (N - 1);
        const int ek = hz::pad16(hz::bitrev(k, lg)), em = hz::pad16(hz::bitrev(m, lg));
        // Y_k = X_f + i X_{f+1};  Y_{N-k} = conj X_f + i conj X_{f+1}
        re[ek] = xr - yi;
        im[ek] = xi + yr;
        if (m != k) {
            re[em] = xr + yi;
            im[em] = yr - xi;
        }
    }
}

template <int PROC, int RMAX>
__global__ __launch_bounds__(kFrameThreads) void stft_pair_kernel(StftArgs a, long nf) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int N = a.N, lg = a.lg;
    double* re = lds;
    double* im = lds + hz::padded_len(N);
    double* scratch = im + hz::padded_len(N);
    double2* T = (double2*)(scratch + 2 * (blockDim.x >> 6));
    for (int k = threadIdx.x; k < hz::twc_len(lg); k += blockDim.x) T[k] = a.tw[k];
    const int pl = frame_of_block(blockIdx.x, gridDim.x);   // frame pair within the launch
    const long f0 = frame_at(a, 2L * pl);
    const bool two = 2L * pl + 1 < nf;
    const long f1 = two ? frame_at(a, 2L * pl + 1) : f0;
    const long off0 = frame_start(f0, a.laps, a.stride, N) - a.T0 + (N - 1);
    const long off1 = two ? frame_start(f1, a.laps, a.stride, N) - a.T0 + (N - 1) : 0;
    // batches of 8 samples per thread: every global load of a batch issued before its LDS stores
    // (one memory latency per batch instead of one per sample; a 4096-point frame is one batch)
    constexpr int PB = 8;
    for (int k0 = threadIdx.x; k0 < N; k0 += PB * blockDim.x) {
        double v0[PB], v1[PB], w[PB];
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            const int k = k0 + i * blockDim.x;
            const bool ok = k < N;
            const long u0 = off0 + k, u1 = off1 + k;   // positions in [history (N-1) | block input]
            v0[i] = ok ? (u0 < N - 1 ? a.hr[u0] : a.inr[u0 - (N - 1)]) : 0.0;
            v1[i] = ok && two ? (u1 < N - 1 ? a.hr[u1] : a.inr[u1 - (N - 1)]) : 0.0;
            w[i] = ok ? a.win[k] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < PB; ++i) {
            const int k = k0 + i * blockDim.x;
            if (k < N) {
                const int e = hz::pad16(k);
                re[e] = w[i] * v0[i];   // fourier.h:110-112, real input
                im[e] = w[i] * v1[i];
            }
        }
    }
    __syncthreads();
    hz::fft_fwd_lead<RMAX>(re, im, lg, T, true);
    pair_gate<PROC, pair_items<RMAX>()>(re, im, lg, a.p0, a.p1, scratch);
    __syncthreads();
    hz::fft_inv_tail<RMAX>(re, im, lg, T, true);
    double* o0 = a.fo + (f0 % a.R) * N;
    double* o1 = a.fo + (f1 % a.R) * N;
    // the Re planes only: a real frame's Im output is 0, which the overlap-add knows
    // (hz_stft::im_zero_from) instead of reading 2 N zeros per pair back from the ring
    for (int k = threadIdx.x; k < N; k += blockDim.x) {
        const int e = hz::pad16(k);
        o0[k] = re[e];
        if (two) o1[k] = im[e];
    }
}

// ---- N = 4096 pair frames (StaticSTFT's default size; C4), specialised ---------------------------
// stft_pair_kernel<PROC, 3> at lg = 12 with the pass plan fixed at compile time: the same stage
// arithmetic (hz::dif_regs / dit_regs order, the same twiddle values, so the same bits), with
//   * the twiddles expanded once per workgroup from the compact table into a full half-table in
//     LDS (one lookup per stage instead of the symmetry selects of hz::twc),
//   * the frame in LDS at e ^ ((e >> 3) & 31): every pass of the plan conflict-free
//     (scripts/probe/stft_layout.py; the pad16 layout cost 62 % of the LDS cycles in bank
//     conflicts, rocprofv3 SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE on the C4 step),
//   * the window product straight into the first pass's registers and the last inverse pass
//     straight to the ring (two LDS round trips fewer),
//   * the pair gate walking spectrum POSITIONS: bin k = bitrev(q) pairs with bin N - k at
//     q ^ (hibit(q) - 1), the mirror of q within its power-of-two octave, so both reads of a
//     pair run over contiguous positions.
namespace p4 {
constexpr int kLg = 12, kN = 1 << kLg, kH = kN / 2, kT = kN / 8;
__device__ __forceinline__ int lx(int e) { return e ^ ((e >> 3) & 31); }
inline size_t lds_bytes() { return sizeof(double) * 2 * kN + sizeof(double) * 32; }

// (x + iy) *= w (conj: w̄): contracted (FMA); the FFT passes of this kernel need no op-by-op
// agreement with the generic kernel, only the tolerance of the parity tests
__device__ __forceinline__ void cmul_fma(double& r, double& i, double2 w, bool conj) {
    const double wi = conj ? -w.y : w.y;
    const double nr = fma(r, w.x, -i * wi);
    const double ni = fma(r, wi, i * w.x);
    r = nr;
    i = ni;
}

// Twiddles once per element (an A/B alternative; the stage-wise form below is the default): a radix-8 DIF group {base + j d} (p its offset in the span) is the
// 8-point DFT of its elements followed by W_N^(e r) on output j, r = bitrev3(j), e = p 2^(lg-1-lh);
// the DIT group mirrors it (conj W_N^(e r) on input j, e = p 2^(lg-3-lh), then the butterflies).
// The stage-by-stage form (hz::dif_regs / dit_regs) multiplied every stage's differences: 12
// complex products per group and pass against 7 here.  Host-built tables after the N/2 table
// (hz_stft_create), contiguous in p: A[r-1][p] = W^(p r), p < 512 (forward lh 11, inverse lh 9);
// B[r-1][p] = W^(8 p r), p < 64 (lh 8 / 6); C[r-1][p] = W^(64 p r), p < 8 (lh 5 / 3); lh 2 / 0 have
// p = 0 (no twiddles).  A thread's 21 twiddles load once.
constexpr int kTwA = 0, kTwB = 7 * 512, kTwC = kTwB + 7 * 64, kTwLen = kTwC + 7 * 8;
constexpr int kBr3[8] = {0, 4, 2, 6, 1, 5, 3, 7};

// the stage-by-stage form (hz::dif_regs<3, true> order: stage k's differences times W^(e 2^k))
template <bool UNIT>
__device__ __forceinline__ void dif8s(double (&xr)[8], double (&xi)[8], const double2 (&tw)[7]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int S = 8 >> (k + 1);
        const double2 w = tw[(1 << k) - 1];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j & S) continue;
            const double ar = xr[j], ai = xi[j], cr = xr[j + S], ci = xi[j + S];
            double dr = ar - cr, di = ai - ci;
            if (!UNIT) cmul_fma(dr, di, w, false);
            hz::mul_root16(dr, di, (j & (S - 1)) << (1 + k), false);
            xr[j] = ar + cr;
            xi[j] = ai + ci;
            xr[j + S] = dr;
            xi[j + S] = di;
        }
    }
}

// hz::dit_regs<3, true> order: stage k's second inputs times conj W^(e 2^(2-k))
template <bool UNIT>
__device__ __forceinline__ void dit8s(double (&xr)[8], double (&xi)[8], const double2 (&tw)[7]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int S = 1 << k;
        const double2 w = tw[(1 << (2 - k)) - 1];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j & S) continue;
            double cr = xr[j + S], ci = xi[j + S];
            if (!UNIT) cmul_fma(cr, ci, w, true);
            hz::mul_root16(cr, ci, (j & (S - 1)) << (3 - k), true);
            const double ar = xr[j], ai = xi[j];
            xr[j] = ar + cr;
            xi[j] = ai + ci;
            xr[j + S] = ar - cr;
            xi[j + S] = ai - ci;
        }
    }
}

// radix-8 DIF group: butterflies with the pass-internal roots, then the output twiddles
template <bool UNIT>
__device__ __forceinline__ void dif8(double (&xr)[8], double (&xi)[8], const double2 (&tw)[7]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int S = 8 >> (k + 1);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j & S) continue;
            const double ar = xr[j], ai = xi[j], cr = xr[j + S], ci = xi[j + S];
            double dr = ar - cr, di = ai - ci;
            hz::mul_root16(dr, di, (j & (S - 1)) << (1 + k), false);
            xr[j] = ar + cr;
            xi[j] = ai + ci;
            xr[j + S] = dr;
            xi[j + S] = di;
        }
    }
    if (!UNIT) {
#pragma unroll
        for (int j = 1; j < 8; ++j) cmul_fma(xr[j], xi[j], tw[kBr3[j] - 1], false);
    }
}

// radix-8 DIT group: the input twiddles (conjugate), then the butterflies with the internal roots
template <bool UNIT>
__device__ __forceinline__ void dit8(double (&xr)[8], double (&xi)[8], const double2 (&tw)[7]) {
    if (!UNIT) {
#pragma unroll
        for (int j = 1; j < 8; ++j) cmul_fma(xr[j], xi[j], tw[kBr3[j] - 1], true);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int S = 1 << k;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            if (j & S) continue;
            double cr = xr[j + S], ci = xi[j + S];
            hz::mul_root16(cr, ci, (j & (S - 1)) << (3 - k), true);
            const double ar = xr[j], ai = xi[j];
            xr[j] = ar + cr;
            xi[j] = ai + ci;
            xr[j + S] = ar - cr;
            xi[j + S] = ai - ci;
        }
    }
}

template <int LD>   // a DIF pass's group (fft_fwd_lead: lh = LD + 2): base, stride 2^LD
__device__ __forceinline__ int dif_base(int b) { return ((b >> LD) << (LD + 3)) + (b & ((1 << LD) - 1)); }
template <int LH>   // a DIT pass's group (fft_inv_tail): base, stride 2^LH
__device__ __forceinline__ int dit_base(int b) { return ((b >> LH) << (LH + 3)) + (b & ((1 << LH) - 1)); }

// the frame as interleaved complex: one ds_read_b128 / ds_write_b128 per element (b128 reads reach
// the LDS rate at one wave per SIMD, b64 reads need about four)
template <int STRIDE>
__device__ __forceinline__ void lds_get(const double2* z, int base, double (&xr)[8], double (&xi)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const double2 v = z[lx(base + j * STRIDE)];
        xr[j] = v.x;
        xi[j] = v.y;
    }
}
template <int STRIDE>
__device__ __forceinline__ void lds_put(double2* z, int base, const double (&xr)[8], const double (&xi)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) z[lx(base + j * STRIDE)] = make_double2(xr[j], xi[j]);
}

__device__ __forceinline__ int hibit(int x) { return 1 << (31 - __builtin_clz(x)); }

// After the first forward pass the 4096-point DIF splits into eight 512-point transforms, and the
// groups of forward lh 8, 5, 2 and inverse lh 0, 3, 6 of wave w all lie in [512 w, 512 w + 512):
// between those passes a wave waits only for its own LDS writes (a wave's LDS operations complete
// in order), not for the workgroup
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// pair_gate over positions (see above); c = 2 for a pair, 1 for bins 0 and N/2
template <int PROC>
__device__ __forceinline__ void gate(double2* zf, double p0, double p1, double* scratch) {
#pragma clang fp contract(off)
    constexpr int kItems = 5;   // 2047 pairs + the two self-paired bins (u = 2047, 2048) over 512 threads
    const int b = threadIdx.x;
    double ar[kItems], ai[kItems], br[kItems], bi[kItems];
    int ek[kItems], em[kItems];
    bool live[kItems], self[kItems];
    double pa = 0.0, pb = 0.0, la = 0.0, lb = 0.0;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const int u = b + kT * i;
        int q, qq;
        if (u < kH - 1) {
            q = (u + 1) + hibit(u + 1);
            qq = q ^ (hibit(q) - 1);
        } else {   // u = 2047: bin 0 (position 0); u = 2048..: bin N/2 (position 1) on u = 2048 only
            q = qq = u == kH - 1 ? 0 : 1;
        }
        live[i] = u <= kH;
        self[i] = q == qq;
        // k <= N/2 is the pair's first bin (pair_gate's k), m = N - k its partner
        const int kq = hz::bitrev(q, kLg), kqq = hz::bitrev(qq, kLg);
        const int qk = kq <= kqq ? q : qq, qm = kq <= kqq ? qq : q;
        ek[i] = lx(qk);
        em[i] = lx(qm);
        ar[i] = ai[i] = br[i] = bi[i] = 0.0;
        if (live[i]) {
            const double2 zv = zf[ek[i]], wv = zf[em[i]];
            const double zr = zv.x, zi = zv.y, wr = wv.x, wi = wv.y;
            ar[i] = (zr + wr) * 0.5;   // X_f
            ai[i] = (zi - wi) * 0.5;
            br[i] = (zi + wi) * 0.5;   // X_{f+1}
            bi[i] = (wr - zr) * 0.5;
            const double c = self[i] ? 1.0 : 2.0;
            if constexpr (PROC == HZ_PROC_STATIC_GATE) {
                pa += c * (sqrt(ar[i] * ar[i] + ai[i] * ai[i]) / kN);
                pb += c * (sqrt(br[i] * br[i] + bi[i] * bi[i]) / kN);
            } else {
                const double ha = hypot(ar[i], ai[i]), hb = hypot(br[i], bi[i]);
                hz::dd_add(pa, la, ha);
                hz::dd_add(pb, lb, hb);
                if (c == 2.0) {
                    hz::dd_add(pa, la, ha);
                    hz::dd_add(pb, lb, hb);
                }
            }
        }
    }
    double thra, thrb;
    // both frames' sums in one reduction (block_sum / block_sum_dd's order for each)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if constexpr (PROC == HZ_PROC_STATIC_GATE) {   // staticSTFT.h:99-128
        for (int o = 32; o > 0; o >>= 1) {
            pa += __shfl_xor(pa, o, 64);
            pb += __shfl_xor(pb, o, 64);
        }
        if (lane == 0) {
            scratch[2 * wave] = pa;
            scratch[2 * wave + 1] = pb;
        }
        __syncthreads();
        double avga = 0.0, avgb = 0.0;
        for (int w = 0; w < kT / 64; ++w) {
            avga += scratch[2 * w];
            avgb += scratch[2 * w + 1];
        }
        thra = p0 * avga * avga;
        thrb = p0 * avgb * avgb;
    } else {   // tests/spectral.cpp:32-72 (sum / N in long double)
        for (int o = 32; o > 0; o >>= 1) {
            const double ah = __shfl_xor(pa, o, 64), al = __shfl_xor(la, o, 64);
            const double bh = __shfl_xor(pb, o, 64), bl = __shfl_xor(lb, o, 64);
            hz::dd_add(pa, la, ah);
            hz::dd_add(pa, la, al);
            hz::dd_add(pb, lb, bh);
            hz::dd_add(pb, lb, bl);
        }
        if (lane == 0) {
            scratch[4 * wave] = pa;
            scratch[4 * wave + 1] = la;
            scratch[4 * wave + 2] = pb;
            scratch[4 * wave + 3] = lb;
        }
        __syncthreads();
        pa = la = pb = lb = 0.0;
        for (int w = 0; w < kT / 64; ++w) {
            hz::dd_add(pa, la, scratch[4 * w]);
            hz::dd_add(pa, la, scratch[4 * w + 1]);
            hz::dd_add(pb, lb, scratch[4 * w + 2]);
            hz::dd_add(pb, lb, scratch[4 * w + 3]);
        }
        const double qa = pa / kN, qb = pb / kN;
        const double avga = qa + (fma(-qa, (double)kN, pa) + la) / kN;
        const double avgb = qb + (fma(-qb, (double)kN, pb) + lb) / kN;
        thra = p0 * avga * avga;
        thrb = p0 * avgb * avgb;
    }
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        if (!live[i]) continue;
        double xr = ar[i], xi = ai[i], yr = br[i], yi = bi[i];
        if constexpr (PROC == HZ_PROC_STATIC_GATE) {
            if (xr * xr + xi * xi < thra) {
                xr = xr * p1;
                xi = xi * p1;
            }
            if (yr * yr + yi * yi < thrb) {
                yr = yr * p1;
                yi = yi * p1;
            }
        } else {
            if (!(xr * xr + xi * xi > thra)) xr = xi = 0.0;
            if (!(yr * yr + yi * yi > thrb)) yr = yi = 0.0;
        }
        // Y_k = X_f + i X_{f+1};  Y_{N-k} = conj X_f + i conj X_{f+1}
        zf[ek[i]] = make_double2(xr - yi, xi + yr);
        if (!self[i]) zf[em[i]] = make_double2(xr + yi, yr - xi);
    }
}
}  // namespace p4

template <int PROC, bool ONCE>
__global__ __launch_bounds__(p4::kT) void stft_pair4096_kernel(StftArgs a, long nf) {
#pragma clang fp contract(off)
    using namespace p4;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double2* z = (double2*)lds;
    double* scratch = lds + 2 * kN;
    const int b = threadIdx.x;
    const double2* ptw = a.tw + kH;   // the pass tables
    double2 twA[7], twB[7], twC[7];
#pragma unroll
    for (int r = 0; r < 7; ++r) {
        twA[r] = ptw[kTwA + 512 * r + b];
        twB[r] = ptw[kTwB + 64 * r + (b & 63)];
        twC[r] = ptw[kTwC + 8 * r + (b & 7)];
    }
    const int pl = frame_of_block(blockIdx.x, gridDim.x);   // frame pair within the launch
    const bool two = 2L * pl + 1 < nf;
    long off0, off1 = 0, row0, row1;
    if (a.sh_world <= 1) {   // 32-bit arithmetic from the host's per-launch terms
        const int tl = 2 * a.laps;
        const int j0 = a.i0 + 2 * pl, j1 = j0 + (two ? 1 : 0);
        const int c0 = j0 / tl, c1 = j1 / tl;
        off0 = a.u0 + (long)c0 * (2 * kN - 1) + (long)a.stride * (j0 - c0 * tl);
        off1 = two ? a.u0 + (long)c1 * (2 * kN - 1) + (long)a.stride * (j1 - c1 * tl) : 0;
        row0 = (a.r0 + 2 * pl) % a.R;
        row1 = (a.r0 + 2 * pl + (two ? 1 : 0)) % a.R;
    } else {
        const long f0 = frame_at(a, 2L * pl);
        const long f1 = two ? frame_at(a, 2L * pl + 1) : f0;
        off0 = frame_start(f0, a.laps, a.stride, kN) - a.T0 + (kN - 1);
        off1 = two ? frame_start(f1, a.laps, a.stride, kN) - a.T0 + (kN - 1) : 0;
        row0 = f0 % a.R;
        row1 = f1 % a.R;
    }
    double xr[8], xi[8];
    {   // the first forward pass's group {b + 512 j}: window x real input (fourier.h:110-112)
        double v0[8], v1[8], w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = b + kT * j;
            const long u0 = off0 + k, u1 = off1 + k;   // positions in [history (N-1) | block input]
            v0[j] = u0 < kN - 1 ? a.hr[u0] : a.inr[u0 - (kN - 1)];
            v1[j] = two ? (u1 < kN - 1 ? a.hr[u1] : a.inr[u1 - (kN - 1)]) : 0.0;
            w[j] = a.win[k];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            xr[j] = w[j] * v0[j];
            xi[j] = w[j] * v1[j];
        }
    }
    if constexpr (ONCE) dif8<false>(xr, xi, twA); else dif8s<false>(xr, xi, twA);   // lh 11
    lds_put<512>(z, dif_base<9>(b), xr, xi);
    __syncthreads();
    lds_get<64>(z, dif_base<6>(b), xr, xi);
    if constexpr (ONCE) dif8<false>(xr, xi, twB); else dif8s<false>(xr, xi, twB);   // lh 8
    lds_put<64>(z, dif_base<6>(b), xr, xi);
    wave_sync();
    lds_get<8>(z, dif_base<3>(b), xr, xi);
    if constexpr (ONCE) dif8<false>(xr, xi, twC); else dif8s<false>(xr, xi, twC);   // lh 5
    lds_put<8>(z, dif_base<3>(b), xr, xi);
    wave_sync();
    lds_get<1>(z, dif_base<0>(b), xr, xi);
    if constexpr (ONCE) dif8<true>(xr, xi, twC); else dif8s<true>(xr, xi, twC);   // lh 2
    lds_put<1>(z, dif_base<0>(b), xr, xi);
    __syncthreads();
    gate<PROC>(z, a.p0, a.p1, scratch);
    __syncthreads();
    lds_get<1>(z, dit_base<0>(b), xr, xi);
    if constexpr (ONCE) dit8<true>(xr, xi, twC); else dit8s<true>(xr, xi, twC);   // lh 0
    lds_put<1>(z, dit_base<0>(b), xr, xi);
    wave_sync();
    lds_get<8>(z, dit_base<3>(b), xr, xi);
    if constexpr (ONCE) dit8<false>(xr, xi, twC); else dit8s<false>(xr, xi, twC);   // lh 3
    lds_put<8>(z, dit_base<3>(b), xr, xi);
    wave_sync();
    lds_get<64>(z, dit_base<6>(b), xr, xi);
    if constexpr (ONCE) dit8<false>(xr, xi, twB); else dit8s<false>(xr, xi, twB);   // lh 6
    lds_put<64>(z, dit_base<6>(b), xr, xi);
    __syncthreads();
    lds_get<512>(z, dit_base<9>(b), xr, xi);
    if constexpr (ONCE) dit8<false>(xr, xi, twA); else dit8s<false>(xr, xi, twA);   // lh 9
    // natural order {b + 512 j}: straight to the ring (the Re planes only, as stft_pair_kernel)
    double* o0 = a.fo + row0 * kN;
    double* o1 = a.fo + row1 * kN;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        o0[b + kT * j] = xr[j];
        if (two) o1[b + kT * j] = xi[j];
    }
}

// ---- N = 4096, one real frame per workgroup (StaticSTFT's gate on real input; C4) ------------------
// The frame's 4096 real samples as 2048 complex ones, z[n] = w x[2n] + i w x[2n+1] (fourier.h:110-112
// windowing), so the transform is a 2048-point one on 256 threads (4 waves, 32 KB of LDS): twice the
// workgroups of the pair kernel at half the size, two or more resident per CU, where the pair kernel
// ran one 8-wave workgroup per CU and exposed every pass's barrier and LDS round trip.
//   forward: Z = DFT_M(z), M = N/2; per bin pair (k, M - k): E = (Z_k + conj Z_{M-k}) / 2,
//            O = (Z_k - conj Z_{M-k}) / 2i, t = W_N^k O, X_k = E + t, X_{M-k} = conj(E - t)
//            (bins N - k are conj X_k; bin 0 and M from Z_0, bin M/2 = conj Z_{M/2})
//   gate:    the reference's per-bin test on |X_k|^2 against p0 avg^2 (staticSTFT.h:99-128, or the
//            gate625 callback), avg over all N bins
//   inverse: Z''_k = S + V, Z''_{M-k} = conj(S - V), S = X'_k + conj X'_{M-k}, V = i conj(W_N^k)
//            (X'_k - conj X'_{M-k}); z'' = IDFT_M(Z''), y[2n] + i y[2n+1] = z''[n] (unnormalised, as
//            FFTW's backward transform; the overlap-add divides)
// Pass plan: DIF lh 10-9-8 (stride 256), 7-6-5 (32), 4-3-2 (4), 1-0 (radix 4, contiguous); the
// inverse mirrored. Twiddles W_{8s}^{p r} of a stride-s pass are W_N^{(N/8s) p r} of the N/2 table.
// The layout p4::lx is conflict-free for every pass (scripts/probe/stft_layout_half.py).
namespace h4 {
constexpr int kM = 2048, kLgM = 11, kT = 256, kN = 4096;
inline size_t lds_bytes() { return sizeof(double2) * kM + sizeof(double) * 16; }

// the last forward pass: stages lh 1, 0 on two radix-4 groups of contiguous elements
__device__ __forceinline__ void dif4x2(double (&xr)[8], double (&xi)[8]) {
#pragma unroll
    for (int g = 0; g < 8; g += 4) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {   // h = 2: the difference times W_4^e
            const double ar = xr[g + e], ai = xi[g + e], cr = xr[g + e + 2], ci = xi[g + e + 2];
            const double dr = ar - cr, di = ai - ci;
            xr[g + e] = ar + cr;
            xi[g + e] = ai + ci;
            if (e == 0) {
                xr[g + 2] = dr;
                xi[g + 2] = di;
            } else {   // (dr + i di)(-i)
                xr[g + 3] = di;
                xi[g + 3] = -dr;
            }
        }
#pragma unroll
        for (int e = 0; e < 4; e += 2) {   // h = 1
            const double ar = xr[g + e], ai = xi[g + e], cr = xr[g + e + 1], ci = xi[g + e + 1];
            xr[g + e] = ar + cr;
            xi[g + e] = ai + ci;
            xr[g + e + 1] = ar - cr;
            xi[g + e + 1] = ai - ci;
        }
    }
}

// the first inverse pass: stages lh 0, 1 (DIT: the second input times conj W_4^e)
__device__ __forceinline__ void dit4x2(double (&xr)[8], double (&xi)[8]) {
#pragma unroll
    for (int g = 0; g < 8; g += 4) {
#pragma unroll
        for (int e = 0; e < 4; e += 2) {   // h = 1
            const double ar = xr[g + e], ai = xi[g + e], cr = xr[g + e + 1], ci = xi[g + e + 1];
            xr[g + e] = ar + cr;
            xi[g + e] = ai + ci;
            xr[g + e + 1] = ar - cr;
            xi[g + e + 1] = ai - ci;
        }
#pragma unroll
        for (int e = 0; e < 2; ++e) {   // h = 2
            double cr = xr[g + e + 2], ci = xi[g + e + 2];
            if (e == 1) {   // (cr + i ci) i
                const double t = cr;
                cr = -ci;
                ci = t;
            }
            const double ar = xr[g + e], ai = xi[g + e];
            xr[g + e] = ar + cr;
            xi[g + e] = ai + ci;
            xr[g + e + 2] = ar - cr;
            xi[g + e + 2] = ai - ci;
        }
    }
}

// a stride-s pass's stage twiddles for dif8s / dit8s (entries 0, 1, 3 = W_{8s}^{p}, ^{2p}, ^{4p})
template <int F>   // F = N / (8 s)
__device__ __forceinline__ void pass_tw(const double2* __restrict__ tw, int p, double2 (&t)[7]) {
    t[0] = tw[F * p];
    t[1] = tw[2 * F * p];
    t[3] = tw[4 * F * p];
    t[2] = t[4] = t[5] = t[6] = make_double2(1.0, 0.0);
}

// split, gate and merge over spectrum positions (p4::gate's walk at lg = 11)
template <int PROC>
__device__ __forceinline__ void gate(double2* zf, const double2* __restrict__ tw, double p0, double p1,
                                     double* scratch) {
#pragma clang fp contract(off)
    constexpr int kItems = 5;   // 1023 pairs, then u = 1023 (bins 0 and M) and u = 1024 (bin M/2)
    const int b = threadIdx.x;
    double er[kItems], ei[kItems], tr[kItems], ti[kItems], wr[kItems], wi[kItems];
    int ek[kItems], em[kItems], kind[kItems];   // kind 0 pair, 1 bins 0 / M, 2 bin M/2, 3 none
    double pa = 0.0, la = 0.0;
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        const int u = b + kT * i;
        kind[i] = u < kM / 2 - 1 ? 0 : u == kM / 2 - 1 ? 1 : u == kM / 2 ? 2 : 3;
        er[i] = ei[i] = tr[i] = ti[i] = wr[i] = wi[i] = 0.0;
        ek[i] = em[i] = 0;
        if (kind[i] == 3) continue;
        double xa_r, xa_i, xb_r = 0.0, xb_i = 0.0, ca, cb;   // the item's bins and their counts
        if (kind[i] == 0) {
            const int q = (u + 1) + p4::hibit(u + 1), qq = q ^ (p4::hibit(q) - 1);
            const int kq = hz::bitrev(q, kLgM), kqq = hz::bitrev(qq, kLgM);
            const int k = kq < kqq ? kq : kqq;
            ek[i] = p4::lx(kq < kqq ? q : qq);
            em[i] = p4::lx(kq < kqq ? qq : q);
            const double2 zk = zf[ek[i]], zm = zf[em[i]], w = tw[k];
            wr[i] = w.x;
            wi[i] = w.y;
            er[i] = (zk.x + zm.x) * 0.5;
            ei[i] = (zk.y - zm.y) * 0.5;
            const double orr = (zk.y + zm.y) * 0.5, oi = (zm.x - zk.x) * 0.5;
            tr[i] = w.x * orr - w.y * oi;   // t = W^k O
            ti[i] = w.x * oi + w.y * orr;
            xa_r = er[i] + tr[i];   // X_k
            xa_i = ei[i] + ti[i];
            xb_r = er[i] - tr[i];   // X_{M-k} = conj(E - t)
            xb_i = -(ei[i] - ti[i]);
            ca = cb = 2.0;
        } else if (kind[i] == 1) {
            ek[i] = p4::lx(0);
            const double2 z0 = zf[ek[i]];
            er[i] = z0.x;   // E_0, O_0
            tr[i] = z0.y;
            xa_r = z0.x + z0.y;   // X_0
            xa_i = 0.0;
            xb_r = z0.x - z0.y;   // X_M
            ca = cb = 1.0;
        } else {
            ek[i] = p4::lx(1);
            const double2 zh = zf[ek[i]];
            xa_r = zh.x;   // X_{M/2} = conj Z_{M/2}
            xa_i = -zh.y;
            ca = 2.0;
            cb = 0.0;
        }
        er[i] = kind[i] == 0 ? er[i] : xa_r;   // kinds 1, 2 keep the bins themselves
        ei[i] = kind[i] == 0 ? ei[i] : xa_i;
        tr[i] = kind[i] == 0 ? tr[i] : xb_r;
        ti[i] = kind[i] == 0 ? ti[i] : xb_i;
        if constexpr (PROC == HZ_PROC_STATIC_GATE) {
            pa += ca * (sqrt(xa_r * xa_r + xa_i * xa_i) / kN);
            if (cb != 0.0) pa += cb * (sqrt(xb_r * xb_r + xb_i * xb_i) / kN);
        } else {
            const double ha = hypot(xa_r, xa_i), hb = hypot(xb_r, xb_i);
            hz::dd_add(pa, la, ha);
            if (ca == 2.0) hz::dd_add(pa, la, ha);
            if (cb != 0.0) hz::dd_add(pa, la, hb);
            if (cb == 2.0) hz::dd_add(pa, la, hb);
        }
    }
    double thr;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if constexpr (PROC == HZ_PROC_STATIC_GATE) {   // staticSTFT.h:99-128
        for (int o = 32; o > 0; o >>= 1) pa += __shfl_xor(pa, o, 64);
        if (lane == 0) scratch[wave] = pa;
        __syncthreads();
        double avg = 0.0;
        for (int w = 0; w < kT / 64; ++w) avg += scratch[w];
        thr = p0 * avg * avg;
    } else {   // tests/spectral.cpp:32-72 (sum / N in long double)
        for (int o = 32; o > 0; o >>= 1) {
            const double ah = __shfl_xor(pa, o, 64), al = __shfl_xor(la, o, 64);
            hz::dd_add(pa, la, ah);
            hz::dd_add(pa, la, al);
        }
        if (lane == 0) {
            scratch[2 * wave] = pa;
            scratch[2 * wave + 1] = la;
        }
        __syncthreads();
        pa = la = 0.0;
        for (int w = 0; w < kT / 64; ++w) {
            hz::dd_add(pa, la, scratch[2 * w]);
            hz::dd_add(pa, la, scratch[2 * w + 1]);
        }
        const double qa = pa / kN;
        const double avg = qa + (fma(-qa, (double)kN, pa) + la) / kN;
        thr = p0 * avg * avg;
    }
    auto gated = [&](double& xr, double& xi) {
        if constexpr (PROC == HZ_PROC_STATIC_GATE) {
            if (xr * xr + xi * xi < thr) {
                xr = xr * p1;
                xi = xi * p1;
            }
        } else {
            if (!(xr * xr + xi * xi > thr)) xr = xi = 0.0;
        }
    };
#pragma unroll
    for (int i = 0; i < kItems; ++i) {
        if (kind[i] == 3) continue;
        if (kind[i] == 0) {
            double ar = er[i] + tr[i], ai = ei[i] + ti[i];      // X_k
            double br = er[i] - tr[i], bi = -(ei[i] - ti[i]);   // X_{M-k}
            gated(ar, ai);
            gated(br, bi);
            // S = X'_k + conj X'_{M-k}, D = X'_k - conj X'_{M-k}, V = i conj(W^k) D
            const double sr = ar + br, si = ai - bi, dr = ar - br, di = ai + bi;
            const double cr = wr[i] * dr + wi[i] * di, ci = wr[i] * di - wi[i] * dr;   // conj(W^k) D
            const double vr = -ci, vi = cr;
            zf[ek[i]] = make_double2(sr + vr, si + vi);
            zf[em[i]] = make_double2(sr - vr, -(si - vi));
        } else if (kind[i] == 1) {
            double ar = er[i], ai = 0.0, br = tr[i], bi = 0.0;
            gated(ar, ai);
            gated(br, bi);
            zf[ek[i]] = make_double2(ar + br, ar - br);
        } else {
            double ar = er[i], ai = ei[i];
            gated(ar, ai);
            zf[ek[i]] = make_double2(2.0 * ar, -2.0 * ai);
        }
    }
}
}  // namespace h4

template <int PROC>
__global__ __launch_bounds__(h4::kT) void stft_half4096_kernel(StftArgs a, long nf) {
#pragma clang fp contract(off)
    using namespace h4;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double2* z = (double2*)lds;
    double* scratch = lds + 2 * kM;
    const int b = threadIdx.x;
    double2 twA[7], twB[7], twC[7];
    pass_tw<2>(a.tw, b, twA);          // stride 256
    pass_tw<16>(a.tw, b & 31, twB);    // stride 32
    pass_tw<128>(a.tw, b & 3, twC);    // stride 4
    const int fl = frame_of_block(blockIdx.x, gridDim.x);
    long off, row;
    if (a.sh_world <= 1) {
        const int tl = 2 * a.laps;
        const int j0 = a.i0 + fl;
        const int c0 = j0 / tl;
        off = a.u0 + (long)c0 * (2 * kN - 1) + (long)a.stride * (j0 - c0 * tl);
        row = (a.r0 + fl) % a.R;
    } else {
        const long f = frame_at(a, fl);
        off = frame_start(f, a.laps, a.stride, kN) - a.T0 + (kN - 1);
        row = f % a.R;
    }
    (void)nf;
    double xr[8], xi[8];
    {   // z[n] = w x[2n] + i w x[2n+1], n = b + 256 j (fourier.h:110-112)
        double v0[8], v1[8];
        double2 w[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int n = b + kT * j;
            const long u = off + 2 * n;   // position in [history (N-1) | block input]
            v0[j] = u < kN - 1 ? a.hr[u] : a.inr[u - (kN - 1)];
            v1[j] = u + 1 < kN - 1 ? a.hr[u + 1] : a.inr[u + 1 - (kN - 1)];
            w[j] = ((const double2*)a.win)[n];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            xr[j] = w[j].x * v0[j];
            xi[j] = w[j].y * v1[j];
        }
    }
    p4::dif8s<false>(xr, xi, twA);   // lh 10, 9, 8
    p4::lds_put<256>(z, b, xr, xi);
    __syncthreads();
    p4::lds_get<32>(z, p4::dif_base<5>(b), xr, xi);
    p4::dif8s<false>(xr, xi, twB);   // lh 7, 6, 5
    p4::lds_put<32>(z, p4::dif_base<5>(b), xr, xi);
    p4::wave_sync();
    p4::lds_get<4>(z, p4::dif_base<2>(b), xr, xi);
    p4::dif8s<false>(xr, xi, twC);   // lh 4, 3, 2
    p4::lds_put<4>(z, p4::dif_base<2>(b), xr, xi);
    p4::wave_sync();
    p4::lds_get<1>(z, 8 * b, xr, xi);
    dif4x2(xr, xi);                  // lh 1, 0
    p4::lds_put<1>(z, 8 * b, xr, xi);
    __syncthreads();
    gate<PROC>(z, a.tw, a.p0, a.p1, scratch);
    __syncthreads();
    p4::lds_get<1>(z, 8 * b, xr, xi);
    dit4x2(xr, xi);                  // lh 0, 1
    p4::lds_put<1>(z, 8 * b, xr, xi);
    p4::wave_sync();
    p4::lds_get<4>(z, p4::dit_base<2>(b), xr, xi);
    p4::dit8s<false>(xr, xi, twC);   // lh 2, 3, 4
    p4::lds_put<4>(z, p4::dit_base<2>(b), xr, xi);
    p4::wave_sync();
    p4::lds_get<32>(z, p4::dit_base<5>(b), xr, xi);
    p4::dit8s<false>(xr, xi, twB);   // lh 5, 6, 7
    p4::lds_put<32>(z, p4::dit_base<5>(b), xr, xi);
    __syncthreads();
    p4::lds_get<256>(z, b, xr, xi);
    p4::dit8s<false>(xr, xi, twA);   // lh 8, 9, 10
    // natural order z''[b + 256 j] = y[2n] + i y[2n + 1]: straight to the ring's Re plane
    double2* o = (double2*)(a.fo + row * kN);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[b + kT * j] = make_double2(xr[j], xi[j]);
}

struct OlaArgs {
    const double* fo;   // planar ring (Re plane, then Im plane of R*N)
    const double* win;
    double* out_re;
    double* out_im;
    long T0, n;
    int N, laps, stride, R;
    // history carry for the next block (folded in to save a launch): the last N-1 samples of
    // [history (N-1) | block input (n)] from hist_old / in_re / in_im into hist_new
    const double* hist_old;
    const double* in_re;
    const double* in_im;
    double* hist_new;
    // time-range shards (hz_stft_set_frame_shard): frame f is this handle's iff
    // (f / sh_block) % sh_world == sh_rank; the others contribute nothing
    long sh_block;
    int sh_world, sh_rank;
    double sh_inv;   // 1 / sh_block
    long im_zero_from;   // frames from here on: Im part 0, not in the ring (hz_stft::im_zero_from)
    // stft_ola_seg_kernel: the launch's first period and its first ring row, (c_first 2 laps) mod R
    long c_first;
    int row_first;
};

__device__ __forceinline__ bool frame_owned(long f, long block, int world, int rank, double inv) {
    if (world <= 1) return true;
    long q = (long)((double)f * inv);   // f / block without a 64-bit divide (exact after the fix)
    if (q * block > f) --q;
    else if ((q + 1) * block <= f) ++q;
    return (int)(q % world) == rank;
}

__global__ __launch_bounds__(256) void stft_ola_kernel(OlaArgs a) {
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < a.N - 1) {
        const int N1 = a.N - 1;
        const long s = j + a.n;
        if (s < N1) {
            a.hist_new[j] = a.hist_old[s];
            a.hist_new[N1 + j] = a.hist_old[N1 + s];
        } else {
            a.hist_new[j] = a.in_re[s - N1];
            a.hist_new[N1 + j] = a.in_im ? a.in_im[s - N1] : 0.0;
        }
    }
    if (j >= a.n) return;
    const long t = a.T0 + j;
    const long P = 2L * a.N - 1;
    const long u0 = t - (a.N - 1);
    double rh = 0.0, rl = 0.0, ih = 0.0, il = 0.0;
    if (u0 >= 0) {
        // u0 = c P + r without a 64-bit divide: double quotient, then one correction step
        long c = (long)((double)u0 / (double)P);
        long r = u0 - c * P;
        if (r < 0) {
            r += P;
            --c;
        } else if (r >= P) {
            r -= P;
            ++c;
        }
        // ring row of frame f = c 2 laps + i is (f mod R); track (c 2 laps) mod R incrementally
        const long cf = c * 2 * a.laps;
        int base = (int)(cf - (long)((double)cf / (double)a.R) * a.R);
        if (base < 0) base += a.R;
        if (base >= a.R) base -= a.R;
        const long plane = (long)a.R * a.N;
        for (int i = 0; i < 2 * a.laps; ++i) {   // fourier.h:153-172, slot order
            if (i) {
                r -= a.stride;
                if (r < 0) {   // stride < P: at most one wrap per slot
                    r += P;
                    --c;
                    base -= 2 * a.laps;
                    if (base < 0) base += a.R;
                }
            }
            if (c < 0) break;
            if (r >= a.N) continue;
            if (!frame_owned(c * 2 * a.laps + i, a.sh_block, a.sh_world, a.sh_rank, a.sh_inv)) continue;
            int row = base + i;
            if (row >= a.R) row -= a.R;
            const long q = (long)row * a.N + r;
            const double w = a.win[r];
            hz::dd_add(rh, rl, w * a.fo[q]);
            if (a.out_im && c * 2 * a.laps + i < a.im_zero_from) hz::dd_add(ih, il, w * a.fo[plane + q]);
        }
    }
    const double D = (double)(a.N * a.laps / 2);   // int expression, fourier.h:174-175
    double q = rh / D;
    q += (fma(-q, D, rh) + rl) / D;
    a.out_re[j] = q;
    if (a.out_im) {
        double qi = ih / D;
        qi += (fma(-qi, D, ih) + il) / D;
        a.out_im[j] = qi;
    }
}

// Overlap-add by segments (fourier.h:153-172, LAPS-specialised). In period c (2N - 1 positions,
// 2 LAPS slots) the positions r in segment k = [stride k, stride (k + 1)) all read the same slots:
// slot i <= k from this period's frame at offset r - stride i (live iff k - i < LAPS), slot i > k
// from the previous period's frame at r + P - stride i (live iff i > k + LAPS, and i = k + LAPS at
// r = stride k only). So a workgroup owns one segment: the slot list (rows, offsets, shard and Im
// flags) is decided once, and each thread issues all its samples' loads before the dd sums, which
// run in the reference's slot order (ascending i). The last N - 1 inputs are carried into the
// next call's history by the first `aux` workgroups, which also write the zeros before the first
// frame completes.
template <int LAPS, int SPLIT>   // SPLIT workgroups per segment
__global__ __launch_bounds__(256) void stft_ola_seg_kernel(OlaArgs a, long g0, long u_lo, long u_hi, int aux) {
    constexpr int S = 2 * LAPS;
    constexpr int SPT = 16 / LAPS / SPLIT > 0 ? 16 / LAPS / SPLIT : 1;   // samples per thread per round
    const int N = a.N, stride = a.stride;
    const long P = 2L * N - 1;
    const long tb = (long)blockIdx.x;
    if (tb < aux) {
        const int N1 = N - 1;
        const long zp = a.T0 < N1 ? std::min((long)N1, a.T0 + a.n) - a.T0 : 0;   // outputs before any frame
        for (long j = tb * 256 + threadIdx.x; j < std::max((long)N1, zp); j += (long)aux * 256) {
            if (j < N1) {
                const long s = j + a.n;
                if (s < N1) {
                    a.hist_new[j] = a.hist_old[s];
                    a.hist_new[N1 + j] = a.hist_old[N1 + s];
                } else {
                    a.hist_new[j] = a.in_re[s - N1];
                    a.hist_new[N1 + j] = a.in_im ? a.in_im[s - N1] : 0.0;
                }
            }
            if (j < zp) {
                a.out_re[j] = 0.0;
                if (a.out_im) a.out_im[j] = 0.0;
            }
        }
        return;
    }
    const long g = g0 + (tb - aux) / SPLIT;
    const int part = (int)((tb - aux) % SPLIT);
    const long c = g / S;
    const int k = (int)(g - c * S);
    const long ubase = c * P + (long)stride * k;   // position of the segment's first sample
    const int seglen = (int)std::min((long)stride, P - (long)stride * k);
    const int piece = stride / SPLIT;
    const int j_lo = (int)std::max((long)part * piece, u_lo - ubase);
    const int j_hi = (int)std::min((long)(part == SPLIT - 1 ? seglen : (part + 1) * piece), u_hi - ubase + 1);
    // the LAPS live slots for r > stride k, ascending: this period's i = k - ncur + 1 .. k, then the
    // previous period's i = k + LAPS + 1 .. S - 1. Ring rows in 32 bits from the launch's first
    // period (row_first = (c_first S) mod R on the host; a launch spans < 2^20 / P periods), so no
    // 64-bit divide runs on the device
    const int ncur = k < LAPS - 1 ? k + 1 : LAPS;
    const unsigned R = (unsigned)a.R;
    const unsigned cur0 = ((unsigned)a.row_first + (unsigned)(c - a.c_first) * S) % R;
    const unsigned prv0 = cur0 >= (unsigned)S ? cur0 - S : cur0 + R - S;
    const unsigned plane = R * (unsigned)N;
    unsigned roff[LAPS];
    int dl[LAPS];
    bool live[LAPS], imv[LAPS];
#pragma unroll
    for (int m = 0; m < LAPS; ++m) {
        const bool cur = m < ncur;
        const int i = cur ? k - ncur + 1 + m : k + LAPS + 1 + (m - ncur);
        const long f = cur ? c * S + i : (c - 1) * S + i;
        unsigned row = (cur ? cur0 : prv0) + i;
        if (row >= R) row -= R;
        roff[m] = row * (unsigned)N;
        dl[m] = cur ? stride * (k - i) : (int)(P - (long)stride * (i - k));
        live[m] = (cur || c > 0) && frame_owned(f, a.sh_block, a.sh_world, a.sh_rank, a.sh_inv);
        imv[m] = a.out_im != nullptr && f < a.im_zero_from;
    }
    // D = N LAPS / 2 (an int expression, fourier.h:174-175) is a power of two (N = 2^lg): the
    // quotients below are the products by 1 / D, bit for bit
    const double D = (double)(N * LAPS / 2), invD = 1.0 / D;
    const long o0 = ubase + (N - 1) - a.T0;   // output index of the segment's first sample
    double* __restrict__ ore = a.out_re + o0;
    double* __restrict__ oim = a.out_im ? a.out_im + o0 : nullptr;
    const double* __restrict__ fo = a.fo;
    const double* __restrict__ win = a.win;
    for (int jb = j_lo + (int)threadIdx.x; jb < j_hi; jb += 256 * SPT) {
        double fr[SPT][LAPS], fi[SPT][LAPS], w[SPT][LAPS];
#pragma unroll
        for (int s = 0; s < SPT; ++s) {
            const int j = jb + 256 * s;
#pragma unroll
            for (int m = 0; m < LAPS; ++m) {
                const bool ok = live[m] && j < j_hi;
                const unsigned q = (unsigned)(j + dl[m]);
                w[s][m] = ok ? win[q] : 0.0;
                fr[s][m] = ok ? fo[roff[m] + q] : 0.0;
                fi[s][m] = ok && imv[m] ? fo[plane + roff[m] + q] : 0.0;
            }
        }
#pragma unroll
        for (int s = 0; s < SPT; ++s) {
            const int j = jb + 256 * s;
            if (j >= j_hi) break;
            double rh = 0.0, rl = 0.0, ih = 0.0, il = 0.0;
#pragma unroll
            for (int m = 0; m <= LAPS; ++m) {
                if (j == 0 && m == ncur && k + LAPS < S && c > 0) {
                    // r = stride k: the previous period's slot k + LAPS at offset N - 1 comes first
                    const int i = k + LAPS;
                    const long f = (c - 1) * S + i;
                    if (frame_owned(f, a.sh_block, a.sh_world, a.sh_rank, a.sh_inv)) {
                        unsigned row = prv0 + i;
                        if (row >= R) row -= R;
                        const double wv = win[N - 1];
                        hz::dd_add(rh, rl, wv * fo[row * (unsigned)N + (N - 1)]);
                        if (a.out_im && f < a.im_zero_from) hz::dd_add(ih, il, wv * fo[plane + row * (unsigned)N + (N - 1)]);
                    }
                }
                if (m < LAPS && live[m]) {
                    hz::dd_add(rh, rl, w[s][m] * fr[s][m]);
                    if (imv[m]) hz::dd_add(ih, il, w[s][m] * fi[s][m]);
                }
            }
            double q = rh * invD;
            q += (fma(-q, D, rh) + rl) * invD;
            ore[j] = q;
            if (oim) {
                double qi = ih * invD;
                qi += (fma(-qi, D, ih) + il) * invD;
                oim[j] = qi;
            }
        }
    }
}

// ---- Cosine: REDFT10 / REDFT01 via a length-N complex FFT (one workgroup per transform)
__global__ __launch_bounds__(kThreads) void dct2_kernel(const double* __restrict__ x, double* __restrict__ y, int N,
                                                        int lg, const double2* __restrict__ tw,
                                                        const double2* __restrict__ rot) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + N;
    const double* xb = x + (long)blockIdx.x * N;
    double* yb = y + (long)blockIdx.x * N;
    for (int k = threadIdx.x; k < N / 2; k += blockDim.x) {   // v[k] = x[2k], v[N-1-k] = x[2k+1]
        re[k] = xb[2 * k];
        re[N - 1 - k] = xb[2 * k + 1];
        im[k] = 0.0;
        im[N - 1 - k] = 0.0;
    }
    __syncthreads();
    hz::lds_fft_fwd(re, im, N, lg, tw);
    for (int p = threadIdx.x; p < N; p += blockDim.x) {   // Y_k = 2 Re(V_k e^{-i pi k/2N})
        const int k = hz::bitrev(p, lg);
        const double2 w = rot[k];
        yb[k] = 2.0 * (re[p] * w.x - im[p] * w.y);
    }
}

__global__ __launch_bounds__(kThreads) void dct3_kernel(const double* __restrict__ x, double* __restrict__ y, int N,
                                                        int lg, const double2* __restrict__ tw,
                                                        const double2* __restrict__ rot) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + N;
    const double* xb = x + (long)blockIdx.x * N;
    double* yb = y + (long)blockIdx.x * N;
    for (int p = threadIdx.x; p < N; p += blockDim.x) {   // V_j = e^{i pi j/2N} (x_j - i x_{N-j})
        const int j = hz::bitrev(p, lg);
        const double a = xb[j], b = j ? xb[N - j] : 0.0;
        const double2 w = rot[j];   // e^{-i pi j / 2N}; use its conjugate
        re[p] = a * w.x + b * (-w.y);
        im[p] = -a * w.y - b * w.x;
    }
    __syncthreads();
    hz::lds_fft_inv(re, im, N, lg, tw);
    for (int k = threadIdx.x; k < N / 2; k += blockDim.x) {
        yb[2 * k] = re[k];
        yb[2 * k + 1] = re[N - 1 - k];
    }
}

int ilog2(int N) {
    int lg = 0;
    while ((1 << lg) < N) ++lg;
    return lg;
}

bool pow2(int N) { return N >= 4 && (N & (N - 1)) == 0; }
// ---- per-sample slot mode (hz_stft_write / read / forward / backward / process_slot) ----------
// The reference's own state machine runs on the host (fourier.h:102-177: O(2 laps) bookkeeping
// per sample); the transforms and device processors of a completed slot run here, one
// workgroup per N-point transform, natural order in and out (FFTW's dft_1d convention,
// unnormalised): forward = the frame kernel's passes, then the bit-reversal on the way out;
// inverse = the bit-reversal on the way in, then the inverse passes.
template <int RMAX, bool INV>
__global__ __launch_bounds__(kFrameThreads) void slot_fft_kernel(const double2* __restrict__ src, double2* __restrict__ dst,
                                                                int N, int lg, const double2* __restrict__ tw) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + hz::padded_len(N);
    double2* T = (double2*)(im + hz::padded_len(N) + 2 * (blockDim.x >> 6));
    for (int k = threadIdx.x; k < hz::twc_len(lg); k += blockDim.x) T[k] = tw[k];
    for (int p = threadIdx.x; p < N; p += blockDim.x) {
        const double2 v = src[INV ? hz::bitrev(p, lg) : p];
        re[hz::pad16(p)] = v.x;
        im[hz::pad16(p)] = v.y;
    }
    __syncthreads();
    if constexpr (INV) hz::fft_inv_tail<RMAX>(re, im, lg, T, true);
    else hz::fft_fwd_lead<RMAX>(re, im, lg, T, true);
    for (int p = threadIdx.x; p < N; p += blockDim.x) {
        const int e = hz::pad16(p);
        dst[INV ? p : hz::bitrev(p, lg)] = make_double2(re[e], im[e]);
    }
}

// a device processor on one natural-order spectrum: in -> out (out is the slot's persistent
// output buffer: the gates write every bin of it, as the reference's processors do)
template <int PROC>
__global__ __launch_bounds__(kFrameThreads) void slot_proc_kernel(const double2* __restrict__ in, double2* __restrict__ out,
                                                                  int N, double p0, double p1) {
#pragma clang fp contract(off)
    __shared__ double scratch[2 * (kFrameThreads / 64)];
    if constexpr (PROC == HZ_PROC_STATIC_GATE) {   // staticSTFT.h:99-128
        const double inv_n = 1.0 / N;
        double part = 0.0;
        for (int k = threadIdx.x; k < N; k += blockDim.x) part += sqrt(in[k].x * in[k].x + in[k].y * in[k].y) * inv_n;
        const double average = block_sum(part, scratch);
        const double thr = p0 * average * average;
        for (int k = threadIdx.x; k < N; k += blockDim.x) {
            const double2 v = in[k];
            out[k] = v.x * v.x + v.y * v.y < thr ? make_double2(v.x * p1, v.y * p1) : v;
        }
    } else if constexpr (PROC == HZ_PROC_GATE_KEEP) {   // tests/spectral.cpp:32-72
        double hi = 0.0, lo = 0.0;
        for (int k = threadIdx.x; k < N; k += blockDim.x) hz::dd_add(hi, lo, hypot(in[k].x, in[k].y));
        block_sum_dd(hi, lo, scratch);
        const double q = hi / N;
        const double avg = q + (fma(-q, (double)N, hi) + lo) / N;
        const double thr = p0 * avg * avg;
        for (int k = threadIdx.x; k < N; k += blockDim.x) {
            const double2 v = in[k];
            out[k] = v.x * v.x + v.y * v.y > thr ? v : make_double2(0.0, 0.0);
        }
    } else if constexpr (PROC == HZ_PROC_HILBERT) {   // tests/SFML/hilbert.cpp:37-49: bins k < N/2
        for (int k = threadIdx.x; k < N; k += blockDim.x) out[k] = k < N / 2 ? in[k] : make_double2(0.0, 0.0);
    } else {
        for (int k = threadIdx.x; k < N; k += blockDim.x) out[k] = in[k];
    }
}



std::vector<double2> twiddles(int N) {
    std::vector<double2> tw(N / 2);
    const long double pi = acosl(-1.0L);
    for (int k = 0; k < N / 2; ++k) {
        const long double a = -2.0L * pi * k / N;
        tw[k] = make_double2((double)cosl(a), (double)sinl(a));
    }
    return tw;
}

}  // namespace

struct hz_stft {
    int N = 0, laps = 0, stride = 0, lg = 0, window = 0, proc = 0, device = 0, R = 0;
    double p0 = 0, p1 = 0;
    hz_stft_proc host_proc = nullptr;
    long T = 0;        // samples processed
    long frames = 0;   // frames completed
    double* d_win = nullptr;
    double2 *d_tw = nullptr, *d_spec = nullptr;
    double* d_fo = nullptr;                    // planar frame ring: Re [R][N], Im [R][N]
    double* d_hist[2] = {nullptr, nullptr};    // last N-1 input samples, [Re | Im] (ping-pong)
    long last_cplx = -1;                       // last sample index that came with an imaginary part
    // frames >= im_zero_from came from the pair kernel, whose Im plane (all zeros) is not written:
    // the overlap-add reads no Im part for them (LONG_MAX: none since the last other launch)
    long im_zero_from = LONG_MAX;
    int hcur = 0;
    size_t spec_cap = 0;
    double *d_in = nullptr, *d_out = nullptr;
    size_t io_cap = 0;
    std::vector<double2> h_spec, h_out;   // host-processor path: spectra + per-slot out buffers
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool prof = false;
    long chunk = 0;        // samples per internal block (a frame launch covers one)
    int prof_repeat = 1;   // frame launches per block while profiling (hz_stft_profile)
    bool pair_ok = true;   // two real frames per transform (stft_pair_kernel)
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    long launches = 0;
    // time-range shards: frame f is computed here iff (f / sh_block) % sh_world == sh_rank
    long sh_block = 1;
    int sh_world = 1, sh_rank = 0;
    // per-sample slot mode (fourier.h:102-177 on the host, transforms on the device): the
    // reference's in / middle / out slot buffers [2 laps][N] and its read / write heads
    bool slot_mode = false;
    std::vector<double2> s_in, s_mid, s_out;
    std::vector<int> s_wp, s_rp;
    std::vector<char> s_reading, s_writing;
    std::vector<double> h_win;
    double2* d_slot = nullptr;   // [2][N] device scratch
};

namespace {

int stft_check(hz_stft* h) {
    if (!h) {
        hz::set_error("null hz_stft handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    return HZ_OK;
}

// number of frames with completion time e_f = s_f + N - 1 < T
long frames_before(const hz_stft* h, long T) {
    const long P = 2L * h->N - 1;
    long cnt = 0;
    for (int i = 0; i < 2 * h->laps; ++i) {
        const long lim = T - (h->N - 1) - (long)h->stride * i;   // c*P < lim
        if (lim > 0) cnt += (lim + P - 1) / P;
    }
    return cnt;
}

template <int PROC, int MODE>
void frame_attr(int lds) {
    (void)hipFuncSetAttribute((const void*)stft_frame_kernel<PROC, MODE, 3>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)stft_frame_kernel<PROC, MODE, 4>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

template <int PROC, int MODE>
void launch_frames(hz_stft* h, const StftArgs& a, long nf) {
    if (frame_rmax(h->N) == 3)
        hipLaunchKernelGGL((stft_frame_kernel<PROC, MODE, 3>), dim3((unsigned)nf), dim3(frame_threads(h->N)),
                           frame_lds(h->N), h->stream, a);
    else
        hipLaunchKernelGGL((stft_frame_kernel<PROC, MODE, 4>), dim3((unsigned)nf), dim3(frame_threads(h->N)),
                           frame_lds(h->N), h->stream, a);
}

template <int PROC>
void launch_pairs(hz_stft* h, const StftArgs& a, long nf) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)stft_pair_kernel<PROC, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)frame_lds(kMaxN));
        (void)hipFuncSetAttribute((const void*)stft_pair_kernel<PROC, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)frame_lds(kMaxN));
        attr = true;
    }
    static const bool generic = std::getenv("HZ_STFT_GENERIC_PAIR") != nullptr;   // (A/B measurements)
    // twiddles once per element (7 products per group and pass) measured slower on one box than the
    // stage-wise form (12): 15.1 vs 14.6 us per C4 step, alternating runs (profiles/r4/rows/c4/ab.log);
    // HZ_STFT_TWIDDLE_ONCE=1 selects it for such A/B runs
    static const bool stagewise = std::getenv("HZ_STFT_TWIDDLE_ONCE") == nullptr;
    // HZ_STFT_FRAME=half: one frame per workgroup (2048-point even/odd transform); pair (default):
    // two frames per 4096-point transform -- for A/B runs
    static const bool pair4096 = [] {
        const char* v = std::getenv("HZ_STFT_FRAME");
        return !(v && std::strcmp(v, "half") == 0);
    }();
    if (h->N == h4::kN && !generic && !pair4096) {
        hipLaunchKernelGGL((stft_half4096_kernel<PROC>), dim3((unsigned)nf), dim3(h4::kT), h4::lds_bytes(),
                           h->stream, a, nf);
    } else if (h->N == p4::kN && !generic) {
        static bool attr4 = false;
        if (!attr4) {
            for (const void* k : {(const void*)stft_pair4096_kernel<PROC, true>, (const void*)stft_pair4096_kernel<PROC, false>})
                (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)p4::lds_bytes());
            attr4 = true;
        }
        if (stagewise)
            hipLaunchKernelGGL((stft_pair4096_kernel<PROC, false>), dim3((unsigned)((nf + 1) / 2)), dim3(p4::kT),
                               p4::lds_bytes(), h->stream, a, nf);
        else
            hipLaunchKernelGGL((stft_pair4096_kernel<PROC, true>), dim3((unsigned)((nf + 1) / 2)), dim3(p4::kT),
                               p4::lds_bytes(), h->stream, a, nf);
    } else if (frame_rmax(h->N) == 3)
        hipLaunchKernelGGL((stft_pair_kernel<PROC, 3>), dim3((unsigned)((nf + 1) / 2)), dim3(frame_threads(h->N)),
                           frame_lds(h->N), h->stream, a, nf);
    else
        hipLaunchKernelGGL((stft_pair_kernel<PROC, 4>), dim3((unsigned)((nf + 1) / 2)), dim3(frame_threads(h->N)),
                           frame_lds(h->N), h->stream, a, nf);
}

// real input and a magnitude gate: two frames per transform (stft_pair_kernel)
bool pair_launch(const hz_stft* h, const StftArgs& a) {
    return h->pair_ok && !a.hi && h->N >= 16 && (h->proc == HZ_PROC_STATIC_GATE || h->proc == HZ_PROC_GATE_KEEP);
}

int frames_fused(hz_stft* h, const StftArgs& a, long nf) {
    if (pair_launch(h, a)) {
        if (h->proc == HZ_PROC_STATIC_GATE) launch_pairs<HZ_PROC_STATIC_GATE>(h, a, nf);
        else launch_pairs<HZ_PROC_GATE_KEEP>(h, a, nf);
        HZ_TRY_HIP(hipGetLastError());
        return HZ_OK;
    }
    switch (h->proc) {
    case HZ_PROC_STATIC_GATE: launch_frames<HZ_PROC_STATIC_GATE, 0>(h, a, nf); break;
    case HZ_PROC_GATE_KEEP: launch_frames<HZ_PROC_GATE_KEEP, 0>(h, a, nf); break;
    case HZ_PROC_HILBERT: launch_frames<HZ_PROC_HILBERT, 0>(h, a, nf); break;
    default: launch_frames<HZ_PROC_IDENTITY, 0>(h, a, nf); break;
    }
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

int ensure_dev(void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return HZ_OK;
    if (*p) HZ_TRY_HIP(hipFree(*p));
    *p = nullptr;
    HZ_TRY_HIP(hipMalloc(p, bytes));
    *cap = bytes;
    return HZ_OK;
}

int stft_block(hz_stft* h, const double* d_re, const double* d_im, double* d_ore, double* d_oim, long n) {
    const int N = h->N;
    double* hc = h->d_hist[h->hcur];
    double* hn = h->d_hist[h->hcur ^ 1];
    if (d_im) h->last_cplx = h->T + n - 1;

    hipEvent_t* e = nullptr;
    if (h->prof) {
        if (h->ev_used + 3 > h->ev.size())
            for (int q = 0; q < 96; ++q) {
                hipEvent_t ne;
                HZ_TRY_HIP(hz::prof_event_create(&ne));
                h->ev.push_back(ne);
            }
        e = &h->ev[h->ev_used];
        h->ev_used += 3;
        HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
    }
    const long f_first = frames_before(h, h->T), f_done = frames_before(h, h->T + n);
    StftArgs a;
    a.hr = hc;
    a.hi = nullptr;
    a.inr = d_re;
    a.ini = d_im;
    a.fo = h->d_fo;
    a.spec = h->d_spec;
    a.win = h->d_win;
    a.tw = h->d_tw;
    a.T0 = h->T;
    a.N = N;
    a.lg = h->lg;
    a.laps = h->laps;
    a.stride = h->stride;
    a.R = h->R;
    a.p0 = h->p0;
    a.p1 = h->p1;
    // time-range shards: this handle's frames of the block, as one launch (frame_at maps the
    // launch's frames onto its runs); unsharded: the whole block
    long f_lo = f_first, nf = f_done - f_first;
    a.sh_world = h->sh_world;
    a.sh_block = h->sh_block;
    a.sh_q0 = 0;
    a.sh_off = 0;
    if (h->sh_world > 1 && nf > 0) {
        const long B = h->sh_block, W = h->sh_world;
        long q = f_first / B;
        const long q0 = q + ((h->sh_rank - q % W) % W + W) % W;   // first run of this rank
        a.sh_q0 = q0;
        a.sh_off = q0 == q ? (int)(f_first - q * B) : 0;
        f_lo = q0 * B + a.sh_off;
        nf = 0;
        for (q = q0; q * B < f_done; q += W) nf += std::min(f_done, (q + 1) * B) - std::max(f_first, q * B);
    }
    {
        const long f_hi = f_lo + nf;   // (unsharded: host-processor frames are f_lo .. f_hi - 1)
        a.f_lo = f_lo;
        a.i0 = (int)(f_lo % (2L * h->laps));
        a.u0 = (f_lo / (2L * h->laps)) * (2L * N - 1) - a.T0 + (N - 1);
        a.r0 = (int)(f_lo % h->R);
        // frames start in increasing order: the first one decides whether any reads an Im part
        a.hi = (nf > 0 && frame_start(f_lo, h->laps, h->stride, N) <= h->last_cplx) ? hc + (N - 1) : nullptr;
        if (nf > 0) {
            // Im planes: a pair launch leaves them unwritten (0); any other launch writes them, so
            // the last 2 laps pair frames before it, which the overlap-add still reads, get
            // explicit zeros first
            const bool pair = h->proc != HZ_PROC_HOST && pair_launch(h, a);
            if (pair) {
                if (h->im_zero_from == LONG_MAX) h->im_zero_from = f_lo;
            } else if (h->im_zero_from != LONG_MAX) {
                for (long f = std::max(h->im_zero_from, f_lo - 2L * h->laps); f < f_lo; ++f)
                    HZ_TRY_HIP(hipMemsetAsync(h->d_fo + (size_t)h->R * N + (size_t)(f % h->R) * N, 0,
                                              sizeof(double) * N, h->stream));
                h->im_zero_from = LONG_MAX;
            }
            if (h->proc != HZ_PROC_HOST) {
                // profiling may repeat the (idempotent) frame launch so the event pair brackets
                // several back-to-back launches: per-launch time without the event overhead
                for (int r = 0; r < (h->prof ? h->prof_repeat : 1); ++r) HZ_TRY(frames_fused(h, a, nf));
            } else {
                HZ_TRY(ensure_dev((void**)&h->d_spec, &h->spec_cap, sizeof(double2) * (size_t)nf * N));
                a.spec = h->d_spec;
                launch_frames<HZ_PROC_IDENTITY, 1>(h, a, nf);
                HZ_TRY_HIP(hipGetLastError());
                h->h_spec.resize((size_t)nf * N);
                HZ_TRY_HIP(hipMemcpyAsync(h->h_spec.data(), h->d_spec, sizeof(double2) * (size_t)nf * N,
                                          hipMemcpyDeviceToHost, h->stream));
                HZ_TRY_HIP(hipStreamSynchronize(h->stream));
                for (long f = f_lo; f < f_hi; ++f) {   // frame order == the reference's order
                    const int slot = (int)(f % (2 * h->laps));
                    double2* so = &h->h_out[(size_t)slot * N];
                    double2* sp = &h->h_spec[(size_t)(f - f_lo) * N];
                    h->host_proc((const double*)sp, (double*)so);
                    std::memcpy(sp, so, sizeof(double2) * N);
                }
                HZ_TRY_HIP(hipMemcpyAsync(h->d_spec, h->h_spec.data(), sizeof(double2) * (size_t)nf * N,
                                          hipMemcpyHostToDevice, h->stream));
                launch_frames<HZ_PROC_IDENTITY, 2>(h, a, nf);
                HZ_TRY_HIP(hipGetLastError());
            }
        }
    }
    if (e) HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
    OlaArgs o;
    o.fo = h->d_fo;
    o.win = h->d_win;
    o.out_re = d_ore;
    o.out_im = d_oim;
    o.T0 = h->T;
    o.n = n;
    o.N = N;
    o.laps = h->laps;
    o.stride = h->stride;
    o.R = h->R;
    o.hist_old = hc;
    o.in_re = d_re;
    o.in_im = d_im;
    o.hist_new = hn;
    o.sh_block = h->sh_block;
    o.sh_world = h->sh_world;
    o.sh_rank = h->sh_rank;
    o.sh_inv = 1.0 / (double)h->sh_block;
    o.im_zero_from = h->im_zero_from;
    static const bool ola_flat = std::getenv("HZ_STFT_OLA_FLAT") != nullptr;   // (A/B measurements)
    if (!ola_flat && (h->laps == 2 || h->laps == 4 || h->laps == 8) && h->stride * h->laps == N) {
        // segment overlap-add: one workgroup per stride-long segment of the period grid
        const long P = 2L * N - 1, S = 2L * h->laps;
        const long u_lo = std::max(h->T - (N - 1), 0L), u_hi = h->T + n - 1 - (N - 1);
        auto seg = [&](long u) {
            const long c = u / P;
            return c * S + (u - c * P) / h->stride;
        };
        const long g0 = u_hi >= u_lo ? seg(u_lo) : 0;
        o.c_first = g0 / S;
        o.row_first = (int)((o.c_first * S) % h->R);
        const long nseg = u_hi >= u_lo ? seg(u_hi) - g0 + 1 : 0;
        const long zp = h->T < N - 1 ? std::min((long)N - 1, h->T + n) - h->T : 0;
        const int aux = (int)((std::max((long)N - 1, zp) + 255) / 256);
        // (diagnostics) HZ_STFT_OLA_REPEAT=r launches the idempotent overlap-add r times: the later
        // launches show its time with the ring already in the L2s
        static const int ola_rep = std::max(1, std::getenv("HZ_STFT_OLA_REPEAT") ? std::atoi(std::getenv("HZ_STFT_OLA_REPEAT")) : 1);
        // two workgroups per segment by default (7.4 against 7.8 us per C4 launch, alternating runs,
        // profiles/r5/c4_half/olasplit.txt); HZ_STFT_OLA_SPLIT=1|2|4 for A/B runs
        static const int split = [] {
            const char* v = std::getenv("HZ_STFT_OLA_SPLIT");
            const int x = v ? std::atoi(v) : 2;
            return x == 1 || x == 4 ? x : 2;
        }();
        const dim3 gridS((unsigned)(aux + split * nseg));
        for (int rep = 0; rep < ola_rep; ++rep) {
            auto go = [&](auto kern) { hipLaunchKernelGGL(kern, gridS, dim3(256), 0, h->stream, o, g0, u_lo, u_hi, aux); };
            if (h->laps == 2) split == 1 ? go(stft_ola_seg_kernel<2, 1>) : split == 2 ? go(stft_ola_seg_kernel<2, 2>) : go(stft_ola_seg_kernel<2, 4>);
            else if (h->laps == 4) split == 1 ? go(stft_ola_seg_kernel<4, 1>) : split == 2 ? go(stft_ola_seg_kernel<4, 2>) : go(stft_ola_seg_kernel<4, 4>);
            else split == 1 ? go(stft_ola_seg_kernel<8, 1>) : split == 2 ? go(stft_ola_seg_kernel<8, 2>) : go(stft_ola_seg_kernel<8, 4>);
        }
    } else {
        const long threads = std::max(n, (long)N - 1);
        hipLaunchKernelGGL(stft_ola_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, h->stream, o);
    }
    HZ_TRY_HIP(hipGetLastError());
    if (e) HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
    h->hcur ^= 1;   // the overlap-add launch wrote the next block's history
    h->T += n;
    h->frames = f_done;
    h->launches += h->prof ? 1 : 0;
    return HZ_OK;
}

int stft_run(hz_stft* h, const double* d_re, const double* d_im, double* d_ore, double* d_oim, long n) {
    for (long o = 0; o < n; o += h->chunk) {
        const long m = std::min(h->chunk, n - o);
        HZ_TRY(stft_block(h, d_re + o, d_im ? d_im + o : nullptr, d_ore + o, d_oim ? d_oim + o : nullptr, m));
    }
    return HZ_OK;
}

}  // namespace

extern "C" {

int hz_stft_create(int N, int laps, int window, int proc, double p0, double p1, int device, hz_stft** out) {
    if (!out || !pow2(N) || N > kMaxN || laps <= 0 || laps > N || (window != HZ_WIN_HALFHANN && window != HZ_WIN_HANN) ||
        proc < HZ_PROC_IDENTITY || proc > HZ_PROC_HOST) {
        hz::set_error("hz_stft_create: invalid arguments (N must be a power of two in [4, %d])", kMaxN);
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_stft* h = new (std::nothrow) hz_stft();
    if (!h) return HZ_E_ALLOC;
    h->N = N;
    h->laps = laps;
    h->stride = N / laps;
    h->lg = ilog2(N);
    h->window = window;
    h->proc = proc;
    h->p0 = p0;
    h->p1 = p1;
    h->device = device;
    // frames completing inside one internal block, plus those still being read
    const long P = 2L * N - 1;
    auto ring = [&](long c) { return (c + P - 1) / P * 2 * laps + 2 * laps + 2; };
    h->chunk = kChunkMax;
    while (h->chunk > 4L * N && (size_t)ring(h->chunk) * N * sizeof(double2) > kRingBytes) h->chunk >>= 1;
    h->R = (int)ring(h->chunk);
    h->h_out.assign((size_t)2 * laps * N, make_double2(0.0, 0.0));
    std::vector<double> win(N);
    for (int k = 0; k < N; ++k) {   // src/wave.h:148-149 with the truncated PI, in double
        const double p = k / (double)N;
        const double hann = 0.5 * (1 - cos(2 * hz::kPI * p));
        win[k] = window == HZ_WIN_HANN ? hann : sqrt(hann);
    }
    h->h_win = win;
    const std::vector<double2> tw = twiddles(N);
    bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMalloc(&h->d_win, sizeof(double) * N) == hipSuccess;
    // N = 4096: the specialised pair kernel's pass tables after the N/2 table (p4::kTwLen)
    std::vector<double2> twx = tw;
    if (N == p4::kN) {   // W^((p << s) r) mod N, r = 1..7, in long double
        twx.resize(N / 2 + p4::kTwLen);
        const long double pi = acosl(-1.0L);
        for (int i = 0; i < p4::kTwLen; ++i) {
            int r, p, sh;
            if (i < p4::kTwB) r = i / 512 + 1, p = i % 512, sh = 0;
            else if (i < p4::kTwC) r = (i - p4::kTwB) / 64 + 1, p = (i - p4::kTwB) % 64, sh = 3;
            else r = (i - p4::kTwC) / 8 + 1, p = (i - p4::kTwC) % 8, sh = 6;
            const long k = ((long)(p << sh) * r) % N;
            const long double ang = -2.0L * pi * k / N;
            twx[N / 2 + i] = make_double2((double)cosl(ang), (double)sinl(ang));
        }
    }
    ok = ok && hipMalloc(&h->d_tw, sizeof(double2) * twx.size()) == hipSuccess;
    ok = ok && hipMalloc(&h->d_fo, sizeof(double2) * (size_t)h->R * N) == hipSuccess;
    for (double*& p : h->d_hist) {
        ok = ok && hipMalloc(&p, 2 * sizeof(double) * (N - 1)) == hipSuccess;
        ok = ok && hipMemset(p, 0, 2 * sizeof(double) * (N - 1)) == hipSuccess;
    }
    ok = ok && hipMemcpy(h->d_win, win.data(), sizeof(double) * N, hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(h->d_tw, twx.data(), sizeof(double2) * twx.size(), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemset(h->d_fo, 0, sizeof(double2) * (size_t)h->R * N) == hipSuccess;
    if (!ok) {
        hz::set_error("hz_stft_create: device allocation failed");
        if (h->stream) (void)hipStreamDestroy(h->stream);
        for (void* p : {(void*)h->d_win, (void*)h->d_tw, (void*)h->d_fo, (void*)h->d_hist[0], (void*)h->d_hist[1]})
            if (p) (void)hipFree(p);
        delete h;
        return HZ_E_ALLOC;
    }
    h->own_stream = true;
    static bool attr = false;
    if (!attr) {   // padded frame: 2 (N + N/16) doubles of LDS per workgroup (136 KB at N = 8192)
        const int lds = (int)std::max(frame_lds(kMaxN), sizeof(double) * (2 * kMaxN + 2 * (kThreads / 64)));
        frame_attr<HZ_PROC_IDENTITY, 0>(lds);
        frame_attr<HZ_PROC_STATIC_GATE, 0>(lds);
        frame_attr<HZ_PROC_GATE_KEEP, 0>(lds);
        frame_attr<HZ_PROC_HILBERT, 0>(lds);
        frame_attr<HZ_PROC_IDENTITY, 1>(lds);
        frame_attr<HZ_PROC_IDENTITY, 2>(lds);
        for (const void* k : {(const void*)slot_fft_kernel<3, false>, (const void*)slot_fft_kernel<3, true>,
                              (const void*)slot_fft_kernel<4, false>, (const void*)slot_fft_kernel<4, true>})
            (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        (void)hipFuncSetAttribute((const void*)dct2_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        (void)hipFuncSetAttribute((const void*)dct3_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr = true;
    }
    *out = h;
    return HZ_OK;
}

int hz_stft_destroy(hz_stft* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->d_win, (void*)h->d_tw, (void*)h->d_fo, (void*)h->d_hist[0], (void*)h->d_hist[1],
                    (void*)h->d_spec, (void*)h->d_in, (void*)h->d_out, (void*)h->d_slot})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_stft_set_processor(hz_stft* h, hz_stft_proc fn) {
    if (!h || !fn) {
        hz::set_error("hz_stft_set_processor: null argument");
        return HZ_E_INVALID;
    }
    h->host_proc = fn;
    h->proc = HZ_PROC_HOST;
    return HZ_OK;
}

int hz_stft_process_block_device(hz_stft* h, const double* d_re, const double* d_im, double* d_out_re,
                                 double* d_out_im, size_t n) {
    HZ_TRY(stft_check(h));
    if (n == 0) return HZ_OK;
    if (h->slot_mode) {
        hz::set_error("hz_stft_process_block: this object is driven per sample (write / read); an object runs "
                      "either per sample or by blocks");
        return HZ_E_STATE;
    }
    if (!d_re || !d_out_re) return HZ_E_INVALID;
    if (h->proc == HZ_PROC_HOST && !h->host_proc) {
        hz::set_error("hz_stft: HZ_PROC_HOST without hz_stft_set_processor");
        return HZ_E_INVALID;
    }
    return stft_run(h, d_re, d_im, d_out_re, d_out_im, (long)n);
}

int hz_stft_process_block(hz_stft* h, const double* re, const double* im, double* out_re, double* out_im,
                          size_t n) {
    HZ_TRY(stft_check(h));
    if (n == 0) return HZ_OK;
    if (!re || !out_re) return HZ_E_INVALID;
    const size_t bytes = sizeof(double) * n * 2;
    if (bytes > h->io_cap) {
        for (double** p : {&h->d_in, &h->d_out})
            if (*p) HZ_TRY_HIP(hipFree(*p));
        h->d_in = h->d_out = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_in, bytes));
        HZ_TRY_HIP(hipMalloc(&h->d_out, bytes));
        h->io_cap = bytes;
    }
    HZ_TRY_HIP(hipMemcpyAsync(h->d_in, re, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
    if (im) HZ_TRY_HIP(hipMemcpyAsync(h->d_in + n, im, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
    HZ_TRY(hz_stft_process_block_device(h, h->d_in, im ? h->d_in + n : nullptr, h->d_out, out_im ? h->d_out + n : nullptr,
                                        n));
    HZ_TRY_HIP(hipMemcpyAsync(out_re, h->d_out, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
    if (out_im)
        HZ_TRY_HIP(hipMemcpyAsync(out_im, h->d_out + n, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

}  // extern "C"

namespace {

int slot_enter(hz_stft* h) {
    if (h->slot_mode) return HZ_OK;
    if (h->T != 0 || h->sh_world > 1) {
        hz::set_error("hz_stft: per-sample calls on an object already driven by blocks (or time-sharded); an "
                      "object runs either per sample or by blocks");
        return HZ_E_STATE;
    }
    const int S = 2 * h->laps, N = h->N;
    h->s_in.assign((size_t)S * N, make_double2(0.0, 0.0));
    h->s_mid.assign((size_t)S * N, make_double2(0.0, 0.0));
    h->s_out.assign((size_t)S * N, make_double2(0.0, 0.0));
    h->s_wp.assign(S, 0);
    h->s_rp.assign(S, 0);
    h->s_reading.assign(S, 0);
    h->s_writing.assign(S, 1);
    for (int i = 0; i < S; ++i) h->s_wp[i] = -h->stride * i;   // fourier.h:76-77
    if (!h->d_slot) HZ_TRY_HIP(hipMalloc(&h->d_slot, sizeof(double2) * 2 * (size_t)N));
    h->slot_mode = true;
    return HZ_OK;
}

int slot_check(hz_stft* h, int i) {
    HZ_TRY(stft_check(h));
    HZ_TRY(slot_enter(h));
    if (i < 0 || i >= 2 * h->laps) {
        hz::set_error("hz_stft: slot %d out of range [0, %d)", i, 2 * h->laps);
        return HZ_E_RANGE;
    }
    return HZ_OK;
}

// one N-point transform of a host slot buffer on the device: src -> dst (natural order)
int slot_transform(hz_stft* h, const double2* src, double2* dst, bool inverse) {
    const int N = h->N;
    HZ_TRY_HIP(hipMemcpyAsync(h->d_slot, src, sizeof(double2) * N, hipMemcpyHostToDevice, h->stream));
    auto launch = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(1), dim3(frame_threads(N)), frame_lds(N), h->stream, (const double2*)h->d_slot,
                           h->d_slot + N, N, h->lg, (const double2*)h->d_tw);
    };
    if (frame_rmax(N) == 3) {
        if (inverse) launch(slot_fft_kernel<3, true>);
        else launch(slot_fft_kernel<3, false>);
    } else {
        if (inverse) launch(slot_fft_kernel<4, true>);
        else launch(slot_fft_kernel<4, false>);
    }
    HZ_TRY_HIP(hipGetLastError());
    HZ_TRY_HIP(hipMemcpyAsync(dst, h->d_slot + N, sizeof(double2) * N, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

// process(i): the processor on middle[i] -> out[i] (fourier.h:141-144; the host callback's
// return value is ignored there too)
int slot_process(hz_stft* h, int i) {
    const int N = h->N;
    double2* mid = &h->s_mid[(size_t)i * N];
    double2* out = &h->s_out[(size_t)i * N];
    if (h->proc == HZ_PROC_HOST) {
        if (!h->host_proc) {
            hz::set_error("hz_stft: HZ_PROC_HOST without hz_stft_set_processor");
            return HZ_E_INVALID;
        }
        (void)h->host_proc((const double*)mid, (double*)out);
        return HZ_OK;
    }
    HZ_TRY_HIP(hipMemcpyAsync(h->d_slot, mid, sizeof(double2) * N, hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipMemcpyAsync(h->d_slot + N, out, sizeof(double2) * N, hipMemcpyHostToDevice, h->stream));
    const double2* a = h->d_slot;
    double2* b = h->d_slot + N;
    switch (h->proc) {
    case HZ_PROC_STATIC_GATE:
        hipLaunchKernelGGL(slot_proc_kernel<HZ_PROC_STATIC_GATE>, dim3(1), dim3(kFrameThreads), 0, h->stream, a, b, N,
                           h->p0, h->p1);
        break;
    case HZ_PROC_GATE_KEEP:
        hipLaunchKernelGGL(slot_proc_kernel<HZ_PROC_GATE_KEEP>, dim3(1), dim3(kFrameThreads), 0, h->stream, a, b, N,
                           h->p0, h->p1);
        break;
    case HZ_PROC_HILBERT:
        hipLaunchKernelGGL(slot_proc_kernel<HZ_PROC_HILBERT>, dim3(1), dim3(kFrameThreads), 0, h->stream, a, b, N,
                           h->p0, h->p1);
        break;
    default:
        hipLaunchKernelGGL(slot_proc_kernel<HZ_PROC_IDENTITY>, dim3(1), dim3(kFrameThreads), 0, h->stream, a, b, N,
                           h->p0, h->p1);
    }
    HZ_TRY_HIP(hipGetLastError());
    HZ_TRY_HIP(hipMemcpyAsync(out, b, sizeof(double2) * N, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

}  // namespace

extern "C" {

// fourier.h:102-128: the window times the sample into every writing slot; a full slot turns to
// reading and runs forward(i), process(i), backward(i)
int hz_stft_write(hz_stft* h, double real, double imag) {
    HZ_TRY(stft_check(h));
    HZ_TRY(slot_enter(h));
    const int N = h->N;
    for (int i = 0; i < 2 * h->laps; ++i) {
        if (!h->s_writing[i]) continue;
        const int wp = h->s_wp[i];
        if (wp >= 0) {
            const double window = h->h_win[wp];   // halfhann / hann (wp / (double) N), as created
            h->s_in[(size_t)i * N + wp] = make_double2(window * real, window * imag);
        }
        if (++h->s_wp[i] == N) {
            h->s_writing[i] = 0;
            h->s_reading[i] = 1;
            h->s_rp[i] = 0;
            HZ_TRY(hz_stft_forward(h, i));
            HZ_TRY(hz_stft_process_slot(h, i));
            HZ_TRY(hz_stft_backward(h, i));
            ++h->frames;
        }
    }
    return HZ_OK;
}

// fourier.h:147-177: the windowed overlap-add of the reading slots, in long double, divided by
// the int N * laps / 2; a slot read to its end turns back to writing
int hz_stft_read(hz_stft* h, double* real, double* imag) {
    HZ_TRY(stft_check(h));
    HZ_TRY(slot_enter(h));
    const int N = h->N;
    long double ra = 0, ia = 0;
    for (int i = 0; i < 2 * h->laps; ++i) {
        if (!h->s_reading[i]) continue;
        const int rp = h->s_rp[i];
        const double window = h->h_win[rp];
        const double2 v = h->s_in[(size_t)i * N + rp];
        ra += window * v.x;
        ia += window * v.y;
        if (++h->s_rp[i] == N) {
            h->s_writing[i] = 1;
            h->s_reading[i] = 0;
            h->s_wp[i] = 0;
        }
    }
    ra /= N * h->laps / 2;
    ia /= N * h->laps / 2;
    if (real) *real = (double)ra;
    if (imag) *imag = (double)ia;
    return HZ_OK;
}

int hz_stft_forward(hz_stft* h, int i) {   // fourier.h:130-133: FFT in[i] -> middle[i]
    HZ_TRY(slot_check(h, i));
    return slot_transform(h, &h->s_in[(size_t)i * h->N], &h->s_mid[(size_t)i * h->N], false);
}

int hz_stft_backward(hz_stft* h, int i) {   // fourier.h:135-138: IFFT out[i] -> in[i]
    HZ_TRY(slot_check(h, i));
    return slot_transform(h, &h->s_out[(size_t)i * h->N], &h->s_in[(size_t)i * h->N], true);
}

int hz_stft_process_slot(hz_stft* h, int i) {   // fourier.h:141-144
    HZ_TRY(slot_check(h, i));
    return slot_process(h, i);
}

int hz_stft_set_frame_shard(hz_stft* h, int rank, int world, long block) {
    HZ_TRY(stft_check(h));
    if (world < 1 || rank < 0 || rank >= world || block < 1) {
        hz::set_error("hz_stft_set_frame_shard: bad shard (rank %d of %d, block %ld)", rank, world, block);
        return HZ_E_INVALID;
    }
    if (h->proc == HZ_PROC_HOST && world > 1) {
        hz::set_error("hz_stft_set_frame_shard: a host processor sees every frame in order (replicas only)");
        return HZ_E_UNSUPPORTED;
    }
    h->sh_rank = rank;
    h->sh_world = world;
    h->sh_block = block;
    return HZ_OK;
}

int hz_stft_frames_before(int N, int laps, long samples, long* frames) {
    if (!frames || !pow2(N) || laps <= 0 || laps > N || samples < 0) return HZ_E_INVALID;
    hz_stft tmp;
    tmp.N = N;
    tmp.laps = laps;
    tmp.stride = N / laps;
    *frames = frames_before(&tmp, samples);
    return HZ_OK;
}

int hz_stft_frames(hz_stft* h, long* frames, long* samples) {
    if (!h) return HZ_E_INVALID;
    if (frames) *frames = h->frames;
    if (samples) *samples = h->T;
    return HZ_OK;
}

int hz_stft_set_stream(hz_stft* h, void* stream) {
    HZ_TRY(stft_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) HZ_TRY_HIP(hipStreamDestroy(h->stream));
    h->stream = (hipStream_t)stream;
    h->own_stream = false;
    return HZ_OK;
}

int hz_stft_synchronize(hz_stft* h) {
    HZ_TRY(stft_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_stft_profile(hz_stft* h, int enable) {
    HZ_TRY(stft_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    h->prof = enable != 0;
    h->prof_repeat = enable > 1 ? enable : 1;
    h->ev_used = 0;
    h->launches = 0;
    return HZ_OK;
}

int hz_stft_profile_read(hz_stft* h, double* frame_ms, double* ola_ms, long* blocks) {
    HZ_TRY(stft_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    double fm = 0.0, om = 0.0;
    for (size_t i = 0; i + 2 < h->ev_used; i += 3) {
        float t0 = 0.f, t1 = 0.f;
        HZ_TRY_HIP(hipEventElapsedTime(&t0, h->ev[i], h->ev[i + 1]));
        HZ_TRY_HIP(hipEventElapsedTime(&t1, h->ev[i + 1], h->ev[i + 2]));
        fm += t0;
        om += t1;
    }
    if (frame_ms) *frame_ms = fm / (h->proc != HZ_PROC_HOST ? h->prof_repeat : 1);   // per single launch
    if (ola_ms) *ola_ms = om;
    if (blocks) *blocks = h->launches;
    h->ev_used = 0;
    h->launches = 0;
    return HZ_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Cosine
// ---------------------------------------------------------------------------
struct hz_dct {
    int N = 0, lg = 0, device = 0;
    double *h_in = nullptr, *h_out = nullptr;   // pinned, owned (fourier.h:201-207)
    double *d_a = nullptr, *d_b = nullptr;
    double2 *d_tw = nullptr, *d_rot = nullptr;
    hipStream_t stream = nullptr;
};

namespace {

int dct_launch(hz_dct* h, const double* d_x, double* d_y, int batch, int kind) {
    const size_t lds = sizeof(double) * 2 * (size_t)h->N;
    if (kind == 10)
        hipLaunchKernelGGL(dct2_kernel, dim3((unsigned)batch), dim3(kThreads), lds, h->stream, d_x, d_y, h->N, h->lg,
                           (const double2*)h->d_tw, (const double2*)h->d_rot);
    else
        hipLaunchKernelGGL(dct3_kernel, dim3((unsigned)batch), dim3(kThreads), lds, h->stream, d_x, d_y, h->N, h->lg,
                           (const double2*)h->d_tw, (const double2*)h->d_rot);
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

}  // namespace

extern "C" {

int hz_dct_create(int N, int device, hz_dct** out) {
    if (!out || !pow2(N) || N > kMaxN) {
        hz::set_error("hz_dct_create: N must be a power of two in [4, %d]", kMaxN);
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_dct* h = new (std::nothrow) hz_dct();
    if (!h) return HZ_E_ALLOC;
    h->N = N;
    h->lg = ilog2(N);
    h->device = device;
    const std::vector<double2> tw = twiddles(N);
    std::vector<double2> rot(N);
    const long double pi = acosl(-1.0L);
    for (int k = 0; k < N; ++k) {
        const long double a = -pi * k / (2.0L * N);
        rot[k] = make_double2((double)cosl(a), (double)sinl(a));
    }
    bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipHostMalloc(&h->h_in, sizeof(double) * N) == hipSuccess;
    ok = ok && hipHostMalloc(&h->h_out, sizeof(double) * N) == hipSuccess;
    ok = ok && hipMalloc(&h->d_a, sizeof(double) * N) == hipSuccess;
    ok = ok && hipMalloc(&h->d_b, sizeof(double) * N) == hipSuccess;
    ok = ok && hipMalloc(&h->d_tw, sizeof(double2) * (N / 2)) == hipSuccess;
    ok = ok && hipMalloc(&h->d_rot, sizeof(double2) * N) == hipSuccess;
    ok = ok && hipMemcpy(h->d_tw, tw.data(), sizeof(double2) * (N / 2), hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(h->d_rot, rot.data(), sizeof(double2) * N, hipMemcpyHostToDevice) == hipSuccess;
    if (!ok) {
        hz::set_error("hz_dct_create: allocation failed");
        if (h->stream) (void)hipStreamDestroy(h->stream);
        for (double* p : {h->h_in, h->h_out})
            if (p) (void)hipHostFree(p);
        for (void* p : {(void*)h->d_a, (void*)h->d_b, (void*)h->d_tw, (void*)h->d_rot})
            if (p) (void)hipFree(p);
        delete h;
        return HZ_E_ALLOC;
    }
    std::memset(h->h_in, 0, sizeof(double) * N);
    std::memset(h->h_out, 0, sizeof(double) * N);
    *out = h;
    return HZ_OK;
}

int hz_dct_destroy(hz_dct* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (double* p : {h->h_in, h->h_out})
        if (p) (void)hipHostFree(p);
    for (void* p : {(void*)h->d_a, (void*)h->d_b, (void*)h->d_tw, (void*)h->d_rot})
        if (p) (void)hipFree(p);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_dct_buffers(hz_dct* h, double** in, double** out) {   // Cosine(N, &in, &out)
    if (!h) return HZ_E_INVALID;
    if (in) *in = h->h_in;
    if (out) *out = h->h_out;
    return HZ_OK;
}

int hz_dct_forward(hz_dct* h) {   // REDFT10: in -> out
    if (!h) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->device));
    HZ_TRY_HIP(hipMemcpyAsync(h->d_a, h->h_in, sizeof(double) * h->N, hipMemcpyHostToDevice, h->stream));
    HZ_TRY(dct_launch(h, h->d_a, h->d_b, 1, 10));
    HZ_TRY_HIP(hipMemcpyAsync(h->h_out, h->d_b, sizeof(double) * h->N, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_dct_backward(hz_dct* h) {   // REDFT01: out -> in
    if (!h) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->device));
    HZ_TRY_HIP(hipMemcpyAsync(h->d_b, h->h_out, sizeof(double) * h->N, hipMemcpyHostToDevice, h->stream));
    HZ_TRY(dct_launch(h, h->d_b, h->d_a, 1, 1));
    HZ_TRY_HIP(hipMemcpyAsync(h->h_in, h->d_a, sizeof(double) * h->N, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_dct_forward_device(hz_dct* h, const double* d_in, double* d_out, int batch) {
    if (!h || !d_in || !d_out || batch < 0) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->device));
    if (batch) HZ_TRY(dct_launch(h, d_in, d_out, batch, 10));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_dct_backward_device(hz_dct* h, const double* d_in, double* d_out, int batch) {
    if (!h || !d_in || !d_out || batch < 0) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->device));
    if (batch) HZ_TRY(dct_launch(h, d_in, d_out, batch, 1));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

}  // extern "C"
