// hz_fb_stream.hip -- the stationary Filterbank<double> engine for streaming calls (one
// launch per 1024-sample block).
//
// The reference runs the bank inside a 1024-sample audio callback, one sample at a time
// (tests/resynthesis.cpp:33-42 -> src/filterbank.h:125-148).  Once the bank is stationary
// (hz_fb_resp.hip: converged for its horizon K), the block's mixdown is
//     out[t] = sum_{tau < K} h[tau] x[t - tau]
// and a block call runs here as ONE kernel launch of a uniformly partitioned overlap-save
// convolution with P = 1024-sample partitions (the call length) and F = 2048-point real transforms,
// whose frequency-domain delay line -- the spectra Z of the last Q = K / P windows -- stays on the
// device between calls.  Each transform is split column-wise (four-step, n = 32 n1 + n2,
// k = k1 + 64 k2), so workgroup c (c = 0..32) computes its 32 bins straight from the samples and
// Hermitian symmetry gives columns 33..63.  The launch has three roles that share no data, so no
// workgroup waits for another (an in-launch exchange of the inverse columns measured 10 us per
// block: its write-through, arrival and reload round trips are the block's latency):
//   outputs    y_b = head_b + tail_b: head = the partition-0 term h[0..1023] * x, direct in time;
//              tail = the Hermitian combine of 33 inverse columns C_b the PREVIOUS launch wrote
//   transform  Z_b into the ring; Y_{b+1} = H_1 Z_b + H_2 Z_{b-1} + R_{b+1}; C_{b+1} = its inverse
//              columns (the next block's tail)
//   MAC        R_{b+2} = sum_{p >= 3} H_p Z_{b+2-p} over the ring (Z_{b-1} and older)
// tests/stream_model.py restates this schedule and is checked against a direct convolution.
//
// Band states stay implicit (every mode): they are the zero-start response of the last K inputs,
// which the engine keeps in a mirrored device ring (every sample written at i and i + R, so any K
// consecutive samples are contiguous), and are computed by the band-state pass
// (hz_fb_state.hip) only when a later call, get_state, tick or a setter needs them.
#include <cstdio>
#include <type_traits>
#include <utility>

#include "hz_dd.h"
#include "hz_fb_impl.h"

#ifndef HZ_STREAM_OUTN
#define HZ_STREAM_OUTN 16
#endif

namespace {

constexpr int kSP = hz_fbi::kStreamBlock;   // partition = call length
constexpr int kSF = 2 * kSP;                // real transform length
constexpr int kCols = 33;                   // stored columns k1 = 0..32
constexpr int kT = 256;                     // threads per column workgroup
constexpr long kMaxK = 1L << 17;            // longest head streamed (Q <= 128 partitions of 1024)
constexpr long kMaxTailK = 1L << 21;        // longest horizon streamed with a response tail
constexpr long kE = 16384;                  // tail epoch: h[K1, K) convolved per 16384 outputs
// twiddle table (double2): W_64^m (m < 64), W_32^m (m < 32), W_2048^m (m < 1024)
constexpr int kTw64 = 0, kTw32 = 64, kTw2k = 96, kTwN = 96 + 1024;

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
// conj(a) b
__device__ __forceinline__ double2 cmulc(double2 a, double2 b) {
    return make_double2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
// write-through (sc1) 8-byte store / load: agent-scope relaxed atomics
__device__ __forceinline__ void st_sc1(double* p, double v) {
    __hip_atomic_store((unsigned long long*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
    return __longlong_as_double(
        (long long)__hip_atomic_load((unsigned long long*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// sum of lanes l and l + 32 (the two thread groups g = 2w, 2w + 1 of a wave)
__device__ __forceinline__ double2 half_sum(double2 v) {
    return make_double2(v.x + __shfl_xor(v.x, 32), v.y + __shfl_xor(v.y, 32));
}

struct ColLds {
    double2 a[4][32];    // stage-1 partials per wave
    double2 x[4][32];    // stage-3 partials
    double2 m[4][32];    // MAC partials
    double2 y[32];       // the column's output spectrum
    double2 c[4][32];    // inverse partials
    double2 col[kCols][32];   // (last workgroup) the published columns
    double2 tw[64];           // (last workgroup) W_64^m
    int last;
};

// Thread layout: t = 64 w + l, j = l & 31 (n2 / k2 / n2), g = 2 w + (l >> 5) (0..7).
// Stage 1: A[n2] = sum_{n1 < 64} win[32 n1 + n2] W_64^(n1 c); the thread sums n1 = g + 8 i.
__device__ __forceinline__ double2 stage1(const double (&v)[8], const double2 (&t64)[8]) {
    double2 a = make_double2(0.0, 0.0);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a.x = fma(v[i], t64[i].x, a.x);
        a.y = fma(v[i], t64[i].y, a.y);
    }
    return half_sum(a);
}
// Stage 3 partial: sum_{q < 4} W_32^((4g+q) k2) W_2048^((4g+q) c) A[4g+q]
__device__ __forceinline__ double2 stage3(const ColLds& s, int g, const double2 (&t2k)[4], const double2 (&t32)[4]) {
    double2 xp = make_double2(0.0, 0.0);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int n2 = 4 * g + q;
        double2 a = cadd(cadd(s.a[0][n2], s.a[1][n2]), cadd(s.a[2][n2], s.a[3][n2]));
        xp = cadd(xp, cmul(t32[q], cmul(t2k[q], a)));
    }
    return half_sum(xp);
}

struct ColTw {   // the thread's twiddles for column c
    double2 t64[8], t2k[4], t32[4];
    __device__ __forceinline__ void load(const double2* __restrict__ tw, int c, int j, int g) {
#pragma unroll
        for (int i = 0; i < 8; ++i) t64[i] = tw[kTw64 + (((g + 8 * i) * c) & 63)];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            t2k[q] = tw[kTw2k + (4 * g + q) * c];
            t32[q] = tw[kTw32 + (((4 * g + q) * j) & 31)];
        }
    }
};

// One column's bins of a window's spectrum into dst[k2] (k2 < 32): prime / partition spectra.
// (v[i] = the window at 32 (g + 8 i) + j)
__device__ __forceinline__ void col_forward_v(ColLds& s, const double2* __restrict__ tw, int c, const double (&v)[8],
                                              double2* __restrict__ dst) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    ColTw ct;
    ct.load(tw, c, j, g);
    const double2 a = stage1(v, ct.t64);
    if (l < 32) s.a[w][j] = a;
    __syncthreads();
    const double2 xp = stage3(s, g, ct.t2k, ct.t32);
    if (l < 32) s.x[w][j] = xp;
    __syncthreads();
    if (t < 32) dst[t] = cadd(cadd(s.x[0][t], s.x[1][t]), cadd(s.x[2][t], s.x[3][t]));
}
template <class Load>
__device__ __forceinline__ void col_forward(ColLds& s, const double2* __restrict__ tw, int c, Load load,
                                            double2* __restrict__ dst) {
    const int t = threadIdx.x, l = t & 63, g = 2 * (t >> 6) + (l >> 5), j = l & 31;
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = load(32 * (g + 8 * i) + j);
    col_forward_v(s, tw, c, v, dst);
}

// Partition spectra HS[p][c][k2] = DFT_2048(h[pP, (p+1)P) zero-padded) / F, grid (33, Q)
__global__ __launch_bounds__(kT) void stream_hs_kernel(const double* __restrict__ h, const double2* __restrict__ tw,
                                                       double2* __restrict__ HS) {
    __shared__ ColLds s;
    const int c = blockIdx.x, p = blockIdx.y;
    const double* hp = h + (long)p * kSP;
    col_forward(s, tw, c, [&](int n) { return n < kSP ? hp[n] * (1.0 / kSF) : 0.0; },
                HS + ((long)p * kCols + c) * 32);
}

struct StreamArgs {
    const double* x;      // [1024] the call's input
    double* out;          // [1024]
    double* line;         // [2 R] mirrored input ring
    long R;
    long wpos;            // write position of the call's first sample (pos mod R, a multiple of 1024)
    long prev;            // ring index of the previous block's first sample ((pos - 1024) mod R)
    const double2* HS;    // [Q + 8][33][32] (rows past Q zero)
    double2* ZS;          // [Q][33][32] window spectra ring
    int Q, head;          // partitions; slot of this call's window Z_b (Z_{b-p}: head - p mod Q)
    const double2* tw;
    const double* h;      // [K] the bank response (head taps 0 .. 1023)
    const double2* Cin;   // [33][32] inverse columns of this block's tail (previous launch)
    double2* Cout;        // [33][32] ... of the next block's tail
    const double2* Rin;   // [33][32] R_{b+1} = sum_{p >= 3} H_p Z_{b+1-p} (previous launch)
    double2* Rout;        // [33][32] R_{b+2}
    // host-buffer calls (hz_fb_process): every workgroup posts `seq` to flags[blockIdx] in pinned
    // host memory once its reads of x and writes of out are done, so the host returns without a
    // stream synchronisation (null: device-buffer calls)
    long long* flags;
    long long seq;
    const double* tail2;  // [1024] the response tail's contribution to this block (null: none)
    // (a gain transient, DUAL) h_D's spectra, taps and C / R parities; s_g^(pos - dref + 1), s_g^j
    const double2* HSD;
    const double* hD;
    const double2* CDin;
    double2* CDout;
    const double2* RDin;
    double2* RDout;
    double dscale;
    const double* sgpow;
    unsigned long long* trace;   // (diagnostic, HZ_STREAM_TRACE) [2][512]: every workgroup's start and end
};

// all of this workgroup's stores complete, then one system-scope release of the flag
// (only the plain launch's workgroups post -- blockIdx < fb_stream_workgroups(), the host's flag
// slots; a transient's extra roles write only the next launch's parities, stream-ordered)
constexpr int kOutN = HZ_STREAM_OUTN;   // outputs per output workgroup (64: 4.4 us per plain block,
                                        // 32: 3.8 us -- the role's head FMAs and LDS reads)
constexpr int kOG = kOutN / 8;           // output groups of 8 per thread
constexpr int kQG = kT / kOG;            // head tap groups
constexpr int kTG = kSP / kQG;           // taps per group
constexpr int kNG = kT / kOutN;          // partial-sum / tail column groups
__device__ __forceinline__ void post_done(const StreamArgs& a) {
    if (!a.flags || (int)blockIdx.x >= 2 * kCols + kSP / kOutN) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(a.flags + blockIdx.x, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ int ring_slot(int head, int back, int Q) {
    int s = head - back;
    while (s < 0) s += Q;
    return s;
}

// inverse column (s.y holds the column's 32 bins Y[k2]): C[n2] = W_2048^(-n2 c) sum_k2 W_32^(-n2 k2)
// Y[k2] -> dst[n2] (n2 < 32); the thread sums k2 = 4 g + q with the forward's stage-3 twiddles
// conjugated (index (4g+q) j mod 32 either way)
__device__ __forceinline__ void col_inverse_store(ColLds& s, const ColTw& ct, double2 tcol, double2* __restrict__ dst) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    double2 cp = make_double2(0.0, 0.0);
#pragma unroll
    for (int q = 0; q < 4; ++q) cp = cadd(cp, cmulc(ct.t32[q], s.y[4 * g + q]));
    cp = half_sum(cp);
    if (l < 32) s.c[w][j] = cp;
    __syncthreads();
    if (t < 32) dst[t] = cmulc(tcol, cadd(cadd(s.c[0][t], s.c[1][t]), cadd(s.c[2][t], s.c[3][t])));
}

// The ring's windows b - p (p = 1 .. Q - 1) from the history: slot (head - p) mod Q <- the window
// [pos - P (p + 1), pos - P (p - 1)), grid (33, Q - 1)
__global__ __launch_bounds__(kT) void stream_prime_kernel(StreamArgs a) {
    __shared__ ColLds s;
    const int c = blockIdx.x, p = blockIdx.y + 1;
    long ws = a.wpos - (long)kSP * (p + 1);
    if (ws < 0) ws += a.R;
    const double* src = a.line + ws;   // contiguous: ws < R, ws + 2048 <= 2 R
    col_forward(s, a.tw, c, [&](int n) { return src[n]; }, a.ZS + ((long)ring_slot(a.head, p, a.Q) * kCols + c) * 32);
}

// after stream_prime_kernel, per column: the first block's tail columns C_b (Y_b = sum_{p >= 1}
// H_p Z_{b-p}) into Cout and R_{b+1} = sum_{p >= 3} H_p Z_{b+1-p} into Rout
template <int QI>
// (blockIdx.y = 1: the same for a gain transient's h_D -- its spectra and C / R parities -- in the
// same launch)
__global__ __launch_bounds__(kT) void stream_prime2_kernel(StreamArgs a) {
    __shared__ ColLds s;
    const int t = threadIdx.x, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    const int c = blockIdx.x;
    const double2* __restrict__ HS = blockIdx.y ? a.HSD : a.HS;
    double2* Rout = blockIdx.y ? a.RDout : a.Rout;
    double2* Cout = blockIdx.y ? a.CDout : a.Cout;
    double2 y = make_double2(0.0, 0.0), r = make_double2(0.0, 0.0);
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        const int p = 1 + g + 8 * i;   // <= Q: row Q of HS is zero
        y = cadd(y, cmul(HS[((long)p * kCols + c) * 32 + j], a.ZS[((long)ring_slot(a.head, p, a.Q) * kCols + c) * 32 + j]));
        const int p3 = 3 + g + 8 * i;  // < Q + 8
        r = cadd(r, cmul(HS[((long)p3 * kCols + c) * 32 + j],
                         a.ZS[((long)ring_slot(a.head, p3 - 1, a.Q) * kCols + c) * 32 + j]));
    }
    ColTw ct;
    ct.load(a.tw, c, j, g);
    const double2 tcol = a.tw[kTw2k + j * c];
    y = half_sum(y);
    r = half_sum(r);
    if (l < 32) {
        s.m[w][j] = y;
        s.x[w][j] = r;
    }
    __syncthreads();
    if (t < 32) {
        s.y[t] = cadd(cadd(s.m[0][t], s.m[1][t]), cadd(s.m[2][t], s.m[3][t]));
        Rout[c * 32 + t] = cadd(cadd(s.x[0][t], s.x[1][t]), cadd(s.x[2][t], s.x[3][t]));
    }
    __syncthreads();
    col_inverse_store(s, ct, tcol, Cout + c * 32);
}

struct OutLds {
    double sx[1088];          // x[t0 - 1023 .. t0 + kOutN - 1]
    double sh[kSP];           // h[0 .. 1023]
    double2 col[kCols][32];   // the tail's inverse columns
    double2 tw[64];
    double part[kQG][kOutN + 1];   // head partials [tap group][output]
    double tpart[kNG][kOutN];      // tail partials [column group][output]
    double red[kNG][kOutN];        // head partials summed over 8 tap groups
};
// (a gain transient, FUSED) the same for h_D
struct OutLdsD {
    OutLds m;
    double shD[kSP];
    double2 colD[kCols][32];
    double partD[kQG][kOutN + 1];
    double tpartD[kNG][kOutN];
    double redD[kNG][kOutN];
};
union StreamLds {
    ColLds col;
    OutLds out;
};
union StreamLdsD {
    ColLds col;
    OutLdsD out;
};

// ---- the three roles of a block launch (tests/stream_model.py) -------------------------------
// transform column c: Z_b's bins from the window (WRITEZ: into the ring); Y_{b+1} = H_1 Z_b +
// H_2 Z_{b-1} + R_{b+1}; its inverse column -> Cout (the next block's tail)
template <bool WRITEZ>
__device__ __forceinline__ void role_transform(const StreamArgs& a, const double2* __restrict__ HS,
                                               const double2* __restrict__ Rin, double2* __restrict__ Cout,
                                               ColLds& s, int c) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    double v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = a.line[a.prev + 32 * (g + 8 * i) + j];
#pragma unroll
    for (int i = 4; i < 8; ++i) v[i] = a.x[32 * (g + 8 * i - 32) + j];
    double2 h1 = make_double2(0.0, 0.0), h2 = h1, z1 = h1, rn = h1;
    if (t < 32) {
        h1 = HS[((long)1 * kCols + c) * 32 + t];
        h2 = HS[((long)2 * kCols + c) * 32 + t];
        z1 = a.ZS[((long)ring_slot(a.head, 1, a.Q) * kCols + c) * 32 + t];
        rn = Rin[c * 32 + t];
    }
    ColTw ct;
    ct.load(a.tw, c, j, g);
    const double2 tcol = a.tw[kTw2k + j * c];
    const double2 a1 = stage1(v, ct.t64);
    if (l < 32) s.a[w][j] = a1;
    __syncthreads();
    const double2 xp = stage3(s, g, ct.t2k, ct.t32);
    if (l < 32) s.x[w][j] = xp;
    __syncthreads();
    if (t < 32) {
        const double2 X = cadd(cadd(s.x[0][t], s.x[1][t]), cadd(s.x[2][t], s.x[3][t]));
        if (WRITEZ) a.ZS[((long)a.head * kCols + c) * 32 + t] = X;
        s.y[t] = cadd(cadd(cmul(h1, X), cmul(h2, z1)), rn);
    }
    __syncthreads();
    col_inverse_store(s, ct, tcol, Cout + c * 32);
}

// MAC column c: R_{b+2} = sum_{p >= 3} H_p Z_{b+2-p} over the ring -> Rout
template <int QI>
__device__ __forceinline__ void role_mac(const StreamArgs& a, const double2* __restrict__ HS, double2* __restrict__ Rout,
                                         ColLds& s, int c) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    double2 hv[QI], zv[QI];
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        const int p = 3 + g + 8 * i;   // < Q + 3; partitions past Q - 1 contribute nothing
        // (masked: slot ring_slot(head, Q) is the one this launch's transform role writes)
        const bool live = p < a.Q;
        hv[i] = live ? HS[((long)p * kCols + c) * 32 + j] : make_double2(0.0, 0.0);
        zv[i] = live ? a.ZS[((long)ring_slot(a.head, p - 2, a.Q) * kCols + c) * 32 + j] : make_double2(0.0, 0.0);
    }
    double2 r = make_double2(0.0, 0.0);
#pragma unroll
    for (int i = 0; i < QI; ++i) r = cadd(r, cmul(hv[i], zv[i]));
    r = half_sum(r);
    if (l < 32) s.m[w][j] = r;
    __syncthreads();
    if (t < 32) Rout[c * 32 + t] = cadd(cadd(s.m[0][t], s.m[1][t]), cadd(s.m[2][t], s.m[3][t]));
}

// head: thread = 8 outputs (o8) x kTG taps (q): y[j] += h[tau] x[t0 + j - tau], partials into part
__device__ __forceinline__ void head_partials(const double* __restrict__ sx, const double* __restrict__ sh,
                                              double (*part)[kOutN + 1]) {
    const int t = threadIdx.x, o8 = t % kOG, q = t / kOG;
    const int j0 = 8 * o8, tau0 = kTG * q;
    double xs[kTG + 7], hs[kTG], acc[8];
#pragma unroll
    for (int i = 0; i < kTG + 7; ++i) xs[i] = sx[1023 + j0 - tau0 - (kTG - 1) + i];   // x[t0 + j0 - tau0 - kTG + 1 + i]
#pragma unroll
    for (int i = 0; i < kTG; ++i) hs[i] = sh[tau0 + i];
#pragma unroll
    for (int r = 0; r < 8; ++r) acc[r] = 0.0;
#pragma unroll
    for (int i = 0; i < kTG; ++i)
#pragma unroll
        for (int r = 0; r < 8; ++r) acc[r] = fma(hs[i], xs[kTG - 1 + r - i], acc[r]);
#pragma unroll
    for (int r = 0; r < 8; ++r) part[q][j0 + r] = acc[r];
}

// tail partials: output o (t % kOutN), columns c = 1 + cg + kNG i (cg = t / kOutN)
__device__ __forceinline__ void tail_partials(const double2 (*col)[32], const double2* __restrict__ tw, int t0,
                                              double (*tpart)[kOutN]) {
    const int t = threadIdx.x, o = t % kOutN, cg = t / kOutN;
    const int n = t0 + o, m = n >> 5, n2 = n & 31, n1 = 32 + m;
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < 32 / kNG; ++i) {
        const int c = 1 + cg + kNG * i;
        if (c < 32) {
            const double2 C = col[c][n2], wv = tw[(n1 * c) & 63];
            acc = fma(wv.x, C.x, fma(wv.y, C.y, acc));
        }
    }
    acc *= 2.0;
    if (cg == 0) acc += col[0][n2].x + ((n1 & 1) ? -col[32][n2].x : col[32][n2].x);
    tpart[cg][o] = acc;
}

// kOutN outputs: head (h[0..1023] direct, the partition-0 term of overlap-save) + tail (the 33
// columns Cin of the previous launch, Hermitian-combined); DUAL (a gain transient): + s_g^(t - dref
// + 1) x the same for h_D (its taps and columns)
template <bool DUAL, class L>
__device__ __forceinline__ void role_out(const StreamArgs& a, L& u, int k) {
    OutLds& s = [&]() -> OutLds& {
        if constexpr (DUAL) return u.m;
        else return u;
    }();
    const int t = threadIdx.x;
    const int t0 = kOutN * k;
    constexpr int nwin = kSP - 1 + kOutN;   // window x[t0 - 1023 .. t0 + kOutN - 1]
    // (diagnostic, HZ_STREAM_TRACE) phase marks of output workgroup k: trace[768 + 4 k + m]
#define OUT_MARK(m) \
    if (a.trace && t == 0) a.trace[768 + 4 * k + (m)] = __builtin_amdgcn_s_memrealtime();
    // every global load of the thread in flight before the first LDS store (a load -> store
    // chain per loop iteration waited one memory latency each): window positions t0 + 1 ..
    // t0 + nwin (2048-sample window: previous block | this block), h[0..1023], the columns
    double xv[5], hv[4], hvD[4];
    double2 cv[5], cvD[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const int i = min(t + q * kT, nwin - 1);
        const int wp = t0 + 1 + i;
        xv[q] = wp < kSP ? a.line[a.prev + wp] : a.x[wp - kSP];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        hv[q] = a.h[t + q * kT];
        if (DUAL) hvD[q] = a.hD[t + q * kT];
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        cv[q] = a.Cin[min(t + q * kT, kCols * 32 - 1)];
        if (DUAL) cvD[q] = a.CDin[min(t + q * kT, kCols * 32 - 1)];
    }
    const double2 twv = a.tw[kTw64 + (t & 63)];
#pragma unroll
    for (int q = 0; q < 5; ++q)
        if (t + q * kT < nwin) s.sx[t + q * kT] = xv[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) s.sh[t + q * kT] = hv[q];
#pragma unroll
    for (int q = 0; q < 5; ++q)
        if (t + q * kT < kCols * 32) (&s.col[0][0])[t + q * kT] = cv[q];
    if constexpr (DUAL) {
#pragma unroll
        for (int q = 0; q < 4; ++q) u.shD[t + q * kT] = hvD[q];
#pragma unroll
        for (int q = 0; q < 5; ++q)
            if (t + q * kT < kCols * 32) (&u.colD[0][0])[t + q * kT] = cvD[q];
    }
    if (t < 64) s.tw[t] = twv;
    __syncthreads();
    OUT_MARK(0)
    // the block's samples into the ring (both mirror positions), for the next calls
    if (t < kOutN) {
        const double xw = s.sx[1023 + t];
        const long kk = a.wpos + t0 + t;
        a.line[kk] = xw;
        a.line[kk + a.R] = xw;
    }
    head_partials(s.sx, s.sh, s.part);
    tail_partials(s.col, s.tw, t0, s.tpart);
    if constexpr (DUAL) {
        head_partials(s.sx, u.shD, u.partD);
        tail_partials(u.colD, s.tw, t0, u.tpartD);
    }
    __syncthreads();
    OUT_MARK(1)
    // the kQG head partials of each output: 8 per thread over all 256 threads (independent LDS reads,
    // one round trip), then kNG per output
    {
        const int o = t % kOutN, qg = t / kOutN;
        double h8[8], h8d[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            h8[i] = s.part[8 * qg + i][o];
            if constexpr (DUAL) h8d[i] = u.partD[8 * qg + i][o];
        }
        s.red[qg][o] = ((h8[0] + h8[1]) + (h8[2] + h8[3])) + ((h8[4] + h8[5]) + (h8[6] + h8[7]));
        if constexpr (DUAL) u.redD[qg][o] = ((h8d[0] + h8d[1]) + (h8d[2] + h8d[3])) + ((h8d[4] + h8d[5]) + (h8d[6] + h8d[7]));
    }
    __syncthreads();
    OUT_MARK(2)
    if (t < kOutN) {
        auto sumg = [&](const double (*v)[kOutN]) {
            double r[kNG];
#pragma unroll
            for (int g = 0; g < kNG; ++g) r[g] = v[g][t];
#pragma unroll
            for (int w = kNG / 2; w >= 1; w /= 2)
#pragma unroll
                for (int g = 0; g < w; ++g) r[g] = r[g] + r[g + w];
            return r[0];
        };
        const double y = sumg(s.red), tail = sumg(s.tpart);
        double o = a.tail2 ? (y + tail) + a.tail2[t0 + t] : y + tail;
        if constexpr (DUAL) o += (a.dscale * a.sgpow[t0 + t]) * (sumg(u.redD) + sumg(u.tpartD));
        a.out[t0 + t] = o;
    }
}

// One 1024-sample block, three roles with no data shared inside the launch (tests/stream_model.py):
//   blocks [0, 33)  transform column c
//   blocks [33, 66) MAC column c
//   blocks [66, 98) kOutN = 32 outputs each: head + tail
// DUAL (a gain transient, hz_fb_stream fb_stream_gain_setter): the transient response's roles in
// the same launch -- its own transform columns (Z_b transformed again: no dependence on the main
// transform role), its MAC columns (h_D's spectra, its C / R parities), and the output role adds
// s_g^(t - dref + 1) (head_D + tail_D).  [98, 131) D transform, [131, 164) D MAC.
// QI = Q / 8: partitions per MAC thread.
template <int QI, bool DUAL>
__global__ __launch_bounds__(kT) void stream_block_kernel(StreamArgs a) {
    using Lds = typename std::conditional<DUAL, StreamLdsD, StreamLds>::type;
    __shared__ Lds u;
    const int blk = blockIdx.x;
    if (a.trace && threadIdx.x == 0) a.trace[blk] = __builtin_amdgcn_s_memrealtime();
    constexpr int kOut0 = 2 * kCols, kOut1 = 2 * kCols + kSP / kOutN;
    if (blk < kCols) {
        role_transform<true>(a, a.HS, a.Rin, a.Cout, u.col, blk);
    } else if (blk < 2 * kCols) {
        role_mac<QI>(a, a.HS, a.Rout, u.col, blk - kCols);
    } else if (blk < kOut1) {
        role_out<DUAL>(a, u.out, blk - kOut0);
    } else if constexpr (DUAL) {
        if (blk < kOut1 + kCols) role_transform<false>(a, a.HSD, a.RDin, a.CDout, u.col, blk - kOut1);
        else role_mac<QI>(a, a.HSD, a.RDout, u.col, blk - kOut1 - kCols);
    }
    post_done(a);
    if (a.trace) {
        __syncthreads();
        if (threadIdx.x == 0) a.trace[512 + blk] = __builtin_amdgcn_s_memrealtime();
    }
}

typedef void (*BlockKernel)(StreamArgs);
template <template <int> class K, int... I>
BlockKernel pick_impl(int qi, std::integer_sequence<int, I...>) {
    BlockKernel k = nullptr;
    ((qi == I + 1 ? (k = K<I + 1>::fn, 0) : 0), ...);
    return k;
}
template <int QI>
struct BlockK {
    static constexpr BlockKernel fn = stream_block_kernel<QI, false>;
};
template <int QI>
struct BlockKD {
    static constexpr BlockKernel fn = stream_block_kernel<QI, true>;
};
constexpr int kBlockWG = 2 * kCols + kSP / kOutN, kBlockWGD = 4 * kCols + kSP / kOutN;
template <int QI>
struct Prime2K {
    static constexpr BlockKernel fn = stream_prime2_kernel<QI>;
};
BlockKernel pick_block(int qi) { return pick_impl<BlockK>(qi, std::make_integer_sequence<int, 16>()); }
BlockKernel pick_block_d(int qi) { return pick_impl<BlockKD>(qi, std::make_integer_sequence<int, 16>()); }
BlockKernel pick_prime2(int qi) { return pick_impl<Prime2K>(qi, std::make_integer_sequence<int, 16>()); }


// Per-band responses r_n (band n's impulse response at pre = pin_n, no gain: the reference recurrence
// in the oracle's operation order, filterbank.h:178-179, as resp_h_kernel) in partition form, once per
// coefficient / pre-amp set when the first gain transient streams.  Past its first O + 1 samples r_n is
// homogeneous, so on partition p > 0 it is the zero-input response of its state there:
//     r_n[1024 p + j] = sum_k S_np[k] phi_nk[j],   phi_nk = the response from the unit state e_k,
// and the partition spectra are the same combination of phi_nk's spectra.  Stored per band:
//     r0 [N][1024]       partition 0 of r_n
//     phi[N][O][1024]    the homogeneous basis responses
//     st [N][Q][O]       S_np (state before sample 1024 p: y[1024 p - 1 - k]; row 0 unused)
//     sp [N][O + 1][33][32]  the column spectra of r0 and phi_nk (as stream_hs_kernel: / 2048)
// S_np is the state after the impulse's taps advanced by M^(1024 p - O - 1), the companion matrix's
// power in double-double (hz_dd.h).  Grid (N, 2): y = 0 runs r0 and the phi_nk (lanes 0 .. O), y = 1
// the states (lane p - 1).
template <int O>
__global__ __launch_bounds__(128) void stream_rbasis_kernel(const double* __restrict__ F, const double* __restrict__ B,
                                                            const double* __restrict__ pin, int Q,
                                                            double* __restrict__ r0, double* __restrict__ phi,
                                                            double* __restrict__ st) {
#pragma clang fp contract(off)
    using hz_dd::dd;
    const int t = threadIdx.x, band = blockIdx.x;
    double f[O + 1], b[O], y[O];
#pragma unroll
    for (int i = 0; i <= O; ++i) f[i] = F[(long)band * (O + 1) + i];
#pragma unroll
    for (int k = 0; k < O; ++k) {
        b[k] = B[(long)band * O + k];
        y[k] = 0.0;
    }
    const double pv = pin[band];
    auto step = [&](long tt, bool input) {
        double ff = 0.0;
        if (input) {
#pragma unroll
            for (int i = 0; i <= O; ++i)
                if (tt == i) ff = f[i];
        }
        double bs = 0.0;
#pragma unroll
        for (int k = 0; k < O; ++k) bs += b[k] * y[k];
        const double yt = ff * pv - bs;
#pragma unroll
        for (int k = O - 1; k >= 1; --k) y[k] = y[k - 1];
        y[0] = yt;
        return yt;
    };
    if (blockIdx.y == 0) {
        if (t > O) return;
        double* dst = t == 0 ? r0 + (long)band * kSP : phi + ((long)band * O + (t - 1)) * kSP;
        if (t > 0) {
#pragma unroll
            for (int k = 0; k < O; ++k) y[k] = k == t - 1 ? 1.0 : 0.0;
        }
        for (int j = 0; j < kSP; ++j) dst[j] = step(j, t == 0);
        return;
    }
    const int p = t + 1;
    if (p >= Q) return;
    for (long tt = 0; tt <= O; ++tt) (void)step(tt, true);
    dd M[O][O], P[O][O];
#pragma unroll
    for (int i = 0; i < O; ++i)
#pragma unroll
        for (int j = 0; j < O; ++j) M[i][j] = {i == 0 ? -b[j] : (j == i - 1 ? 1.0 : 0.0), 0.0};
    hz_dd::mat_pow<O>(M, (long)p * kSP - O - 1, P);
#pragma unroll
    for (int i = 0; i < O; ++i) {
        dd acc{0.0, 0.0};
#pragma unroll
        for (int j = 0; j < O; ++j) acc = hz_dd::add(acc, hz_dd::mul(P[i][j], y[j]));
        st[((long)band * Q + p) * O + i] = acc.hi;
    }
}

// sp[n][s][c][k2]: column c of series s of band n (s = 0: r0, s = 1 + k: phi_nk), grid (33, O + 1, N)
__global__ __launch_bounds__(kT) void stream_rspec_kernel(const double* __restrict__ r0, const double* __restrict__ phi,
                                                          int O, const double2* __restrict__ tw,
                                                          double2* __restrict__ sp) {
    __shared__ ColLds s;
    const int c = blockIdx.x, sr = blockIdx.y, band = blockIdx.z;
    const double* src = sr == 0 ? r0 + (long)band * kSP : phi + ((long)band * O + (sr - 1)) * kSP;
    col_forward(s, tw, c, [&](int n) { return n < kSP ? src[n] * (1.0 / kSF) : 0.0; },
                sp + (((long)band * (O + 1) + sr) * kCols + c) * 32);
}

// A gain setter's bands, in the kernel arguments with their new targets for d_gin (no host copy, no
// stream synchronisation); kChurnArg per launch
constexpr int kChurnArg = 24;
struct ChurnList {
    int m;
    int band[kChurnArg];
    double delta[kChurnArg];
    double gin[kChurnArg];
};
struct SetterArgs {
    // the per-band responses in partition form (stream_rbasis_kernel)
    const double* r0;
    const double* phi;
    const double* st;
    const double2* sp;
    long K;
    int Q, O;
    ChurnList L;          // the setter's bands (a longer list: one launch per kChurnArg bands)
    double rebase;        // s_g^(pos - dref): h_D's decay since the previous setter
    int dfirst;           // the first transient: h_D, its spectra and parities start from zero
    double* h;            // [K] the bank response
    double* hD;           // [K] the transient response
    double2* HS;          // [Q + 8][33][32] their partition spectra
    double2* HSD;
    const double2* ZS;    // the window spectra ring, slot of Z_{b-p}: ring_slot(head, p, Q)
    int head;
    const double2* tw;
    double2* C;           // [33][32] C_b, R_{b+1} as the next block launch reads them (prime2's
    double2* R;           // outputs), and h_D's
    double2* CD;
    double2* RD;
    // the smoothers' upkeep over the streamed samples (stream_upkeep_kernel), upkeep != 0
    int upkeep, N;
    double* pg;
    const double* pin;
    double* gin;
    double sp_m, sg_m;
    const double* line;
    long last;
    double* xhist;
    int skip;             // (diagnostic, HZ_SETTER_SKIP: bit 0 columns, 1 taps, 2 upkeep return at once)
    unsigned long long* trace;    // (diagnostic, HZ_STREAM_TRACE) [2][512]: every workgroup's start and end
};


// A gain setter as a transient, in ONE launch, by linearity (the transient algebra:
// fb_stream_gain_setter).  With d = sum_i delta_i r_{band_i} (the setter's bands in list order):
//   taps      h += d, h_D = rebase h_D - d                              (workgroups [33, 33 + K/256))
//   spectra   dS_p = sum_i delta_i (S_ip . Phi_i) (partition 0: the r0 spectra), HS_p += dS_p,
//             HS_D,p = rebase HS_D,p - dS_p                             (column workgroups [0, 33))
//   parities  the C_b / R_{b+1} the next block launch reads (stream_prime2_kernel's outputs) move by
//             the same MAC over the ring with dS: dY = sum_{p>=1} dS_p Z_{b-p}, C += inverse column(dY),
//             R += sum_{p>=3} dS_p Z_{b+1-p}; h_D's C_D = rebase C_D - inverse(dY), R_D likewise --
//             so no prime launch follows the setter
//   upkeep    the smoothers over the streamed samples toward the targets they ran with, then the
//             setter's new targets into gin (one thread reads and writes a band's)  (the last workgroups)
// QI = Q / 8 partitions per column thread (p = g + 8 i).
// Latency, not work, sets this launch's time (a handful of FMAs per operand): a load that waits for
// an earlier load's value costs a whole memory round trip (~1 us).  So every load that does not
// depend on the setter's bands is issued first, the bands' indices and weights come from the kernel
// arguments (uniform: scalar loads), and each batch of kSetBatch bands issues all of its operand loads
// before using any -- one round trip per batch.  (A first version with a band loop whose loads
// waited on the previous band's took 17-21 us.)
constexpr int kSetBatch = 12;
struct SetterLds {
    ColLds col;
    double S[kSetBatch * 128 * 4];          // the batch's states S_np, [band][p][k] (Q <= 128, O <= 4)
    double2 Ph[kSetBatch][5][32];           // the batch's spectra at this column (r0, phi_k)
};
// arr[i] for a uniform runtime i by a select chain (no dynamic indexing of registers)
template <class T>
__device__ __forceinline__ T pick24(const T (&arr)[kChurnArg], int i) {
    T v = arr[0];
#pragma unroll
    for (int e = 1; e < kChurnArg; ++e) v = i == e ? arr[e] : v;
    return v;
}
// (diagnostic) column workgroup c's phase times into trace[768 + 6 c + k]
#define COL_MARK(k)                                                                                      \
    if (a.trace && t == 0) a.trace[768 + 6 * c + (k)] = __builtin_amdgcn_s_memrealtime();
template <int QI>
__device__ __forceinline__ void setter_roles(const SetterArgs& a, SetterLds& u, const int vblk) {
    const int t = threadIdx.x;
    const int nt = (int)(a.K / kT);
    const int mq = a.L.m;
    const int O = a.O, Q = a.Q;
    // the band list with constant indices (wide scalar loads, one wait), picked by select chains
    int lb[kChurnArg];
#pragma unroll
    for (int e = 0; e < kChurnArg; ++e) lb[e] = a.L.band[e];
    if ((int)vblk >= kCols + nt) {   // upkeep
        if (a.skip & 4) return;
        const int b = (vblk - kCols - nt) * kT + t;
        if (b < a.N) {
            double gb = a.gin[b];
            if (a.upkeep) {
                const double P0 = a.pg[2 * b], G0 = a.pg[2 * b + 1], pb = a.pin[b];
                a.pg[2 * b] = pb + a.sp_m * (P0 - pb);
                a.pg[2 * b + 1] = gb + a.sg_m * (G0 - gb);
            }
#pragma unroll
            for (int i = 0; i < kChurnArg; ++i) {   // (unrolled: the list's scalar loads issued together)
                const bool hit = i < mq && lb[i] == b;
                gb = hit ? a.L.gin[i] : gb;
            }
            a.gin[b] = gb;
        }
        if (a.upkeep && b < O) a.xhist[b] = a.line[a.last - b];
        return;
    }
    if ((int)vblk >= kCols) {   // taps: 256 of partition tp (uniform over the workgroup)
        if (a.skip & 2) return;
        const long tau = (long)(vblk - kCols) * kT + t;
        const int tp = (int)(tau / kSP), tj = (int)(tau % kSP);
        const double hv = a.h[tau], hdv = a.dfirst ? 0.0 : a.hD[tau];
        double d = 0.0;
        constexpr int kTapBatch = 6;
        for (int q0 = 0; q0 < mq; q0 += kTapBatch) {
            long bl[kTapBatch];
            double dl[kTapBatch], v[kTapBatch][4], sv[kTapBatch][4];
#pragma unroll
            for (int e = 0; e < kTapBatch; ++e) {   // (past the list: the last band again, weight 0)
                const int q = min(q0 + e, mq - 1);
                bl[e] = pick24(lb, q);
                dl[e] = q0 + e < mq ? a.L.delta[q] : 0.0;
            }
#pragma unroll
            for (int e = 0; e < kTapBatch; ++e) {
                if (tp == 0) {
                    v[e][0] = a.r0[bl[e] * kSP + tj];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int kk = min(k, O - 1);
                        v[e][k] = a.phi[(bl[e] * O + kk) * kSP + tj];
                        sv[e][k] = a.st[(bl[e] * Q + tp) * O + kk];
                    }
                }
            }
#pragma unroll
            for (int e = 0; e < kTapBatch; ++e) {
                double wv = v[e][0];
                if (tp != 0) {
                    wv = 0.0;
#pragma unroll
                    for (int k = 0; k < 4; ++k) wv = fma(k < O ? sv[e][k] : 0.0, v[e][k], wv);
                }
                d = fma(dl[e], wv, d);
            }
        }
        a.h[tau] = hv + d;
        a.hD[tau] = a.dfirst ? -d : a.rebase * hdv - d;
        return;
    }
    // column c
    if (a.skip & 1) return;
    const int c = vblk, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    // everything that does not depend on the setter's bands, in flight first
    double2 z1[QI], z3[QI], hs[QI], hd[QI];
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        const int p = g + 8 * i;
        const long at = ((long)p * kCols + c) * 32 + j;
        z1[i] = a.ZS[((long)ring_slot(a.head, p, Q) * kCols + c) * 32 + j];   // Z_{b-p}
        z3[i] = a.ZS[((long)ring_slot(a.head, p > 0 ? p - 1 : 0, Q) * kCols + c) * 32 + j];   // Z_{b+1-p}
        hs[i] = a.HS[at];
        hd[i] = a.dfirst ? make_double2(0.0, 0.0) : a.HSD[at];
    }
    ColTw ct;
    ct.load(a.tw, c, j, g);
    const double2 tcol = a.tw[kTw2k + j * c];
    const int cat = c * 32 + (t & 31);
    const double2 zero2 = make_double2(0.0, 0.0);
    const double2 Cv = a.C[cat], Rv = a.R[cat];
    const double2 CDv = a.dfirst ? zero2 : a.CD[cat], RDv = a.dfirst ? zero2 : a.RD[cat];
    double2 dS[QI];
#pragma unroll
    for (int i = 0; i < QI; ++i) dS[i] = zero2;
    const int QO = Q * O, n2 = (O + 1) * 32;
    COL_MARK(0)
    for (int q0 = 0; q0 < ((a.skip & 8) ? 0 : mq); q0 += kSetBatch) {
        const int nb = min(kSetBatch, mq - q0), nS = nb * QO, nP = nb * n2;
        long bl[kSetBatch];
#pragma unroll
        for (int e = 0; e < kSetBatch; ++e) bl[e] = pick24(lb, min(q0 + e, mq - 1));
        // the batch's S rows and Ph columns into LDS: four of each per thread per round, every load of
        // a round issued before its stores (indices clamped: always valid)
        for (int e0 = 0; e0 < max(nS, nP); e0 += 4 * kT) {
            double sv[4];
            double2 pv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int e = e0 + t + r * kT;
                const int es = min(e, nS - 1), qs = es / QO;
                long bs = bl[0];
#pragma unroll
                for (int q = 1; q < kSetBatch; ++q) bs = qs == q ? bl[q] : bs;
                sv[r] = a.st[bs * QO + (es - qs * QO)];
                const int ep = min(e, nP - 1), qp = ep / n2, rest = ep - qp * n2;
                long bp = bl[0];
#pragma unroll
                for (int q = 1; q < kSetBatch; ++q) bp = qp == q ? bl[q] : bp;
                pv[r] = a.sp[((bp * (O + 1) + (rest >> 5)) * kCols + c) * 32 + (rest & 31)];
            }
            // (unconditional stores at the clamped indices -- past the batch they rewrite the last
            // element with its own value -- so no load is sunk into a conditional store's block
            // behind its own wait)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int e = e0 + t + r * kT;
                const int es = min(e, nS - 1), ep = min(e, nP - 1);
                u.S[es] = sv[r];
                (&u.Ph[0][0][0])[(ep / n2) * 5 * 32 + (ep % n2)] = pv[r];
            }
        }
        __syncthreads();
        COL_MARK(1)
        for (int qb = 0; qb < nb; ++qb) {
            // every LDS read of the band first (indices clamped to O - 1, masked below): one LDS
            // round trip per band, not one per term
            const double dq = a.L.delta[q0 + qb];
            double sk[QI][4];
            double2 ph[5];
#pragma unroll
            for (int k = 0; k < 5; ++k) ph[k] = u.Ph[qb][min(k, O)][j];
#pragma unroll
            for (int i = 0; i < QI; ++i)
#pragma unroll
                for (int k = 0; k < 4; ++k) sk[i][k] = u.S[qb * QO + (g + 8 * i) * O + min(k, O - 1)];
#pragma unroll
            for (int i = 0; i < QI; ++i) {
                double2 v = zero2;
                if (g + 8 * i == 0) {
                    v = ph[0];
                } else {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const double w = k < O ? sk[i][k] : 0.0;
                        v.x = fma(w, ph[1 + k].x, v.x);
                        v.y = fma(w, ph[1 + k].y, v.y);
                    }
                }
                dS[i].x = fma(dq, v.x, dS[i].x);
                dS[i].y = fma(dq, v.y, dS[i].y);
            }
        }
        __syncthreads();
    }
    COL_MARK(2)
    if (a.skip & 16) return;
    double2 y = zero2, r = zero2;
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        const int p = g + 8 * i;
        const long at = ((long)p * kCols + c) * 32 + j;
        a.HS[at] = cadd(hs[i], dS[i]);
        a.HSD[at] = make_double2(a.rebase * hd[i].x - dS[i].x, a.rebase * hd[i].y - dS[i].y);
        if (p >= 1) y = cadd(y, cmul(dS[i], z1[i]));
        if (p >= 3) r = cadd(r, cmul(dS[i], z3[i]));
    }
    COL_MARK(3)
    ColLds& s = u.col;
    y = half_sum(y);
    r = half_sum(r);
    if (l < 32) {
        s.m[w][j] = y;
        s.x[w][j] = r;
    }
    __syncthreads();
    if (t < 32) {
        s.y[t] = cadd(cadd(s.m[0][t], s.m[1][t]), cadd(s.m[2][t], s.m[3][t]));
        const double2 dr = cadd(cadd(s.x[0][t], s.x[1][t]), cadd(s.x[2][t], s.x[3][t]));
        a.R[cat] = cadd(Rv, dr);
        a.RD[cat] = make_double2(a.rebase * RDv.x - dr.x, a.rebase * RDv.y - dr.y);
    }
    __syncthreads();
    double2 cp = zero2;
#pragma unroll
    for (int q = 0; q < 4; ++q) cp = cadd(cp, cmulc(ct.t32[q], s.y[4 * g + q]));
    cp = half_sum(cp);
    if (l < 32) s.c[w][j] = cp;
    __syncthreads();
    if (t < 32) {
        const double2 dc = cmulc(tcol, cadd(cadd(s.c[0][t], s.c[1][t]), cadd(s.c[2][t], s.c[3][t])));
        a.C[cat] = cadd(Cv, dc);
        a.CD[cat] = make_double2(a.rebase * CDv.x - dc.x, a.rebase * CDv.y - dc.y);
    }
    COL_MARK(4)
}

template <int QI>
__global__ __launch_bounds__(kT) void stream_setter_kernel(SetterArgs a) {
    __shared__ SetterLds u;
    if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    setter_roles<QI>(a, u, (int)blockIdx.x);
    if (a.trace) {
        __syncthreads();
        if (threadIdx.x == 0) a.trace[512 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    }
}

// (A/B, HZ_SETTER_SPLIT=1) the taps and upkeep roles as a kernel of their own, without the column
// workgroups' LDS (the column kernel then runs kCols workgroups)
__global__ __launch_bounds__(kT) void stream_setter_taps_kernel(SetterArgs a) {
    extern __shared__ double no_lds[];
    if (a.trace && threadIdx.x == 0) a.trace[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    setter_roles<1>(a, *reinterpret_cast<SetterLds*>(no_lds), kCols + (int)blockIdx.x);
    if (a.trace) {
        __syncthreads();
        if (threadIdx.x == 0) a.trace[512 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    }
}

typedef void (*SetterKernel)(SetterArgs);
template <int... I>
SetterKernel pick_setter_impl(int qi, std::integer_sequence<int, I...>) {
    SetterKernel k = nullptr;
    ((qi == I + 1 ? (k = stream_setter_kernel<I + 1>, 0) : 0), ...);
    return k;
}
SetterKernel pick_setter(int qi) { return pick_setter_impl(qi, std::make_integer_sequence<int, 16>()); }

// line[i] = line[i + R] = src[i], i < n, from write position wpos
__global__ __launch_bounds__(256) void stream_put_kernel(const double* __restrict__ src, long n, double* __restrict__ line,
                                                         long R, long wpos) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    long k = wpos + i;
    if (k >= R) k -= R;
    const double v = src[i];
    line[k] = v;
    line[k + R] = v;
}

// dst[i] = line[s + i], i < n (contiguous thanks to the mirror)
__global__ __launch_bounds__(256) void stream_get_kernel(const double* __restrict__ line, long s, long n,
                                                         double* __restrict__ dst) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = line[s + i];
}

// the smoothers' closed form over the streamed samples and the x history (last O inputs)
__global__ __launch_bounds__(256) void stream_upkeep_kernel(double* __restrict__ pg, const double* __restrict__ pin,
                                                            const double* __restrict__ gin, int N, double sp_m,
                                                            double sg_m, const double* __restrict__ line, long last,
                                                            int O, double* __restrict__ xhist) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < N) {
        const double P0 = pg[2 * b], G0 = pg[2 * b + 1], pb = pin[b], gb = gin[b];
        pg[2 * b] = pb + sp_m * (P0 - pb);
        pg[2 * b + 1] = gb + sg_m * (G0 - gb);
    }
    if (b < O) xhist[b] = line[last - b];   // last = ring index + R of the newest sample
}

int s_alloc(double** p, size_t* cap, size_t need) {
    if (need <= *cap) return HZ_OK;
    if (*p) HZ_TRY_HIP(hipFree(*p));
    *p = nullptr;
    HZ_TRY_HIP(hipMalloc(p, need * sizeof(double)));
    *cap = need;
    return HZ_OK;
}

// the side stream's work on the ring done (before anything else reuses or rewrites it)
int tail_quiet(hz_fb::Resp::Stream& S) {
    if (S.side) HZ_TRY_HIP(hipStreamSynchronize(S.side));
    S.tail_async[0] = S.tail_async[1] = false;
    return HZ_OK;
}

// buffers for the current horizon
int stream_setup(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    const long K = R.K;
    const bool tail = K > kMaxK;
    const long K1 = tail ? kMaxK : K;
    // with a tail the ring also keeps the epoch before the oldest input a tail convolution reads
    const long ring = K + 2 * kSP + (tail ? kE : 0);
    if (S.R != ring) {   // a new horizon: the ring's contents no longer hold the history
        HZ_TRY(tail_quiet(S));
        S.R = ring;
        S.line_hist = false;
        S.fdl_valid = false;
        S.hs_gen = -1;
        S.head = 0;
        S.tail_launched = -1;
    }
    S.tail = tail;
    S.K1 = K1;
    const size_t lcap = S.line_cap;
    HZ_TRY(s_alloc(&S.d_line, &S.line_cap, (size_t)(2 * ring)));
    // never-written positions are zeros: a tail convolution's windows reach back past the history
    // (into outputs nobody reads), and a stale NaN there would spread through the window's FFT
    if (S.line_cap != lcap) HZ_TRY_HIP(hipMemset(S.d_line, 0, sizeof(double) * S.line_cap));
    if (tail) {
        HZ_TRY(s_alloc(&S.d_tout, &S.tout_cap, (size_t)(2 * kE)));
        if (!S.side) {
            HZ_TRY_HIP(hipStreamCreateWithFlags(&S.side, hipStreamNonBlocking));
            HZ_TRY_HIP(hipEventCreateWithFlags(&S.ev_main, hipEventDisableTiming));
            HZ_TRY_HIP(hipEventCreateWithFlags(&S.ev_tail[0], hipEventDisableTiming));
            HZ_TRY_HIP(hipEventCreateWithFlags(&S.ev_tail[1], hipEventDisableTiming));
        }
    }
    const size_t col = (size_t)kCols * 32 * 2;   // doubles per spectrum (33 columns x 32 bins)
    const size_t zcap = S.zs_cap, hcap = S.hs_cap;
    HZ_TRY(s_alloc(&S.d_ZS, &S.zs_cap, (size_t)(K1 / kSP) * col));
    HZ_TRY(s_alloc(&S.d_HS, &S.hs_cap, (size_t)(K1 / kSP + 8) * col));   // 8 zero rows past Q
    // zero rows (and never-written slots) must be exact zeros: the MAC multiplies them
    if (S.zs_cap != zcap) HZ_TRY_HIP(hipMemset(S.d_ZS, 0, sizeof(double) * S.zs_cap));
    if (S.hs_cap != hcap) HZ_TRY_HIP(hipMemset(S.d_HS, 0, sizeof(double) * S.hs_cap));
    if (!S.d_CR) {   // tail columns C and MAC sums R, two parities each
        HZ_TRY_HIP(hipMalloc(&S.d_CR, sizeof(double) * 4 * col));
        HZ_TRY_HIP(hipMemset(S.d_CR, 0, sizeof(double) * 4 * col));
    }
    if (!S.d_tw) {   // in long double
        std::vector<double2> tw(kTwN);
        const long double pi = acosl(-1.0L);
        auto root = [&](long m, long n) {
            const long double ang = -2.0L * pi * m / n;
            return make_double2((double)cosl(ang), (double)sinl(ang));
        };
        for (int m = 0; m < 64; ++m) tw[kTw64 + m] = root(m, 64);
        for (int m = 0; m < 32; ++m) tw[kTw32 + m] = root(m, 32);
        for (int m = 0; m < 1024; ++m) tw[kTw2k + m] = root(m, kSF);
        HZ_TRY_HIP(hipMalloc(&S.d_tw, sizeof(double2) * kTwN));
        HZ_TRY_HIP(hipMemcpy(S.d_tw, tw.data(), sizeof(double2) * kTwN, hipMemcpyHostToDevice));
    }
    return HZ_OK;
}

long ring_index(const hz_fb::Resp::Stream& S, long abs_pos) { return ((abs_pos % S.R) + S.R) % S.R; }

// the history (last K inputs) from the long engine's buffer into the ring
int hist_to_line(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    HZ_TRY(stream_setup(h));
    S.pos = R.K;
    if (R.run > 0)
        hipLaunchKernelGGL(stream_put_kernel, dim3((unsigned)((R.K + 255) / 256)), dim3(256), 0, h->stream,
                           (const double*)R.d_hist[R.hcur], R.K, S.d_line, S.R, 0L);
    HZ_TRY_HIP(hipGetLastError());
    S.line_hist = true;
    S.fdl_valid = false;
    return HZ_OK;
}

StreamArgs stream_args(hz_fb* h) {
    hz_fb::Resp::Stream& S = h->resp.st;
    StreamArgs a;
    a.x = nullptr;
    a.out = nullptr;
    a.line = S.d_line;
    a.R = S.R;
    a.wpos = ring_index(S, S.pos);
    a.prev = ring_index(S, S.pos - kSP);
    a.HS = (const double2*)S.d_HS;
    a.ZS = (double2*)S.d_ZS;
    a.Q = (int)(S.K1 / kSP);
    a.head = S.head;
    a.tw = (const double2*)S.d_tw;
    a.h = h->resp.d_h;
    // C_b in parity b, R_b in parity b (block counter blk): this launch reads C_b, R_{b+1} and
    // writes C_{b+1}, R_{b+2}
    const size_t col = (size_t)kCols * 32;
    double2* C = (double2*)S.d_CR;
    double2* Rb = C + 2 * col;
    const int b = (int)(S.blk & 1);
    a.Cin = C + b * col;
    a.Cout = C + (b ^ 1) * col;
    a.Rin = Rb + (b ^ 1) * col;
    a.Rout = Rb + b * col;
    a.flags = nullptr;
    a.seq = 0;
    a.tail2 = nullptr;
    a.HSD = nullptr;
    a.hD = nullptr;
    a.CDin = a.RDin = nullptr;
    a.CDout = a.RDout = nullptr;
    a.dscale = 0.0;
    a.sgpow = nullptr;
    a.trace = nullptr;
    return a;
}

// the D pass's operands: h_D's spectra and taps, its own C / R parities (same parity scheme)
void d_args(hz_fb* h, StreamArgs* a) {
    hz_fb::Resp::Stream& S = h->resp.st;
    const size_t col = (size_t)kCols * 32;
    double2* C = (double2*)S.d_CRD;
    double2* Rb = C + 2 * col;
    const int b = (int)(S.blk & 1);
    a->HSD = (const double2*)S.d_HSD;
    a->hD = S.d_hD;
    a->CDin = C + b * col;
    a->CDout = C + (b ^ 1) * col;
    a->RDin = Rb + (b ^ 1) * col;
    a->RDout = Rb + b * col;
    a->sgpow = S.d_sgpow;
}
// prime2 over h_D: the D fields in the main slots
StreamArgs d_as_main(const StreamArgs& a) {
    StreamArgs d = a;
    d.HS = a.HSD;
    d.h = a.hD;
    d.Cin = a.CDin;
    d.Cout = a.CDout;
    d.Rin = a.RDin;
    d.Rout = a.RDout;
    return d;
}

// the tail's contribution to the outputs of epoch e, out[i] = sum_{tau >= K1} h[tau] x[eE + i - tau]
// (i < kE), into slot e & 1: the long-call engine's convolution of the ring from position eE - K
int tail_issue(hz_fb* h, long e, hipStream_t st) {
    hz_fb::Resp::Stream& S = h->resp.st;
    const long p0 = e * kE - h->resp.K;
    return hz_fbi::fb_resp_tail_conv(h, S.d_line + ring_index(S, p0), kE, S.d_tout + (e & 1) * kE, st);
}

// before a block at position pos: the tail of its epoch is ready on the handle's stream, and the
// next epoch's convolution is issued on the side stream (its inputs are all older than K1 - kE
// samples before the epoch: written long ago; the main stream waits for it at the next epoch)
int tail_schedule(hz_fb* h) {
    hz_fb::Resp::Stream& S = h->resp.st;
    const long e = S.pos / kE;
    if (S.tail_launched < e) {   // (prime: this epoch's tail on the handle's stream)
        HZ_TRY(tail_issue(h, e, h->stream));
        S.tail_async[e & 1] = false;
        S.tail_launched = e;
    }
    if (S.tail_async[e & 1]) {
        HZ_TRY_HIP(hipStreamWaitEvent(h->stream, S.ev_tail[e & 1], 0));
        S.tail_async[e & 1] = false;
    }
    if (S.tail_launched < e + 1) {
        HZ_TRY_HIP(hipEventRecord(S.ev_main, h->stream));   // the ring's writes so far
        HZ_TRY_HIP(hipStreamWaitEvent(S.side, S.ev_main, 0));
        HZ_TRY(tail_issue(h, e + 1, S.side));
        HZ_TRY_HIP(hipEventRecord(S.ev_tail[(e + 1) & 1], S.side));
        S.tail_async[(e + 1) & 1] = true;
        S.tail_launched = e + 1;
    }
    return HZ_OK;
}

// (diagnostic, HZ_STREAM_TRACE=<file>) every streaming launch's workgroup start / end times
// (s_memrealtime, 100 MHz): launches are logged in a device buffer of kTraceN slots and appended to
// the file as {int32 kind (0 block, 1 block with a transient, 2 setter), int32 workgroups,
// uint64 start[512], uint64 end[512]} records when it fills and when the handle's stream state is freed
constexpr int kTraceN = 1024;
void trace_flush(hz_fb* h) {
    hz_fb::Resp::Stream& S = h->resp.st;
    if (!S.d_trace || S.trace_n == 0) return;
    std::vector<unsigned long long> buf((size_t)S.trace_n * 1024);
    if (hipStreamSynchronize(h->stream) == hipSuccess &&
        hipMemcpy(buf.data(), S.d_trace, sizeof(unsigned long long) * buf.size(), hipMemcpyDeviceToHost) == hipSuccess) {
        if (FILE* f = std::fopen(getenv("HZ_STREAM_TRACE"), "ab")) {
            for (int i = 0; i < S.trace_n; ++i) {
                const int hdr[2] = {S.trace_kind[i], S.trace_wg[i]};
                std::fwrite(hdr, sizeof(int), 2, f);
                std::fwrite(&buf[(size_t)i * 1024], sizeof(unsigned long long), 1024, f);
            }
            std::fclose(f);
        }
    }
    S.trace_n = 0;
}
unsigned long long* trace_slot(hz_fb* h, int kind) {
    static const bool on = getenv("HZ_STREAM_TRACE") != nullptr;
    if (!on) return nullptr;
    hz_fb::Resp::Stream& S = h->resp.st;
    if (!S.d_trace && hipMalloc(&S.d_trace, sizeof(unsigned long long) * kTraceN * 1024) != hipSuccess) return nullptr;
    if (S.trace_n == kTraceN) trace_flush(h);
    const int i = S.trace_n++;
    S.trace_kind[i] = kind;
    static const bool split = getenv("HZ_SETTER_SPLIT") && atoi(getenv("HZ_SETTER_SPLIT"));
    S.trace_wg[i] = kind == 3   ? (int)(S.K1 / kT + (h->N + kT - 1) / kT)
                    : kind == 2 ? (split ? kCols : (int)(kCols + S.K1 / kT + (h->N + kT - 1) / kT))
                                : (kind == 1 ? kBlockWGD : kBlockWG);
    return S.d_trace + (size_t)i * 1024;
}

}  // namespace

namespace hz_fbi {

int fb_stream_workgroups() { return kBlockWG; }

bool fb_stream_trackable(hz_fb* h, long n, bool conv) {
    hz_fb::Resp& R = h->resp;
    if (!R.st.on || n != kSP || R.mode == HZ_FB_RESP_OFF || !conv || h->order == 0 ||
        h->dist_id != HZ_DIST_NONE || h->path_mode != HZ_FB_PATH_AUTO || R.over_valid)
        return false;
    // the horizon (hz_fb_resp.hip resp_setup): computed once per coefficient set
    if (R.K == -2 && fb_resp_setup(h) != HZ_OK) return false;
    return R.K > 0 && R.K <= kMaxTailK;
}

bool fb_stream_eligible(hz_fb* h, long n, bool conv) {
    return fb_stream_trackable(h, n, conv) && h->resp.run >= h->resp.K;
}

int fb_launch_stream(hz_fb* h, const double* d_in, double* d_out, long n) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    if (S.dmode) {   // the transient has decayed below 2^-60 of the targets: plain streaming from here
        const double sd = (double)powl((long double)h->sg, (long double)(S.pos - S.dref));
        if (sd * S.dmax <= 0x1p-60 * S.gin_max) {
            fb_stream_dclear(h);   // the response is rebuilt for the long-call engine's spectra too
            h->converged = true;   // pre-amps converged at the first setter, gains now
        }
    }
    HZ_TRY(fb_resp_build(h));   // h (and the band-state operands) for the current bank
    HZ_TRY(stream_setup(h));
    const int Q = (int)(S.K1 / kSP);
    if (S.hs_gen != R.h_gen) {   // partition spectra of the current h
        // rows Q .. Q + 7 are read by the MAC roles and must be exact zeros; a shorter horizon than
        // the buffer was sized for leaves an older response's spectra there
        const size_t col = (size_t)kCols * 32 * 2;
        HZ_TRY_HIP(hipMemsetAsync(S.d_HS + (size_t)Q * col, 0, sizeof(double) * 8 * col, h->stream));
        hipLaunchKernelGGL(stream_hs_kernel, dim3(kCols, (unsigned)Q), dim3(kT), 0, h->stream, (const double*)R.d_h,
                           (const double2*)S.d_tw, (double2*)S.d_HS);
        HZ_TRY_HIP(hipGetLastError());
        if (S.tail) {
            HZ_TRY(tail_quiet(S));
            HZ_TRY(fb_resp_tail_spectra(h, S.K1));
            S.tail_launched = -1;
        }
        S.hs_gen = R.h_gen;
        S.gin_base = h->gin;   // the targets this h was built with (gain transients start from them)
        if (S.fdl_valid) S.prime_main = true;   // a rebuilt h with the ring still valid
    }
    if (!S.line_hist) HZ_TRY(hist_to_line(h));
    if (!S.fdl_valid) {   // the ring of window spectra, the first block's tail columns and R
        hipLaunchKernelGGL(stream_prime_kernel, dim3(kCols, (unsigned)(Q - 1)), dim3(kT), 0, h->stream, stream_args(h));
        HZ_TRY_HIP(hipGetLastError());
        S.blk = 1;   // prime2 writes as the launch before block 0 would: C_0 -> parity 0, R_1 -> parity 1
        hipLaunchKernelGGL(pick_prime2(Q / 8), dim3(kCols), dim3(kT), 0, h->stream, stream_args(h));
        HZ_TRY_HIP(hipGetLastError());
        S.blk = 0;
        S.fdl_valid = true;
        S.prime_main = false;
        S.prime_d = S.dmode;
    }
    // h changed (a gain transient, or a rebuild) with the ring still valid: C_b and R_{b+1} again, as
    // the launch before this block writes them; h_D's in the same launch (grid y = 2)
    const bool pm = S.prime_main, pd = S.dmode && S.prime_d;
    if (pm || pd) {
        const long blk = S.blk;
        S.blk = blk - 1;
        StreamArgs ap = stream_args(h);
        if (pd) d_args(h, &ap);   // (its parities from blk - 1 too)
        S.blk = blk;
        hipLaunchKernelGGL(pick_prime2(Q / 8), dim3(kCols, pm && pd ? 2 : 1), dim3(kT), 0, h->stream,
                           pm ? ap : d_as_main(ap));
        HZ_TRY_HIP(hipGetLastError());
        S.prime_main = S.prime_d = false;
    }
    if (S.tail) HZ_TRY(tail_schedule(h));
    StreamArgs a = stream_args(h);
    a.x = d_in;
    a.out = d_out;
    if (S.tail) a.tail2 = S.d_tout + ((S.pos / kE) & 1) * kE + (S.pos % kE);
    a.flags = S.flags_dev;   // set by hz_fb_process for its zero-copy call only
    a.seq = S.flags_seq;
    hipEvent_t* e = nullptr;
    if (h->prof) {
        HZ_TRY(fb_prof_events(h, &e));
        HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        h->ev_skip[(e - h->ev.data()) / 5] |= 2 | 8;
    }
    a.trace = trace_slot(h, S.dmode ? 1 : 0);
    if (S.dmode) {   // a gain transient: + s_g^(t - dref + 1) conv(h_D, x), its roles in the same launch
        d_args(h, &a);
        // (compute() smooths before the sample's output, filterbank.h:172-173: D is g(dref - 1) -
        // gin, so sample t carries s_g^(t - dref + 1))
        a.dscale = (double)powl((long double)h->sg, (long double)(S.pos - S.dref + 1));
        hipLaunchKernelGGL(pick_block_d(Q / 8), dim3(kBlockWGD), dim3(kT), 0, h->stream, a);
    } else {
        hipLaunchKernelGGL(pick_block(Q / 8), dim3(kBlockWG), dim3(kT), 0, h->stream, a);
    }
    HZ_TRY_HIP(hipGetLastError());
    if (e) {
        HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
        HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
        ++h->prof_launches;
    }
    S.pos += n;
    S.head = (S.head + 1) % Q;
    ++S.blk;
    S.pend += n;
    ++S.calls;
    R.implicit = true;
    R.run = std::min(R.run + n, 1L << 60);
    fb_mirror_advance(h, n);
    return HZ_OK;
}

// a short call on the per-band engines: the ring keeps the history while the bank could stream
int fb_stream_track(hz_fb* h, const double* d_in, long n, bool conv) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    S.fdl_valid = false;
    if (S.tail_launched >= 0) {   // streaming stops: its tail convolutions finish before the ring moves on
        HZ_TRY(tail_quiet(S));
        S.tail_launched = -1;
    }
    if (!fb_stream_trackable(h, n, conv)) {
        R.run = 0;
        fb_stream_dclear(h);
        return HZ_OK;
    }
    // a new horizon (coefficients changed: R.run restarted at 0) re-lays the ring out for it; the
    // samples tracked into the old layout are no longer history
    if (S.line_hist) HZ_TRY(stream_setup(h));
    if (!S.line_hist) {
        if (R.run > 0) {
            HZ_TRY(hist_to_line(h));
        } else {
            HZ_TRY(stream_setup(h));
            S.pos = R.K;   // nothing valid yet: run counts from here
            S.line_hist = true;
        }
    }
    hipLaunchKernelGGL(stream_put_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream, d_in, n, S.d_line,
                       S.R, ring_index(S, S.pos));
    HZ_TRY_HIP(hipGetLastError());
    S.pos += n;
    R.run = std::min(R.run + n, 1L << 60);
    return HZ_OK;
}

// the smoothers and x history after the streamed samples (pend), in place, toward the targets
// (d_pin / d_gin) the samples ran with: fb_upload calls it before new targets are uploaded
int fb_stream_upkeep(hz_fb* h) {
    hz_fb::Resp::Stream& S = h->resp.st;
    if (S.pend == 0) return HZ_OK;
    const double spm = (double)powl((long double)h->sp, (long double)S.pend);
    const double sgm = (double)powl((long double)h->sg, (long double)S.pend);
    const int N = h->N;
    hipLaunchKernelGGL(stream_upkeep_kernel, dim3((unsigned)((std::max(N, 64) + 255) / 256)), dim3(256), 0, h->stream,
                       h->d_pg[h->scur], (const double*)h->d_pin, (const double*)h->d_gin, N, spm, sgm,
                       (const double*)S.d_line, ring_index(S, S.pos - 1) + S.R, h->order, h->d_xhist[h->xcur]);
    HZ_TRY_HIP(hipGetLastError());
    S.pend = 0;
    return HZ_OK;
}

// band states (and smoothers / x history) from the ring: LAZY materialisation after streaming
int fb_stream_materialize(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    HZ_TRY(fb_stream_upkeep(h));
    HZ_TRY(fb_resp_build(h));
    return fb_state_window(h, S.d_line + ring_index(S, S.pos - R.K), R.K, h->d_ystate[h->scur], h->stream);
}

// before a long call: the history back into the long engine's buffer (the band states, if
// implicit, stay the zero-start response of the same K samples)
int fb_stream_to_hist(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    if (!S.line_hist) return HZ_OK;
    HZ_TRY(tail_quiet(S));
    S.tail_launched = -1;
    HZ_TRY(fb_stream_upkeep(h));
    if (R.run > 0) {
        HZ_TRY(fb_resp_setup(h));
        hipLaunchKernelGGL(stream_get_kernel, dim3((unsigned)((R.K + 255) / 256)), dim3(256), 0, h->stream,
                           (const double*)S.d_line, ring_index(S, S.pos - R.K), R.K, R.d_hist[R.hcur]);
        HZ_TRY_HIP(hipGetLastError());
    }
    S.line_hist = false;
    S.fdl_valid = false;
    return HZ_OK;
}

void fb_stream_reset(hz_fb* h) {
    fb_stream_dclear(h);
    hz_fb::Resp::Stream& S = h->resp.st;
    (void)tail_quiet(S);
    S.tail_launched = -1;
    S.pend = 0;
    S.line_hist = false;
    S.fdl_valid = false;
}

bool fb_stream_dmode(const hz_fb* h) { return h->resp.st.dmode; }

// leave the transient mode where the history stops (a call the ring does not stream, a reset): d_h
// still equals sum_n gin_n r_n up to roundoff, but the long-call engine's spectra were built before
// the setters -- rebuilt with the response when next needed
void fb_stream_dclear(hz_fb* h) {
    hz_fb::Resp::Stream& S = h->resp.st;
    if (!S.dmode && S.dsetters == 0) return;
    if (S.dmode || S.dsetters) h->resp.h_valid = false;
    S.dmode = false;
    S.dsetters = 0;
    S.prime_main = S.prime_d = false;
}

// A setter that changed only gains (mix / open) while the bank streams stationary: keep streaming.
// h += sum_n (gin'_n - gin_n) r_n, h_D = s_g^(pos - dref) h_D - (the same sum), dref = pos; both
// responses' spectra and the C / R parities of the next block move by linearity in the same launch
// (stream_setter_kernel, which also brings the smoothers up to date: fb_upload skips its upkeep).
// Returns 0: not applicable here (the caller invalidates the response as before); 1: applied, d_gin
// written by the update launch (no host copy, no synchronisation).
int fb_stream_gain_setter(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    const int N = h->N, O = h->order;
    if (!S.on || !S.line_hist || !S.fdl_valid || !R.h_valid || S.hs_gen != R.h_gen || R.run < R.K || R.over_valid ||
        S.tail || R.mode == HZ_FB_RESP_OFF || h->dist_id != HZ_DIST_NONE || h->path_mode != HZ_FB_PATH_AUTO || O == 0 ||
        (int)S.gin_base.size() != N)
        return 0;
    const long K = S.K1;
    if ((double)N * ((O + 1) * kSP + (double)(K / kSP) * O + (O + 1) * kCols * 64) * 8.0 > 8.0 * (1L << 30))
        return 0;   // the per-band responses stay <= 8 GiB
    if (!S.dmode) {
        // the first transient: pre-amps converged (boost() invalidates instead, so this holds until
        // the transient ends) and gains converged to gin_base (later setters: g_n(t) - gin_base_n =
        // s_g^(t - dref) D_n by construction)
        fb_mirror_sync(h);
        double pmax = 0, gmax = 0;
        for (int b = 0; b < N; ++b) {
            pmax = std::max(pmax, std::fabs(h->pin[b]));
            gmax = std::max(gmax, std::fabs(S.gin_base[b]));
        }
        for (int b = 0; b < N; ++b) {
            if (!(std::fabs(h->pg_host[2 * (size_t)b] - h->pin[b]) <= 0x1p-60 * pmax)) return 0;
            if (!(std::fabs(h->pg_host[2 * (size_t)b + 1] - S.gin_base[b]) <= 0x1p-60 * gmax)) return 0;
        }
    }
    // the setter's bands: one launch per kChurnArg of them (the updates add up; an all-band mix() of
    // the 4096-band bank takes 171 launches, under a millisecond)
    std::vector<ChurnList> lists;
    S.h_delta.clear();
    double dmx = 0;
    for (int b = 0; b < N; ++b) {
        const double d = h->gin[b] - S.gin_base[b];
        if (d != 0.0) {
            if (lists.empty() || lists.back().m == kChurnArg) {
                lists.emplace_back();
                lists.back().m = 0;
            }
            ChurnList& L = lists.back();
            L.band[L.m] = b;
            L.delta[L.m] = d;
            L.gin[L.m] = h->gin[b];
            ++L.m;
            S.h_delta.push_back((double)b);
            dmx = std::max(dmx, std::fabs(d));
        }
    }
    if (lists.empty()) return 1;
    const size_t col = (size_t)kCols * 32 * 2;
    const int Q = (int)(K / kSP);
    if (Q % 8 || Q / 8 > 16) return 0;   // (stream_setter_kernel: p = g + 8 i over QI = Q / 8)
    if (s_alloc(&S.d_r0, &S.r0_cap, (size_t)N * kSP) != HZ_OK ||
        s_alloc(&S.d_phi, &S.phi_cap, (size_t)N * O * kSP) != HZ_OK ||
        s_alloc(&S.d_st, &S.st_cap, (size_t)N * Q * O) != HZ_OK ||
        s_alloc(&S.d_rsp, &S.rsp_cap, (size_t)N * (O + 1) * col) != HZ_OK ||
        s_alloc(&S.d_hD, &S.hD_cap, (size_t)K) != HZ_OK)
        return 0;
    const size_t hcap = S.hsd_cap;
    if (s_alloc(&S.d_HSD, &S.hsd_cap, (size_t)(Q + 8) * col) != HZ_OK) return 0;   // rows past Q stay zero
    if (S.hsd_cap != hcap && hipMemset(S.d_HSD, 0, sizeof(double) * S.hsd_cap) != hipSuccess) return 0;
    if (!S.d_CRD && hipMalloc(&S.d_CRD, sizeof(double) * 4 * col) != hipSuccess) return 0;
    if (S.sgpow_of != h->sg) {
        std::vector<double> sp(kSP);
        for (int j = 0; j < kSP; ++j) sp[j] = (double)powl((long double)h->sg, (long double)j);
        if (!S.d_sgpow && hipMalloc(&S.d_sgpow, sizeof(double) * kSP) != hipSuccess) return 0;
        if (hipMemcpy(S.d_sgpow, sp.data(), sizeof(double) * kSP, hipMemcpyHostToDevice) != hipSuccess) return 0;
        S.sgpow_of = h->sg;
    }
    if (!S.rband_valid) {   // r_n at the current coefficients and pre-amps (R.d_coef: resp_build_h)
        const double* F = R.d_coef;
        const double* Bc = R.d_coef + (size_t)N * (O + 1);
        const dim3 g((unsigned)N, 2);
        const double* pin = h->d_pin;
        switch (O) {
        case 1: hipLaunchKernelGGL(stream_rbasis_kernel<1>, g, dim3(128), 0, h->stream, F, Bc, pin, Q, S.d_r0, S.d_phi, S.d_st); break;
        case 2: hipLaunchKernelGGL(stream_rbasis_kernel<2>, g, dim3(128), 0, h->stream, F, Bc, pin, Q, S.d_r0, S.d_phi, S.d_st); break;
        case 3: hipLaunchKernelGGL(stream_rbasis_kernel<3>, g, dim3(128), 0, h->stream, F, Bc, pin, Q, S.d_r0, S.d_phi, S.d_st); break;
        default: hipLaunchKernelGGL(stream_rbasis_kernel<4>, g, dim3(128), 0, h->stream, F, Bc, pin, Q, S.d_r0, S.d_phi, S.d_st); break;
        }
        hipLaunchKernelGGL(stream_rspec_kernel, dim3(kCols, (unsigned)(O + 1), (unsigned)N), dim3(kT), 0, h->stream,
                           (const double*)S.d_r0, (const double*)S.d_phi, O, (const double2*)S.d_tw, (double2*)S.d_rsp);
        if (hipGetLastError() != hipSuccess) return 0;
        S.rband_valid = true;
    }
    const bool dfirst = !S.dmode;
    const double rebase = dfirst ? 0.0 : (double)powl((long double)h->sg, (long double)(S.pos - S.dref));
    // the C / R parities the next block launch reads: the outputs of launch blk - 1 (as prime2)
    const long blk = S.blk;
    S.blk = blk - 1;
    StreamArgs ap = stream_args(h);
    d_args(h, &ap);
    S.blk = blk;
    SetterArgs sa{};
    sa.r0 = S.d_r0;
    sa.phi = S.d_phi;
    sa.st = S.d_st;
    sa.sp = (const double2*)S.d_rsp;
    sa.K = K;
    sa.Q = Q;
    sa.O = O;
    sa.rebase = rebase;
    sa.dfirst = dfirst ? 1 : 0;
    sa.h = R.d_h;
    sa.hD = S.d_hD;
    sa.HS = (double2*)S.d_HS;
    sa.HSD = (double2*)S.d_HSD;
    sa.ZS = (const double2*)S.d_ZS;
    sa.head = S.head;
    sa.tw = (const double2*)S.d_tw;
    sa.C = ap.Cout;
    sa.R = ap.Rout;
    sa.CD = ap.CDout;
    sa.RD = ap.RDout;
    sa.N = N;
    sa.pg = h->d_pg[h->scur];
    sa.pin = h->d_pin;
    sa.gin = h->d_gin;
    sa.line = S.d_line;
    sa.xhist = h->d_xhist[h->xcur];
    if (S.pend > 0) {   // fb_stream_upkeep's work, folded into the launch
        sa.upkeep = 1;
        sa.sp_m = (double)powl((long double)h->sp, (long double)S.pend);
        sa.sg_m = (double)powl((long double)h->sg, (long double)S.pend);
        sa.last = ring_index(S, S.pos - 1) + S.R;
        S.pend = 0;
    }
    static const int skip = getenv("HZ_SETTER_SKIP") ? atoi(getenv("HZ_SETTER_SKIP")) : 0;
    sa.skip = skip;
    sa.trace = trace_slot(h, 2);
    const unsigned wg = (unsigned)(kCols + K / kT + (N + kT - 1) / kT);
    for (size_t i = 0; i < lists.size(); ++i) {   // (later lists: h_D already rebased, upkeep done)
        sa.L = lists[i];
        if (i > 0) {
            sa.rebase = 1.0;
            sa.dfirst = 0;
            sa.upkeep = 0;
        }
        static const bool split = getenv("HZ_SETTER_SPLIT") && atoi(getenv("HZ_SETTER_SPLIT"));
        if (split) {
            SetterArgs st = sa;
            st.trace = trace_slot(h, 3);
            hipLaunchKernelGGL(stream_setter_taps_kernel, dim3(wg - kCols), dim3(kT), 0, h->stream, st);
            hipLaunchKernelGGL(pick_setter(Q / 8), dim3(kCols), dim3(kT), 0, h->stream, sa);
        } else {
            // (diagnostic, HZ_SETTER_TWICE=1: the same launch twice -- wrong results, the second
            // launch's trace shows the cost with its code and operands warm)
            static const bool twice = getenv("HZ_SETTER_TWICE") && atoi(getenv("HZ_SETTER_TWICE"));
            if (twice) {
                SetterArgs s1 = sa;
                s1.trace = trace_slot(h, 2);
                hipLaunchKernelGGL(pick_setter(Q / 8), dim3(wg), dim3(kT), 0, h->stream, s1);
            }
            hipLaunchKernelGGL(pick_setter(Q / 8), dim3(wg), dim3(kT), 0, h->stream, sa);
        }
    }
    if (hipGetLastError() != hipSuccess) return 0;
    S.dmax = rebase * S.dmax + dmx;
    S.dref = S.pos;
    S.dmode = true;
    // (the parities moved with the spectra: no prime; a prime already pending recomputes them from the
    // updated spectra anyway -- h_D's start exact at the first transient)
    if (dfirst) S.prime_d = false;
    ++S.dsetters;
    for (double b : S.h_delta) S.gin_base[(size_t)b] = h->gin[(size_t)b];
    S.gin_max = 0;
    for (double v : S.gin_base) S.gin_max = std::max(S.gin_max, std::fabs(v));
    return 1;
}

void fb_stream_free(hz_fb* h) {
    hz_fb::Resp::Stream& S = h->resp.st;
    (void)tail_quiet(S);
    trace_flush(h);
    if (S.d_trace) (void)hipFree(S.d_trace);
    S.d_trace = nullptr;
    for (double* p : {S.d_line, S.d_ZS, S.d_HS, S.d_CR, S.d_tw, S.d_tH, S.d_tZ, S.d_tY, S.d_tout, S.d_hD, S.d_HSD,
                      S.d_CRD, S.d_r0, S.d_phi, S.d_st, S.d_rsp, S.d_sgpow})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : {S.ev_main, S.ev_tail[0], S.ev_tail[1]})
        if (e) (void)hipEventDestroy(e);
    if (S.side) (void)hipStreamDestroy(S.side);
    const bool on = S.on;
    S = hz_fb::Resp::Stream();
    S.on = on;
}

}  // namespace hz_fbi

extern "C" {

int hz_fb_tune_stream(hz_fb* h, int enable) {
    if (!h) return HZ_E_INVALID;
    h->resp.st.on = enable != 0;
    return HZ_OK;
}

int hz_fb_stream_info(hz_fb* h, int* enabled, long* block, long* calls, int* history_in_ring) {
    if (!h) return HZ_E_INVALID;
    if (enabled) *enabled = h->resp.st.on ? 1 : 0;
    if (block) *block = kSP;
    if (calls) *calls = h->resp.st.calls;
    if (history_in_ring) *history_in_ring = h->resp.st.line_hist ? 1 : 0;
    return HZ_OK;
}

}  // extern "C"
