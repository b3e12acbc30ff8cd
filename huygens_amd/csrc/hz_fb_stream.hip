// hz_fb_stream.hip -- the stationary Filterbank<double> engine for streaming calls (one
// launch per 1024-sample block).
//
// The reference runs the bank inside a 1024-sample audio callback, one sample at a time
// (tests/resynthesis.cpp:33-42 -> src/filterbank.h:125-148).  Once the bank is stationary
// (hz_fb_resp.hip: converged for its horizon K), the block's mixdown is
//     out[t] = sum_{tau < K} h[tau] x[t - tau]
// and a block call runs here as ONE kernel launch: a uniformly partitioned overlap-save
// convolution with P = 1024-sample partitions (the call length) and F = 2048-point real
// transforms, whose frequency-domain delay line -- the spectra of the last Q = K / P windows --
// stays on the device between calls.  Each transform is split column-wise (four-step,
// n = 32 n1 + n2, k = k1 + 64 k2): workgroup c (c = 0..32) computes, straight from the samples,
// its 32 bins X[c + 64 k2] of the new window's spectrum, its 32 bins of the partition MAC
// Y = sum_p H_p Z_{b-p}, and its column of the inverse transform; it publishes that column
// (512 B, write-through stores) and adds to an arrival counter; the workgroup whose add comes
// last combines the 33 columns (Hermitian symmetry gives the other 31) into the block's 1024
// outputs.  tests/stream_model.py restates this algebra and is checked against a direct
// convolution on the CPU.
//
// Band states stay implicit (every mode): they are the zero-start response of the last K inputs,
// which the engine keeps in a mirrored device ring (every sample written at i and i + R, so any K
// consecutive samples are contiguous), and are computed by the band-state pass
// (hz_fb_state.hip) only when a later call, get_state, tick or a setter needs them.
#include <cstdio>
#include <utility>

#include "hz_fb_impl.h"

namespace {

constexpr int kSP = hz_fbi::kStreamBlock;   // partition = call length
constexpr int kSF = 2 * kSP;                // real transform length
constexpr int kCols = 33;                   // stored columns k1 = 0..32
constexpr int kT = 256;                     // threads per column workgroup
constexpr long kMaxK = 1L << 17;            // longest horizon streamed (Q <= 128 partitions)
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
template <class Load>
__device__ __forceinline__ void col_forward(ColLds& s, const double2* __restrict__ tw, int c, Load load,
                                            double2* __restrict__ dst) {
    const int t = threadIdx.x, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    double v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = load(32 * (g + 8 * i) + j);
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
    const double2* HS;    // [Q][33][32]
    double2* ZS;          // [Q][33][32] window spectra ring
    int Q, head;          // partitions; slot of this call's window (older windows: head - p mod Q)
    const double2* tw;
    double* xch;          // [33][32] complex: the published columns
    unsigned* count;      // arrival counter (0 between launches)
};

// The ring's windows b - p (p = 1 .. Q - 1) from the history: slot (head - p) mod Q <- the window
// [pos - P (p + 1), pos - P (p - 1)), grid (33, Q - 1)
__global__ __launch_bounds__(kT) void stream_prime_kernel(StreamArgs a) {
    __shared__ ColLds s;
    const int c = blockIdx.x, p = blockIdx.y + 1;
    long ws = a.wpos - (long)kSP * (p + 1);
    if (ws < 0) ws += a.R;
    const double* src = a.line + ws;   // contiguous: ws < R, ws + 2048 <= 2 R
    int slot = a.head - p;
    if (slot < 0) slot += a.Q;
    col_forward(s, a.tw, c, [&](int n) { return src[n]; }, a.ZS + ((long)slot * kCols + c) * 32);
}

// One 1024-sample block (see the file comment).  QI = Q / 8 partitions per thread.
template <int QI>
__global__ __launch_bounds__(kT) void stream_block_kernel(StreamArgs a) {
    __shared__ ColLds s;
    const int t = threadIdx.x, l = t & 63, w = t >> 6, j = l & 31, g = 2 * w + (l >> 5);
    const int c = blockIdx.x;
    // ---- every operand of the column in flight at once: the window (previous block from the
    // ring, this block from the caller), the partition spectra and the older windows' spectra of
    // the thread's partitions p = g + 8 i, the twiddles
    double v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = a.line[a.prev + 32 * (g + 8 * i) + j];
#pragma unroll
    for (int i = 4; i < 8; ++i) v[i] = a.x[32 * (g + 8 * i - 32) + j];
    double2 hv[QI], zv[QI];
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        const int p = g + 8 * i;
        hv[i] = a.HS[((long)p * kCols + c) * 32 + j];
        int slot = a.head - p;
        if (slot < 0) slot += a.Q;
        // p = 0 is this call's window (computed below); its slot holds a stale spectrum
        zv[i] = a.ZS[((long)slot * kCols + c) * 32 + j];
    }
    ColTw ct;
    ct.load(a.tw, c, j, g);
    const double2 tcol = a.tw[kTw2k + j * c];   // W_2048^(n2 c), n2 = j (inverse column twiddle)
    // the block's samples into the ring (both mirror positions) for the next calls
    if (c == 0) {
#pragma unroll
        for (int i = 4; i < 8; ++i) {
            const long k = a.wpos + 32 * (g + 8 * i - 32) + j;
            a.line[k] = v[i];
            a.line[k + a.R] = v[i];
        }
    }
    // ---- forward stage 1 + the MAC partial over the thread's older windows
    const double2 a1 = stage1(v, ct.t64);
    double2 mp = make_double2(0.0, 0.0);
#pragma unroll
    for (int i = 0; i < QI; ++i) {
        if (i == 0 && g == 0) continue;   // p = 0: the new window, added below
        mp = cadd(mp, cmul(hv[i], zv[i]));
    }
    mp = half_sum(mp);
    if (l < 32) {
        s.a[w][j] = a1;
        s.m[w][j] = mp;
    }
    __syncthreads();
    // ---- forward stage 3 -> X (this window's bins), Y = H_0 X + sum of the MAC partials
    const double2 xp = stage3(s, g, ct.t2k, ct.t32);
    if (l < 32) s.x[w][j] = xp;
    __syncthreads();
    if (t < 32) {
        const double2 X = cadd(cadd(s.x[0][t], s.x[1][t]), cadd(s.x[2][t], s.x[3][t]));
        a.ZS[((long)a.head * kCols + c) * 32 + t] = X;
        const double2 M = cadd(cadd(s.m[0][t], s.m[1][t]), cadd(s.m[2][t], s.m[3][t]));
        s.y[t] = cadd(M, cmul(hv[0], X));   // thread t < 32: g = 0, hv[0] = H_0
    }
    __syncthreads();
    // ---- inverse column: C[n2] = W_2048^(-n2 c) sum_k2 W_32^(-n2 k2) Y[k2]; the thread sums
    // k2 = 4 g + q (the forward's stage-3 twiddles, conjugated)
    double2 cp = make_double2(0.0, 0.0);
#pragma unroll
    for (int q = 0; q < 4; ++q) cp = cadd(cp, cmulc(ct.t32[q], s.y[4 * g + q]));
    cp = half_sum(cp);
    if (l < 32) s.c[w][j] = cp;
    __syncthreads();
    if (w == 0) {
        if (l < 32) {
            const double2 C = cmulc(tcol, cadd(cadd(s.c[0][l], s.c[1][l]), cadd(s.c[2][l], s.c[3][l])));
            // write-through (sc1) stores: the last workgroup reads them with sc1 loads, no fences
            double* dst = a.xch + 2 * (c * 32 + l);
            st_sc1(dst, C.x);
            st_sc1(dst + 1, C.y);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every store of this (only) storing wave
        if (l == 0) {
            const unsigned prev = __hip_atomic_fetch_add(a.count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s.last = prev == kCols - 1;
        }
    }
    __syncthreads();
    if (!s.last) return;
    // ---- last workgroup: the 33 columns (sc1 loads) and W_64 into LDS, then the outputs
    // out[32 m + n2] = C0 + (-1)^n1 C32 + 2 Re sum_{k1=1}^{31} W_64^(-n1 k1) C[k1], n1 = 32 + m
    {
        double* cl = &s.col[0][0].x;
        for (int i = t; i < kCols * 64; i += kT)
            cl[i] = ld_sc1(a.xch + i);
        if (t < 64) s.tw[t] = a.tw[kTw64 + t];
    }
    __syncthreads();
    if (t == 0) __hip_atomic_store(a.count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double c0 = s.col[0][j].x, c32 = s.col[32][j].x;
    double acc[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = 0.0;
#pragma unroll
    for (int k1 = 1; k1 < 32; ++k1) {
        const double2 C = s.col[k1][j];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int n1 = 32 + g + 8 * r;
            const double2 wv = s.tw[(n1 * k1) & 63];
            acc[r] = fma(wv.x, C.x, fma(wv.y, C.y, acc[r]));
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int m = g + 8 * r;
        const double sgn = (m & 1) ? -c32 : c32;   // (-1)^n1, n1 = 32 + m
        a.out[32 * m + j] = c0 + sgn + 2.0 * acc[r];
    }
}

typedef void (*BlockKernel)(StreamArgs);
template <int... I>
BlockKernel pick_block_impl(int qi, std::integer_sequence<int, I...>) {
    BlockKernel k = nullptr;
    ((qi == I + 1 ? (k = stream_block_kernel<I + 1>, 0) : 0), ...);
    return k;
}
BlockKernel pick_block(int qi) { return pick_block_impl(qi, std::make_integer_sequence<int, 16>()); }

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

// buffers for the current horizon
int stream_setup(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    const long K = R.K;
    const long ring = K + 2 * kSP;
    if (S.R != ring) {   // a new horizon: the ring's contents no longer hold the history
        S.R = ring;
        S.line_hist = false;
        S.fdl_valid = false;
        S.hs_gen = -1;
        S.head = 0;
    }
    HZ_TRY(s_alloc(&S.d_line, &S.line_cap, (size_t)(2 * ring)));
    const size_t spec = (size_t)(K / kSP) * kCols * 32 * 2;
    HZ_TRY(s_alloc(&S.d_ZS, &S.zs_cap, spec));
    HZ_TRY(s_alloc(&S.d_HS, &S.hs_cap, spec));
    if (!S.d_xch) HZ_TRY_HIP(hipMalloc(&S.d_xch, sizeof(double) * kCols * 64));
    if (!S.d_count) {
        HZ_TRY_HIP(hipMalloc(&S.d_count, sizeof(unsigned) * 64));
        HZ_TRY_HIP(hipMemset(S.d_count, 0, sizeof(unsigned) * 64));
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
    a.Q = (int)(h->resp.K / kSP);
    a.head = S.head;
    a.tw = (const double2*)S.d_tw;
    a.xch = S.d_xch;
    a.count = S.d_count;
    return a;
}

}  // namespace

namespace hz_fbi {

bool fb_stream_trackable(hz_fb* h, long n, bool conv) {
    hz_fb::Resp& R = h->resp;
    if (!R.st.on || n != kSP || R.mode == HZ_FB_RESP_OFF || !conv || h->order == 0 ||
        h->dist_id != HZ_DIST_NONE || h->path_mode != HZ_FB_PATH_AUTO || R.over_valid)
        return false;
    // the horizon (hz_fb_resp.hip resp_setup): computed once per coefficient set
    if (R.K == -2 && fb_resp_setup(h) != HZ_OK) return false;
    return R.K > 0 && R.K <= kMaxK;
}

bool fb_stream_eligible(hz_fb* h, long n, bool conv) {
    return fb_stream_trackable(h, n, conv) && h->resp.run >= h->resp.K;
}

int fb_launch_stream(hz_fb* h, const double* d_in, double* d_out, long n) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    HZ_TRY(fb_resp_build(h));   // h (and the band-state operands) for the current bank
    HZ_TRY(stream_setup(h));
    const int Q = (int)(R.K / kSP);
    if (S.hs_gen != R.h_gen) {   // partition spectra of the current h
        hipLaunchKernelGGL(stream_hs_kernel, dim3(kCols, (unsigned)Q), dim3(kT), 0, h->stream, (const double*)R.d_h,
                           (const double2*)S.d_tw, (double2*)S.d_HS);
        HZ_TRY_HIP(hipGetLastError());
        S.hs_gen = R.h_gen;
    }
    if (!S.line_hist) HZ_TRY(hist_to_line(h));
    if (!S.fdl_valid) {
        hipLaunchKernelGGL(stream_prime_kernel, dim3(kCols, (unsigned)(Q - 1)), dim3(kT), 0, h->stream, stream_args(h));
        HZ_TRY_HIP(hipGetLastError());
        S.fdl_valid = true;
    }
    StreamArgs a = stream_args(h);
    a.x = d_in;
    a.out = d_out;
    hipEvent_t* e = nullptr;
    if (h->prof) {
        HZ_TRY(fb_prof_events(h, &e));
        HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        h->ev_skip[(e - h->ev.data()) / 5] |= 2 | 8;
    }
    hipLaunchKernelGGL(pick_block(Q / 8), dim3(kCols), dim3(kT), 0, h->stream, a);
    HZ_TRY_HIP(hipGetLastError());
    if (e) {
        HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
        HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
        ++h->prof_launches;
    }
    S.pos += n;
    S.head = (S.head + 1) % Q;
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
    if (!fb_stream_trackable(h, n, conv)) {
        R.run = 0;
        return HZ_OK;
    }
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

// the smoothers and x history after the streamed samples (pend), in place
static int stream_upkeep(hz_fb* h) {
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
    HZ_TRY(stream_upkeep(h));
    HZ_TRY(fb_resp_build(h));
    return fb_state_window(h, S.d_line + ring_index(S, S.pos - R.K), R.K, h->d_ystate[h->scur], h->stream);
}

// before a long call: the history back into the long engine's buffer (the band states, if
// implicit, stay the zero-start response of the same K samples)
int fb_stream_to_hist(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    hz_fb::Resp::Stream& S = R.st;
    if (!S.line_hist) return HZ_OK;
    HZ_TRY(stream_upkeep(h));
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
    hz_fb::Resp::Stream& S = h->resp.st;
    S.pend = 0;
    S.line_hist = false;
    S.fdl_valid = false;
}

void fb_stream_free(hz_fb* h) {
    hz_fb::Resp::Stream& S = h->resp.st;
    for (double* p : {S.d_line, S.d_ZS, S.d_HS, S.d_xch})
        if (p) (void)hipFree(p);
    if (S.d_tw) (void)hipFree(S.d_tw);
    if (S.d_count) (void)hipFree(S.d_count);
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
