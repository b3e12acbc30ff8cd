// hz_fb_tv.hip -- Filterbank<double> with per-sample coefficient streams.
//
// Subtractive ALLINONE / ONEPERVOICE (src/subtractive.h:215-228, 300-317) retune every band
// in tick(), between samples, so the coefficients of Filterbank::compute (src/filterbank.h:
// 170-187) change every sample and neither the tiled scan of the general engine nor the
// converged engine applies: time is sequential per band.  One thread per band, one wave (64
// bands) per workgroup, the band's recurrence in registers:
//     pre  = (1 - sp) pin + sp pre;   gain = (1 - sg) gin + sg gain          (filterbank.h:172-173)
//     y_t  = (sum_k f_k(t) x_{t-k}) pre - sum_k b_k(t) y_{t-1-k}            (filterbank.h:178-179)
//     out_t = sum_bands [dist](y_t gain)                                    (filterbank.h:125-139)
// with the coefficients of sample t read from a stream in HBM:
//     HZ_FB_TV_COEFFS    [n][2O+1][N]  forward then back, band-minor (a wave reads 512 B rows)
//     HZ_FB_TV_RESONANT  [n][N] Hz     order 2: {g, 0, -g}, {-2 R cos(2 PI f / SR), R^2},
//                                      g = resonant(f, R) (subtractive.h:240-249), computed here.
// The handle's state (y history, smoothers, x history) is the general engine's, so calls of
// both kinds interleave freely.  The mix is summed like the heterodyne chain: 16-channel LDS
// runs, an xor tree per wave, then fixed strided slices of the per-wave rows.
// Algorithmic HBM traffic per band-sample: COEFFS 8 (2O+1) B (40 B at order 2); RESONANT 8 B.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hz_fb_impl.h"
#include "hz_rt.h"

// per-band arithmetic in the restatement's order, without FMA contraction
#pragma clang fp contract(off)

namespace {

using hz_fbi::kMaxOrder;

constexpr int kThreads = 64;              // bands per workgroup: one wave
constexpr int kCH = 16;                   // samples per LDS mix round
constexpr int kLanes = kThreads / kCH;    // lanes summing one sample
constexpr int kRunLen = kThreads / kLanes;
constexpr int kRun = kRunLen + 1;
constexpr int kRow = kLanes * kRun + 1;
constexpr long kPartBytes = 256L << 20;
constexpr int kMixSamples = 64, kMixSlices = 4;

struct TvArgs {
    const double* x;       // [n]
    const double* stream;  // see above
    const double* pin;     // [N]
    const double* gin;     // [N]
    const double* ystate;  // [N][O] y[-1-k] at call start
    const double* pg;      // [N][2] pre, gain at call start
    const double* xhist;   // [O] x[-1-k] at call start
    double* ystate_next;
    double* pg_next;
    double* xhist_next;
    double* part;          // [G][pstride]
    long n, pstride, stream_row;   // stream_row: doubles per sample row
    int N;
    double sp, sg, param, dist_param;
    int fasttrig;          // bounded-range sin / cos for 0 <= arg <= 2 PI (hz_rt.h); 0: libm (env HZ_FB_TV_LIBM=1)
};

// libgcc's __divdc3 (Smith's algorithm) for (a + ib) / (c + id)
__device__ __forceinline__ void cdiv(double a, double b, double c, double d, double& x, double& y) {
    if (fabs(c) < fabs(d)) {
        const double ratio = c / d, denom = (c * ratio) + d;
        x = ((a * ratio) + b) / denom;
        y = ((b * ratio) - a) / denom;
    } else {
        const double ratio = d / c, denom = (d * ratio) + c;
        x = ((b * ratio) + a) / denom;
        y = (b - (a * ratio)) / denom;
    }
}

// x / SR correctly rounded without the IEEE divide sequence: q = x RN(1/SR), then one FMA
// residual step (Markstein; x >= 0 normal here).  Equal to x / 48000.0 -- checked on the
// host (tests/cpp/divcheck.c: random exponents, no mismatch).
__device__ __forceinline__ double div_sr(double x) {
    constexpr double inv = 1.0 / hz::kSR;
    const double q = x * inv;
    return __builtin_fma(__builtin_fma(-q, (double)hz::kSR, x), inv, q);
}

// cdiv(1, 0, c, d): both quotients share the denominator, so one IEEE reciprocal r = RN(1/den)
// serves both: -1/den = -r exactly, and ratio/den is taken as RN(q0 + RN(ratio - den q0) r),
// q0 = RN(ratio r) (one FMA residual step).  Markstein's exactness theorem needs q0 within 1 ulp,
// which RN(ratio r) does not guarantee (up to ~1.5 ulp), so exactness is checked, not proven:
// tests/cpp/divcheck.c compares it bit for bit with the Smith quotient on random resonant()
// operands, generic operands and targeted hard cases (quotient mantissa near 2, reciprocal error
// near 1/2 ulp) -- no mismatch in ~1e9 trials.  The sign of a zero may differ; nothing sees it.
__device__ __forceinline__ void cdiv_one(double c, double d, double& x, double& y) {
    const bool lt = fabs(c) < fabs(d);
    const double ratio = lt ? c / d : d / c;
    const double den = lt ? (c * ratio) + d : (d * ratio) + c;
    const double r = 1.0 / den;
    const double q0 = ratio * r;
    const double q = __builtin_fma(__builtin_fma(-q0, den, ratio), r, q0);   // RN(ratio / den)
    x = lt ? q : r;
    y = lt ? -r : -q;
}

// subtractive.h:240-249
// cos / sincos of an angle: the bounded-range kernels (< 1 ulp, hz_rt.h) for 0 <= x <= 2 PI -- every
// audio frequency's 2 PI f / SR and 4 PI f / SR -- else libm
__device__ __forceinline__ double tv_cos(double x, bool fast) {
    return (fast && x >= 0.0 && x <= 6.2831853072) ? hz_rt::cos_0_2pi(x) : cos(x);
}
__device__ __forceinline__ void tv_sincos(double x, double* s, double* c, bool fast) {
    if (fast && x >= 0.0 && x <= 6.2831853072) hz_rt::sincos_0_2pi(x, s, c);
    else sincos(x, s, c);
}

__device__ __forceinline__ double resonant(double frequency, double Q, bool fast = false) {
    double s2, c2;
    tv_sincos(div_sr(4 * hz::kPI * frequency), &s2, &c2, fast);
    const double ir = 0.0 * s2 - 1.0 * 0.0, ii = 0.0 * 0.0 + 1.0 * s2;   // 1.0i * sine2
    const double dr = (Q - c2) - ir, di = -0.0 - ii;
    double qr, qi;
    cdiv_one(dr, di, qr, qi);
    const double mr = 1.0 / (Q - 1) - qr, mi = 0.0 - qi;
    return 1 / sqrt(hypot(mr, mi));
}

template <int O, int KIND, int DIST>
__global__ __launch_bounds__(kThreads) void fb_tv_kernel(TvArgs a) {
    __shared__ double buf[kCH * kRow];
    __shared__ double xs[kCH + kMaxOrder];   // x[t0 - O .. t0 + kCH - 1]
    const int tid = threadIdx.x;
    const long band = (long)blockIdx.x * kThreads + tid;
    const bool live = band < a.N;
    const long bb = live ? band : 0;
    double y[O > 0 ? O : 1];
#pragma unroll
    for (int k = 0; k < O; ++k) y[k] = a.ystate[bb * O + k];
    double pre = a.pg[2 * bb], gain = a.pg[2 * bb + 1];
    const double pin = a.pin[bb], gin = a.gin[bb];
    const double sp = a.sp, sg = a.sg;
    const double* srow = a.stream + bb;
    double* bcol = buf + (tid / kRunLen) * kRun + tid % kRunLen;
    for (long t0 = 0; t0 < a.n; t0 += kCH) {
        const int m = (int)min((long)kCH, a.n - t0);
        if (tid < kCH + O) {   // the chunk's inputs and the O before it
            const long i = t0 - O + tid;
            xs[tid] = i >= 0 ? (i < a.n ? a.x[i] : 0.0) : a.xhist[-i - 1];
        }
        __syncthreads();
        for (int j = 0; j < m; ++j) {
            const long t = t0 + j;
            double f[O + 1], b[O > 0 ? O : 1];
            if constexpr (KIND == HZ_FB_TV_COEFFS) {
                const double* row = srow + t * a.stream_row;
#pragma unroll
                for (int k = 0; k <= O; ++k) f[k] = row[(long)k * a.N];
#pragma unroll
                for (int k = 0; k < O; ++k) b[k] = row[(long)(O + 1 + k) * a.N];
            } else {   // HZ_FB_TV_RESONANT, O == 2
                const double fr = srow[t * a.stream_row];
                const double R = a.param;
                const double cosine = tv_cos(2 * hz::kPI * fr / hz::kSR, a.fasttrig != 0);
                const double g = resonant(fr, R, a.fasttrig != 0);
                f[0] = g;
                f[1] = 0;
                f[2] = -g;
                b[0] = -2 * R * cosine;
                b[1] = R * R;
            }
            pre = (1 - sp) * pin + sp * pre;
            gain = (1 - sg) * gin + sg * gain;
            double ff = f[0] * xs[j + O];
#pragma unroll
            for (int k = 1; k <= O; ++k) ff += f[k] * xs[j + O - k];
            double bsum = 0;
#pragma unroll
            for (int k = 0; k < O; ++k) bsum += b[k] * y[k];
            const double yn = ff * pre - bsum;
#pragma unroll
            for (int k = O - 1; k > 0; --k) y[k] = y[k - 1];
            if constexpr (O > 0) y[0] = yn;
            const double v = hz::dist_apply<DIST>(yn * gain, a.dist_param);
            bcol[j * kRow] = live ? v : 0.0;
        }
        __syncthreads();
        {
            const int j = tid / kLanes, p = tid % kLanes;
            double s = 0.0;
            if (j < m) {
                const double* row = buf + j * kRow + p * kRun;
#pragma unroll
                for (int k = 0; k < kRunLen; ++k) s += row[k];
            }
#pragma unroll
            for (int w = 1; w < kLanes; w <<= 1) s += __shfl_xor(s, w);
            if (p == 0 && j < m) a.part[blockIdx.x * a.pstride + t0 + j] = s;
        }
    }
    if (live) {
#pragma unroll
        for (int k = 0; k < O; ++k) a.ystate_next[band * O + k] = y[k];
        a.pg_next[2 * band] = pre;
        a.pg_next[2 * band + 1] = gain;
    }
    if (blockIdx.x == 0 && tid < O) {   // x[-1-k] for the next call
        const long i = a.n - 1 - tid;
        a.xhist_next[tid] = i >= 0 ? a.x[i] : a.xhist[-i - 1];
    }
}

// HZ_FB_TV_RESONANT, producer/consumer form.  The coefficients of sample t depend only on the
// frequency stream at t, not on the recurrence, so they are computed time-parallel: per
// workgroup of 64 bands, kResProd producer waves evaluate g = resonant(f, R) and
// b0 = -2 R cos(2 PI f / SR) for a kResTL-sample tile (kResPer samples each, stream loads
// issued together) into LDS, while wave 0 runs the band recurrence over the previous tile from
// LDS (three dependent FP64 ops per sample), and the first producer lanes sum the tile before
// that into the partial mix.  Three tiles in flight, double-buffered, one barrier per tile.
// The per-band arithmetic is fb_tv_kernel's, op for op; the mix order is the same.
constexpr int kResProd = 15;   // 16 waves per workgroup: 4 per SIMD to cover the libm latency
constexpr int kResPer = 2;
constexpr int kResTL = kResProd * kResPer;
static_assert(kResTL * kLanes <= 64 * kResProd, "mix lanes");
constexpr int kResThreads = 64 * (1 + kResProd);

template <int DIST>
__global__ __launch_bounds__(kResThreads) void fb_tv_res_kernel(TvArgs a) {
    constexpr int O = 2;
    __shared__ double gb[2][kResTL][kThreads];
    __shared__ double bb[2][kResTL][kThreads];
    __shared__ double xs[2][kResTL + O];
    __shared__ double vb[2][kResTL * kRow];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const long band = (long)blockIdx.x * kThreads + lane;
    const bool live = band < a.N;
    const long bb_ = live ? band : 0;
    const long ntiles = (a.n + kResTL - 1) / kResTL;
    if (wave == 0) {
        double y0 = a.ystate[bb_ * O], y1 = a.ystate[bb_ * O + 1];
        double pre = a.pg[2 * bb_], gain = a.pg[2 * bb_ + 1];
        const double pin = a.pin[bb_], gin = a.gin[bb_];
        const double sp = a.sp, sg = a.sg, b1 = a.param * a.param;
        const int vcol = (lane / kRunLen) * kRun + lane % kRunLen;
        for (long it = 0; it <= ntiles + 1; ++it) {
            if (it >= 1 && it - 1 < ntiles) {
                const int c = (int)((it - 1) & 1);
                const int m = (int)min((long)kResTL, a.n - (it - 1) * kResTL);
                const double* x = xs[c];
                double* v = vb[c] + vcol;
                for (int j = 0; j < m; ++j) {
                    const double g = gb[c][j][lane], b0 = bb[c][j][lane];
                    pre = (1 - sp) * pin + sp * pre;
                    gain = (1 - sg) * gin + sg * gain;
                    double ff = g * x[j + O];
                    ff += 0.0 * x[j + O - 1];
                    ff += -g * x[j];
                    double bsum = 0;
                    bsum += b0 * y0;
                    bsum += b1 * y1;
                    const double yn = ff * pre - bsum;
                    y1 = y0;
                    y0 = yn;
                    const double o = hz::dist_apply<DIST>(yn * gain, a.dist_param);
                    v[j * kRow] = live ? o : 0.0;
                }
            }
            __syncthreads();
        }
        if (live) {
            a.ystate_next[band * O] = y0;
            a.ystate_next[band * O + 1] = y1;
            a.pg_next[2 * band] = pre;
            a.pg_next[2 * band + 1] = gain;
        }
    } else {
        const int pw = wave - 1;
        const double R = a.param;
        const double* srow = a.stream + bb_;
        for (long it = 0; it <= ntiles + 1; ++it) {
            if (it < ntiles) {
                const int c = (int)(it & 1);
                const long t0 = it * kResTL;
                const int m = (int)min((long)kResTL, a.n - t0);
                double fr[kResPer];
#pragma unroll
                for (int i = 0; i < kResPer; ++i) {
                    const int j = pw * kResPer + i;
                    fr[i] = j < m ? srow[(t0 + j) * a.stream_row] : 0.0;
                }
#pragma unroll
                for (int i = 0; i < kResPer; ++i) {
                    const int j = pw * kResPer + i;
                    const double cosine = tv_cos(div_sr(2 * hz::kPI * fr[i]), a.fasttrig != 0);
                    const double g = resonant(fr[i], R, a.fasttrig != 0);
                    gb[c][j][lane] = g;
                    bb[c][j][lane] = -2 * R * cosine;
                }
                if (pw == kResProd - 1 && lane < kResTL + O) {   // x[t0 - O .. t0 + TL - 1]
                    const long i = t0 - O + lane;
                    xs[c][lane] = i >= 0 ? (i < a.n ? a.x[i] : 0.0) : a.xhist[-i - 1];
                }
            }
            if (it >= 2 && tid - 64 < kResTL * kLanes) {   // partial mix of tile it - 2
                const int r = tid - 64, j = r / kLanes, p = r % kLanes;
                const long t0 = (it - 2) * kResTL;
                const int m = (int)min((long)kResTL, a.n - t0);
                double s = 0.0;
                if (j < m) {
                    const double* row = vb[it & 1] + j * kRow + p * kRun;
#pragma unroll
                    for (int k = 0; k < kRunLen; ++k) s += row[k];
                }
#pragma unroll
                for (int w = 1; w < kLanes; w <<= 1) s += __shfl_xor(s, w);
                if (p == 0 && j < m) a.part[blockIdx.x * a.pstride + t0 + j] = s;
            }
            __syncthreads();
        }
    }
    if (blockIdx.x == 0 && tid < O) {   // x[-1-k] for the next call
        const long i = a.n - 1 - tid;
        a.xhist_next[tid] = i >= 0 ? a.x[i] : a.xhist[-i - 1];
    }
}

__global__ __launch_bounds__(kMixSamples* kMixSlices) void fb_tv_mix_kernel(const double* __restrict__ part,
                                                                          double* __restrict__ out, long n,
                                                                          long pstride, int G) {
    __shared__ double red[kMixSlices][kMixSamples];
    const int s = threadIdx.x % kMixSamples, sl = threadIdx.x / kMixSamples;
    const long t = (long)blockIdx.x * kMixSamples + s;
    double acc = 0.0;
    if (t < n) {
#pragma unroll 8
        for (int g = sl; g < G; g += kMixSlices) acc += part[g * pstride + t];
    }
    red[sl][s] = acc;
    __syncthreads();
    if (sl == 0 && t < n) {
        double mix = red[0][s];
#pragma unroll
        for (int k = 1; k < kMixSlices; ++k) mix += red[k][s];
        out[t] = mix;
    }
}

typedef void (*tv_fn)(TvArgs);

template <int O, int KIND>
tv_fn tv_pick_dist(int dist) {
    switch (dist) {
    case HZ_DIST_SOFTCLIP: return fb_tv_kernel<O, KIND, HZ_DIST_SOFTCLIP>;
    case HZ_DIST_SATURATE: return fb_tv_kernel<O, KIND, HZ_DIST_SATURATE>;
    case HZ_DIST_LIMITER: return fb_tv_kernel<O, KIND, HZ_DIST_LIMITER>;
    default: return fb_tv_kernel<O, KIND, HZ_DIST_NONE>;
    }
}

tv_fn tv_pick_res(int dist) {
    switch (dist) {
    case HZ_DIST_SOFTCLIP: return fb_tv_res_kernel<HZ_DIST_SOFTCLIP>;
    case HZ_DIST_SATURATE: return fb_tv_res_kernel<HZ_DIST_SATURATE>;
    case HZ_DIST_LIMITER: return fb_tv_res_kernel<HZ_DIST_LIMITER>;
    default: return fb_tv_res_kernel<HZ_DIST_NONE>;
    }
}

tv_fn tv_pick(int O, int kind, int dist) {
    if (kind == HZ_FB_TV_RESONANT) return tv_pick_res(dist);
    switch (O) {
    case 0: return tv_pick_dist<0, HZ_FB_TV_COEFFS>(dist);
    case 1: return tv_pick_dist<1, HZ_FB_TV_COEFFS>(dist);
    case 2: return tv_pick_dist<2, HZ_FB_TV_COEFFS>(dist);
    case 3: return tv_pick_dist<3, HZ_FB_TV_COEFFS>(dist);
    default: return tv_pick_dist<4, HZ_FB_TV_COEFFS>(dist);
    }
}

// host restatement of the resonant coefficients (the staged coefficients after a call)
void resonant_host(double f, double R, double* fwd, double* back) {
    const double c2 = std::cos(4 * hz::kPI * f / hz::kSR), s2 = std::sin(4 * hz::kPI * f / hz::kSR);
    const double ir = 0.0 * s2 - 1.0 * 0.0, ii = 0.0 * 0.0 + 1.0 * s2;
    const double dr = (R - c2) - ir, di = -0.0 - ii;
    double qr, qi;
    if (std::fabs(dr) < std::fabs(di)) {
        const double ratio = dr / di, denom = (dr * ratio) + di;
        qr = ((1.0 * ratio) + 0.0) / denom;
        qi = ((0.0 * ratio) - 1.0) / denom;
    } else {
        const double ratio = di / dr, denom = (di * ratio) + dr;
        qr = ((0.0 * ratio) + 1.0) / denom;
        qi = (0.0 - (1.0 * ratio)) / denom;
    }
    const double mr = 1.0 / (R - 1) - qr, mi = 0.0 - qi;
    const double g = 1 / std::sqrt(std::hypot(mr, mi));
    fwd[0] = g;
    fwd[1] = 0;
    fwd[2] = -g;
    back[0] = -2 * R * std::cos(2 * hz::kPI * f / hz::kSR);
    back[1] = R * R;
}

}  // namespace

namespace hz_fbi {

int fb_tv_materialize(hz_fb* h) {
    if (!h->tv_pending) return HZ_OK;
    HZ_TRY_HIP(hipEventSynchronize(h->tv_ev));
    const long N = h->N;
    const int O = h->order;
    const double* last = h->tv_row;
    for (long b = 0; b < N; ++b) {
        double* F = &h->F[(size_t)b * (O + 1)];
        double* B = O > 0 ? &h->B[(size_t)b * O] : nullptr;
        if (h->tv_kind == HZ_FB_TV_COEFFS) {
            for (int q = 0; q <= O; ++q) F[q] = last[(size_t)q * N + b];
            for (int q = 0; q < O; ++q) B[q] = last[(size_t)(O + 1 + q) * N + b];
        } else {
            resonant_host(last[b], h->tv_param, F, B);
        }
    }
    h->tv_pending = false;
    h->dirty_coef = true;
    return HZ_OK;
}

}  // namespace hz_fbi

extern "C" {

int hz_fb_process_tv_device(hz_fb* h, const double* d_in, double* d_out, size_t n, int kind,
                            const double* d_stream, double param) {
    if (!h) {
        hz::set_error("null hz_fb handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    const int O = h->order;
    if ((kind != HZ_FB_TV_COEFFS && kind != HZ_FB_TV_RESONANT) || (kind == HZ_FB_TV_RESONANT && O != 2)) {
        hz::set_error("hz_fb_process_tv: kind %d needs %s", kind,
                      kind == HZ_FB_TV_RESONANT ? "order 2" : "HZ_FB_TV_COEFFS or HZ_FB_TV_RESONANT");
        return HZ_E_INVALID;
    }
    if (n == 0) return HZ_OK;
    if (!d_in || !d_out || !d_stream) {
        hz::set_error("hz_fb_process_tv: null buffer");
        return HZ_E_INVALID;
    }
    if (h->rt.computed) {   // after operator() without tick(): the cached sample first (fb_rt_resolve)
        double y0 = 0;
        const int k = hz_fbi::fb_rt_resolve(h, &y0);
        if (k < 0) return k;
        double* pin0 = hz_fbi::fb_rt_cached_slot(h);
        *pin0 = y0;
        HZ_TRY_HIP(hipMemcpyAsync(d_out, pin0, sizeof(double), hipMemcpyHostToDevice, h->stream));
        const long row0 = kind == HZ_FB_TV_COEFFS ? (2 * O + 1) * (long)h->N : (long)h->N;
        ++d_in;
        ++d_out;
        d_stream += row0;
        if (--n == 0) return HZ_OK;
    }
    HZ_TRY(hz_fbi::fb_rt_stop(h));   // the state back from the per-sample engine
    // pin / gin.  This call's last row supersedes a pending one, and the stream kernel does not
    // read the staged coefficients, so their rebuild waits for the next plain call.
    h->tv_pending = false;
    const bool dirty_coef = h->dirty_coef;
    h->dirty_coef = false;
    const int up = hz_fbi::fb_upload_staged(h);
    h->dirty_coef = dirty_coef;
    HZ_TRY(up);
    HZ_TRY(hz_fbi::fb_resp_materialize(h));   // the stream kernel reads the band states
    hz_fbi::fb_resp_invalidate(h, true);      // and leaves other coefficients behind
    const long N = h->N, G = (N + kThreads - 1) / kThreads;
    const long chunk = std::max(1L, std::min(1L << 20, kPartBytes / (long)sizeof(double) / G));
    const long row = kind == HZ_FB_TV_COEFFS ? (2 * O + 1) * N : N;
    const long need = G * std::min((long)n, chunk);
    if ((size_t)need > h->partial_cap) {
        if (h->d_partial) HZ_TRY_HIP(hipFree(h->d_partial));
        h->d_partial = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_partial, sizeof(double) * need));
        h->partial_cap = need;
    }
    const tv_fn k = tv_pick(O, kind, h->dist_id);
    for (long off = 0; off < (long)n; off += chunk) {
        const long len = std::min(chunk, (long)n - off);
        const long pstride = std::min((long)n, chunk);
        TvArgs a;
        a.x = d_in + off;
        a.stream = d_stream + off * row;
        a.pin = h->d_pin;
        a.gin = h->d_gin;
        a.ystate = h->d_ystate[h->scur];
        a.pg = h->d_pg[h->scur];
        a.xhist = h->d_xhist[h->xcur];
        a.ystate_next = h->d_ystate[h->scur ^ 1];
        a.pg_next = h->d_pg[h->scur ^ 1];
        a.xhist_next = h->d_xhist[h->xcur ^ 1];
        a.part = h->d_partial;
        a.n = len;
        a.pstride = pstride;
        a.stream_row = row;
        a.N = (int)N;
        a.fasttrig = std::getenv("HZ_FB_TV_LIBM") ? 0 : 1;
        a.sp = h->sp;
        a.sg = h->sg;
        a.param = param;
        a.dist_param = h->dist_param;
        hipEvent_t* e = nullptr;
        if (h->prof) {
            HZ_TRY(hz_fbi::fb_prof_events(h, &e));
            HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
            HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
        }
        hipLaunchKernelGGL(k, dim3((unsigned)G), dim3(kind == HZ_FB_TV_RESONANT ? kResThreads : kThreads), 0,
                           h->stream, a);
        HZ_TRY_HIP(hipGetLastError());
        if (e) {
            HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
            HZ_TRY_HIP(hipEventRecord(e[3], h->stream));
        }
        hipLaunchKernelGGL(fb_tv_mix_kernel, dim3((unsigned)((len + kMixSamples - 1) / kMixSamples)),
                           dim3(kMixSamples * kMixSlices), 0, h->stream, (const double*)h->d_partial, d_out + off,
                           len, pstride, (int)G);
        HZ_TRY_HIP(hipGetLastError());
        if (e) {
            HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
            ++h->prof_launches;
        }
        h->scur ^= 1;
        h->xcur ^= 1;
        hz_fbi::fb_mirror_advance(h, len);
    }
    h->last_path = HZ_FB_PATH_GENERAL;
    h->spare_ok = n == 1;   // see hz_fb_tick
    // the coefficients last set (the stream's final row) stay staged for later calls: copied
    // back without blocking, turned into F/B by fb_tv_materialize when next needed
    if ((size_t)row > h->tv_row_cap) {
        if (h->tv_row) HZ_TRY_HIP(hipHostFree(h->tv_row));
        h->tv_row = nullptr;
        h->tv_row_cap = 0;
        HZ_TRY_HIP(hipHostMalloc(&h->tv_row, sizeof(double) * row, hipHostMallocDefault));
        h->tv_row_cap = row;
    }
    if (!h->tv_ev) HZ_TRY_HIP(hipEventCreateWithFlags(&h->tv_ev, hipEventDisableTiming));
    HZ_TRY_HIP(hipMemcpyAsync(h->tv_row, d_stream + ((long)n - 1) * row, sizeof(double) * row,
                              hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipEventRecord(h->tv_ev, h->stream));
    h->tv_pending = true;
    h->tv_kind = kind;
    h->tv_param = param;
    h->dirty_coef = true;
    h->converged = false;
    return HZ_OK;
}

int hz_fb_process_tv(hz_fb* h, const double* in, double* out, size_t n, int kind, const double* stream,
                     double param) {
    if (!h) {
        hz::set_error("null hz_fb handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    if (n == 0) return hz_fb_process_tv_device(h, nullptr, nullptr, 0, kind, nullptr, param);
    if (!in || !out || !stream) {
        hz::set_error("hz_fb_process_tv: null buffer");
        return HZ_E_INVALID;
    }
    const size_t row = kind == HZ_FB_TV_COEFFS ? (size_t)(2 * h->order + 1) * h->N : (size_t)h->N;
    double *d_x = nullptr, *d_y = nullptr, *d_s = nullptr;
    int rc = HZ_OK;
    if (hipMalloc(&d_x, sizeof(double) * n) != hipSuccess || hipMalloc(&d_y, sizeof(double) * n) != hipSuccess ||
        hipMalloc(&d_s, sizeof(double) * n * row) != hipSuccess) {
        hz::set_error("hz_fb_process_tv: device allocation failed (%zu stream doubles)", n * row);
        rc = HZ_E_ALLOC;
    }
    // (blocking copies: complete before the stream's kernel is enqueued, whatever engine and queue
    // the runtime uses for pageable sources)
    if (rc == HZ_OK && (hipStreamSynchronize(h->stream) != hipSuccess ||
                        hipMemcpy(d_x, in, sizeof(double) * n, hipMemcpyHostToDevice) != hipSuccess ||
                        hipMemcpy(d_s, stream, sizeof(double) * n * row, hipMemcpyHostToDevice) != hipSuccess)) {
        hz::set_error("hz_fb_process_tv: upload failed");
        rc = HZ_E_HIP;
    }
    if (rc == HZ_OK) rc = hz_fb_process_tv_device(h, d_x, d_y, n, kind, d_s, param);
    if (rc == HZ_OK &&
        (hipMemcpyAsync(out, d_y, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
         hipStreamSynchronize(h->stream) != hipSuccess)) {
        hz::set_error("hz_fb_process_tv: download failed");
        rc = HZ_E_HIP;
    }
    (void)hipStreamSynchronize(h->stream);
    for (double* p : {d_x, d_y, d_s})
        if (p) (void)hipFree(p);
    return rc;
}

}  // extern "C"
