// hz_het.hip -- the heterodyne bank chain of tests/harmbank.cpp:77-101 on MI355X (gfx950).
//
// Per sample x, for every channel i (src/oscbank.h, modbank.h, slidebank.h, rmsbank.h,
// latchbank.h, stickbank.h), then summed over channels (src/mixer.h:30-33):
//     m   = x a_i                                   Modbank(T, analysis())
//     s   = Slidebank stages q < order: new_q = (1 - r_i) in_q + r_i old_q,
//           in_0 = m, in_q = old_{q-1}; s = new_{order-1}           (slidebank.h:166-175)
//     e   = running sum of |s|^2 over `width` samples; rms = sqrt(e / width)  (rmsbank.h:49-58)
//     l   = s * engaged (armed / engaged hysteresis on rms)          (latchbank.h:75-95)
//     y   = (1 + rad)^so l - sum_k y[t-1-k] back_k                   (stickbank.h:179-195)
//     d   = z_i y;  mix += Re d                                      (Modbank, Mixer)
//     out = 2/PI atan(dry x + gain mix)                              (harmbank.cpp:78, wave.h:150)
//   then the active channels of both Oscbanks tick: z *= w; z /= (1 + |z|^2) / 2.
//
// Everything but the mix is a per-channel recurrence that is nonlinear (the oscillators'
// renormalisation, sqrt, the latch), so time stays sequential per channel and the chain is
// fused into one kernel with a thread per channel: the N-wide signal never leaves
// registers.  Per-channel arithmetic is written without FMA contraction in the reference's
// operation order, so every channel's state is bit-exact with the restatement
// (oracle/hz_oracle_het.c); only the channel sum's order differs (fixed and deterministic:
// 16-channel runs per LDS row, an xor tree of 4 runs per 64-channel group, then 4 strided
// slices of the groups in het_mix_kernel).
//
// Layout in HBM: channel state SoA [field][Np] (Np = channels rounded up to 64); the
// RMSbank history ring [width + 1][Np] (slot-major, so the 64 lanes of a wave read and
// write one contiguous 512 B row per sample); per-group partial mixes [G][chunk].
// Algorithmic traffic per channel-sample: the ring's one read + one write (16 B).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "hz_common.h"

// No FMA contraction anywhere in this file: the per-channel recurrences must round like the
// reference's separate multiplies and adds (bit-exact channel states).
#pragma clang fp contract(off)

namespace {

constexpr int kThreads = 64;     // channels per workgroup: one wave, one partial-mix row
constexpr int kCH = 16;          // samples per LDS mix round
constexpr int kLanes = kThreads / kCH;   // lanes summing one sample (4)
constexpr int kRunLen = kThreads / kLanes;   // channels per run (16)
constexpr int kRun = kRunLen + 1;        // LDS doubles per run (+1 pad: the runs start on different banks)
constexpr int kRow = kLanes * kRun + 1;  // LDS doubles per sample row (odd)
constexpr int kMaxOrder = 8;
constexpr int kMaxStick = 4;
constexpr int kDist = 4;         // ring-load prefetch distance (samples); needs width > kDist
constexpr long kPartBytes = 256L << 20;   // partial-mix slab cap

// SoA field indices (each Np doubles)
enum : int {
    F_ZAR, F_ZAI, F_WAR, F_WAI, F_ZSR, F_ZSI, F_WSR, F_WSI, F_RR, F_RI, F_RSUM,
    F_SLIDE,                             // 2 * kMaxOrder fields: stage q re, im
    F_STICK = F_SLIDE + 2 * kMaxOrder,   // 2 * kMaxStick fields
    F_COUNT = F_STICK + 2 * kMaxStick
};

struct HetArgs {
    const double* x;
    double* part;          // [G][pstride]
    double* st;            // SoA state
    double* ring;          // [W1][Np]
    const unsigned char* act;   // [2][Np] analysis, synthesis activity
    unsigned char* latch;       // [Np] bit 0 armed, bit 1 engaged
    long n, Np, pstride;
    int N;
    unsigned W1, r0;       // ring slots; write slot of the launch's first sample
    double lo, hi;         // thresh * ratio, thresh * (1 - ratio)
    double width, sgain;   // (double)width; pow(1 + rad, stick_order)
    double back[kMaxStick];
};

// The two quotients r / nrm and m / nrm share one reciprocal.  This is the f64 divide's own
// sequence (v_rcp + two Newton steps, q0 = n y, e = n - d q0, q = q0 + e y: what div_fmas
// computes when div_scale leaves its operands alone) with the reciprocal computed once.
// div_scale only rescales for exponents near the ends of the range and div_fixup only acts
// on 0 / inf / NaN divisors; nrm = (1 + |z w|^2) / 2 lies in [1/2, 3/2] (|z| <= 1, |w| = 1),
// so every quotient is the correctly rounded one the divide instruction sequence returns.
__device__ __forceinline__ double rcp_newton(double d) {
    const double y0 = __builtin_amdgcn_rcp(d);
    const double e0 = fma(-d, y0, 1.0);
    const double y1 = fma(y0, e0, y0);
    const double e1 = fma(-d, y1, 1.0);
    return fma(y1, e1, y1);
}

__device__ __forceinline__ double div_with(double n, double d, double y) {
    const double q0 = n * y;
    const double e = fma(-d, q0, n);
    return fma(e, y, q0);
}

__device__ __forceinline__ void osc_tick(double& zr, double& zi, double wr, double wi) {
    // oscbank.h:61-62 (Eigen's complex packet product: re = ar br - ai bi, im = ar bi + ai br)
    const double r = zr * wr - zi * wi, m = zr * wi + zi * wr;
    const double nrm = (1.0 + (r * r + m * m)) / 2;
#ifdef HZ_HET_PLAIN_DIV
    zr = r / nrm;
    zi = m / nrm;
#else
    const double y = rcp_newton(nrm);
    zr = div_with(r, nrm, y);
    zi = div_with(m, nrm, y);
#endif
}

// O Slidebank stages, S Stickbank taps (compile-time: only the live state occupies VGPRs);
// PREF: the ring read of sample t is issued kDist samples ahead (width > kDist)
template <int O, int S, bool PREF>
__global__ __launch_bounds__(kThreads, 24) void het_chain_kernel(HetArgs a) {
    __shared__ double buf[kCH * kRow];
    __shared__ double xs[kCH];
    const int tid = threadIdx.x;
    const long c = (long)blockIdx.x * kThreads + tid;
    const long Np = a.Np;
    double* st = a.st + c;
    double zar = st[F_ZAR * Np], zai = st[F_ZAI * Np];
    const double war = st[F_WAR * Np], wai = st[F_WAI * Np];
    double zsr = st[F_ZSR * Np], zsi = st[F_ZSI * Np];
    const double wsr = st[F_WSR * Np], wsi = st[F_WSI * Np];
    const double rr = st[F_RR * Np], ri = st[F_RI * Np];
    double rsum = st[F_RSUM * Np];
    double slr[O], sli[O], ykr[S], yki[S];
#pragma unroll
    for (int q = 0; q < O; ++q) {
        slr[q] = st[(F_SLIDE + 2 * q) * Np];
        sli[q] = st[(F_SLIDE + 2 * q + 1) * Np];
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {
        ykr[k] = st[(F_STICK + 2 * k) * Np];
        yki[k] = st[(F_STICK + 2 * k + 1) * Np];
    }
    const bool act_a = a.act[c] != 0, act_s = a.act[Np + c] != 0;
    bool armed = (a.latch[c] & 1) != 0, engaged = (a.latch[c] & 2) != 0;
    const bool live = c < a.N;
    const double cr = 1.0 - rr, ci = 0.0 - ri;   // std::complex(1, 0) - radii (slidebank.h:77)
    const double lo = a.lo, hi = a.hi, width = a.width, sgain = a.sgain;
    double* ring = a.ring + c;
    const unsigned W1 = a.W1;
    // write slot of sample t: (r0 - t) mod W1; read slot (the sample `width` ago): one less
    unsigned sw = a.r0;
    unsigned sr = sw == 0 ? W1 - 1 : sw - 1;
    double pre[kDist];
    if constexpr (PREF) {
#pragma unroll
        for (int d = 0; d < kDist; ++d) {
            pre[d] = ring[(long)sr * Np];   // slots are always in range; values past n are unused
            sr = sr == 0 ? W1 - 1 : sr - 1;
        }
    }
    double* bcol = buf + (tid / kRunLen) * kRun + tid % kRunLen;   // this channel's column
    for (long t0 = 0; t0 < a.n; t0 += kCH) {
        const int m = (int)min((long)kCH, a.n - t0);
        if (tid < m) xs[tid] = a.x[t0 + tid];
        __syncthreads();   // xs ready; the previous round's buf reads done
        for (int j = 0; j < m; ++j) {
            double old;
            if constexpr (PREF) {
                old = pre[0];
#pragma unroll
                for (int d = 0; d + 1 < kDist; ++d) pre[d] = pre[d + 1];
                pre[kDist - 1] = ring[(long)sr * Np];
            } else {
                old = ring[(long)sr * Np];
            }
            sr = sr == 0 ? W1 - 1 : sr - 1;
            const double x = xs[j];
            // modulators(x, analysis()) (modbank.h: T * complex)
            double inr = x * zar, ini = x * zai;
            // slidebank (sparse product, column order: (1 - r) in_q, then r old_q)
#pragma unroll
            for (int q = 0; q < O; ++q) {
                const double ar = cr * inr - ci * ini, ai = cr * ini + ci * inr;
                const double br = rr * slr[q] - ri * sli[q], bi = rr * sli[q] + ri * slr[q];
                inr = slr[q];
                ini = sli[q];
                slr[q] = ar + br;
                sli[q] = ai + bi;
            }
            const double sre = slr[O - 1], sim = sli[O - 1];
            // rmsbank: inputs(origin) = |s|^2; out = inputs(origin) - inputs(origin + width) + lastout
            const double a2 = sre * sre + sim * sim;
            ring[(long)sw * Np] = a2;
            sw = sw == 0 ? W1 - 1 : sw - 1;
            rsum = a2 - old + rsum;
            const double rms = sqrt(rsum / width);
            // latchbank(&rmsbank, signal)
            armed = armed || rms < lo;
            const bool t1 = engaged && rms < lo;
            const bool t2 = !engaged && rms > hi && armed;
            engaged = engaged && !t1;
            armed = armed && !t1;
            engaged = engaged || t2;
            const double eg = engaged ? 1.0 : 0.0;
            const double lr = sre * eg, li = sim * eg;
            // smoothbank: y = (1 + rad)^order l - block * back (back real, as complex b + 0i)
            double accr = 0.0, acci = 0.0;
#pragma unroll
            for (int k = 0; k < S; ++k) {
                const double pr = ykr[k] * a.back[k] - yki[k] * 0.0, pi = ykr[k] * 0.0 + yki[k] * a.back[k];
                accr = accr + pr;
                acci = acci + pi;
            }
            const double yr = sgain * lr - accr, yi = sgain * li - acci;
#pragma unroll
            for (int k = S - 1; k > 0; --k) {
                ykr[k] = ykr[k - 1];
                yki[k] = yki[k - 1];
            }
            ykr[0] = yr;
            yki[0] = yi;
            // demodulators(synthesis(), y); mixdown takes the real part
            const double dr = zsr * yr - zsi * yi;
            bcol[j * kRow] = live ? dr : 0.0;
            // analysis.tick(); synthesis.tick() (active channels only)
            if (act_a) osc_tick(zar, zai, war, wai);
            if (act_s) osc_tick(zsr, zsi, wsr, wsi);
        }
        __syncthreads();   // buf complete
        {
            const int j = tid / kLanes, p = tid % kLanes;   // kLanes lanes per sample: run p
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
    st[F_ZAR * Np] = zar;
    st[F_ZAI * Np] = zai;
    st[F_ZSR * Np] = zsr;
    st[F_ZSI * Np] = zsi;
    st[F_RSUM * Np] = rsum;
#pragma unroll
    for (int q = 0; q < O; ++q) {
        st[(F_SLIDE + 2 * q) * Np] = slr[q];
        st[(F_SLIDE + 2 * q + 1) * Np] = sli[q];
    }
#pragma unroll
    for (int k = 0; k < S; ++k) {
        st[(F_STICK + 2 * k) * Np] = ykr[k];
        st[(F_STICK + 2 * k + 1) * Np] = yki[k];
    }
    a.latch[c] = (unsigned char)((armed ? 1 : 0) | (engaged ? 2 : 0));
}

typedef void (*chain_fn)(HetArgs);

template <int O, int S>
constexpr chain_fn chain_pick(bool pref) {
    return pref ? het_chain_kernel<O, S, true> : het_chain_kernel<O, S, false>;
}

template <int S>
chain_fn chain_for_order(int order, bool pref) {
    switch (order) {
    case 1: return chain_pick<1, S>(pref);
    case 2: return chain_pick<2, S>(pref);
    case 3: return chain_pick<3, S>(pref);
    case 4: return chain_pick<4, S>(pref);
    case 5: return chain_pick<5, S>(pref);
    case 6: return chain_pick<6, S>(pref);
    case 7: return chain_pick<7, S>(pref);
    default: return chain_pick<8, S>(pref);
    }
}

chain_fn chain_kernel(int order, int sorder, bool pref) {
    switch (sorder) {
    case 1: return chain_for_order<1>(order, pref);
    case 2: return chain_for_order<2>(order, pref);
    case 3: return chain_for_order<3>(order, pref);
    default: return chain_for_order<4>(order, pref);
    }
}

// out[t] = limiter(dry x[t] + gain mix[t]); mix[t] = four strided slices of the group rows
// (g = sl mod 4, in order), added in slice order: fixed, deterministic.  64 samples x 4
// slices per block, so a launch has n / 64 blocks and each lane streams G / 4 rows.
constexpr int kMixSamples = 64, kMixSlices = 4;

__global__ __launch_bounds__(kMixSamples* kMixSlices) void het_mix_kernel(const double* __restrict__ x,
                                                                        const double* __restrict__ part,
                                                                        double* __restrict__ out, long n,
                                                                        long pstride, int G, double dry,
                                                                        double gain) {
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
        out[t] = hz::dist_apply<HZ_DIST_LIMITER>(dry * x[t] + gain * mix, 0.0);
    }
}

}  // namespace

struct hz_het {
    int N = 0, order = 1, sorder = 1, device = 0;
    long Np = 0, G = 0;
    unsigned width = 0, W1 = 1, r = 0;   // RMSbank origin (decrements per sample)
    double thresh = 0, ratio = 0, dry = 0, gain = 0, sgain = 1;
    double back[kMaxStick] = {};
    std::vector<double> w[2];             // host mirrors of the Oscbank frequencies (re, im interleaved)
    std::vector<unsigned char> act;       // [2][Np]
    bool w_dirty = false, act_dirty = false;
    double* d_st = nullptr;               // [F_COUNT][Np]
    double* d_ring = nullptr;             // [W1][Np]
    unsigned char* d_act = nullptr;       // [2][Np]
    unsigned char* d_latch = nullptr;     // [Np]
    double* d_part = nullptr;
    long chunk = 0;                       // samples per launch pair
    double *d_in = nullptr, *d_out = nullptr;
    size_t io_cap = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool prof = false;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    long launches = 0, channel_samples = 0;
};

namespace {

int het_check(hz_het* h) {
    if (!h) {
        hz::set_error("null hz_het handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    return HZ_OK;
}

// stickbank.h:197-217: coefficients of the monic polynomial with `order` roots at rad
void stick_coefficients(int order, double rad, double* back) {
    std::vector<double> c = {rad, 1.0};
    for (int deg = 2; deg <= order; ++deg) {
        std::vector<double> t(deg + 1, 0.0);
        for (int i = 0; i < deg; ++i) {
            t[i] += rad * c[i];
            t[i + 1] += c[i];
        }
        c = t;
    }
    for (int i = 0; i < order; ++i) back[i] = c[i];
}

int upload_field(hz_het* h, int f, const double* src) {
    HZ_TRY_HIP(hipMemcpyAsync(h->d_st + (long)f * h->Np, src, sizeof(double) * h->Np, hipMemcpyHostToDevice,
                              h->stream));
    return HZ_OK;
}

// push pending host-side changes (frequencies, activity) before a launch or readback
int het_flush(hz_het* h) {
    if (h->w_dirty) {
        std::vector<double> re(h->Np), im(h->Np);
        for (int b = 0; b < 2; ++b) {
            for (long i = 0; i < h->Np; ++i) {
                re[i] = h->w[b][2 * i];
                im[i] = h->w[b][2 * i + 1];
            }
            HZ_TRY(upload_field(h, b ? F_WSR : F_WAR, re.data()));
            HZ_TRY(upload_field(h, b ? F_WSI : F_WAI, im.data()));
        }
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // re/im are stack-owned
        h->w_dirty = false;
    }
    if (h->act_dirty) {
        HZ_TRY_HIP(hipMemcpyAsync(h->d_act, h->act.data(), 2 * h->Np, hipMemcpyHostToDevice, h->stream));
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        h->act_dirty = false;
    }
    return HZ_OK;
}

int het_setup(hz_het* h, int order, const double* radii) {
    if (order > kMaxOrder) {
        hz::set_error("Slidebank order %d > %d is not supported", order, kMaxOrder);
        return HZ_E_INVALID;
    }
    h->order = std::max(1, order);   // slidebank.h:65
    std::vector<double> re(h->Np, 0.0), im(h->Np, 0.0), zero(h->Np, 0.0);
    for (int i = 0; i < h->N; ++i) {
        re[i] = radii[2 * i];
        im[i] = radii[2 * i + 1];
    }
    HZ_TRY(upload_field(h, F_RR, re.data()));
    HZ_TRY(upload_field(h, F_RI, im.data()));
    for (int f = F_SLIDE; f < F_SLIDE + 2 * kMaxOrder; ++f) HZ_TRY(upload_field(h, f, zero.data()));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int ensure(double** p, size_t* cap, size_t n) {
    if (n <= *cap) return HZ_OK;
    if (*p) HZ_TRY_HIP(hipFree(*p));
    *p = nullptr;
    HZ_TRY_HIP(hipMalloc(p, n * sizeof(double)));
    *cap = n;
    return HZ_OK;
}

int het_run(hz_het* h, const double* d_in, double* d_out, long n) {
    if (n <= 0) return HZ_OK;
    HZ_TRY(het_flush(h));
    for (long c0 = 0; c0 < n; c0 += h->chunk) {
        const long m = std::min(h->chunk, n - c0);
        HetArgs a;
        a.x = d_in + c0;
        a.part = h->d_part;
        a.st = h->d_st;
        a.ring = h->d_ring;
        a.act = h->d_act;
        a.latch = h->d_latch;
        a.n = m;
        a.Np = h->Np;
        a.pstride = h->chunk;
        a.N = h->N;
        a.W1 = h->W1;
        a.r0 = h->r;
        a.lo = h->thresh * h->ratio;
        a.hi = h->thresh * (1 - h->ratio);
        a.width = (double)h->width;
        a.sgain = h->sgain;
        for (int k = 0; k < kMaxStick; ++k) a.back[k] = h->back[k];
        hipEvent_t* e = nullptr;
        if (h->prof) {
            if (h->ev_used + 2 > h->ev.size())
                for (int q = 0; q < 64; ++q) {
                    hipEvent_t ne;
                    HZ_TRY_HIP(hz::prof_event_create(&ne));
                    h->ev.push_back(ne);
                }
            e = &h->ev[h->ev_used];
            h->ev_used += 2;
            HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        }
        hipLaunchKernelGGL(chain_kernel(h->order, h->sorder, h->width > (unsigned)kDist), dim3((unsigned)h->G),
                           dim3(kThreads), 0, h->stream, a);
        HZ_TRY_HIP(hipGetLastError());
        if (e) {
            HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
            ++h->launches;
            h->channel_samples += (long)h->N * m;
        }
        hipLaunchKernelGGL(het_mix_kernel, dim3((unsigned)((m + kMixSamples - 1) / kMixSamples)),
                           dim3(kMixSamples * kMixSlices), 0, h->stream, d_in + c0,
                           (const double*)h->d_part, d_out + c0, m, h->chunk, (int)h->G, h->dry, h->gain);
        HZ_TRY_HIP(hipGetLastError());
        h->r = (unsigned)(((long)h->r - m % h->W1 + h->W1) % h->W1);
    }
    return HZ_OK;
}

}  // namespace

extern "C" {

int hz_het_create(int channels, int order, const double* radii, double thresh, double ratio, unsigned width,
                  int stick_order, double stick_rad, double dry, double gain, int device, hz_het** out) {
    if (!out || channels <= 0 || !radii || width == 0 || width > (1u << 24) || stick_order > kMaxStick ||
        order > kMaxOrder) {
        hz::set_error("hz_het_create: invalid arguments (channels > 0, radii, 0 < width <= 2^24, order <= %d, "
                      "stick_order <= %d)", kMaxOrder, kMaxStick);
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_het* h = new (std::nothrow) hz_het();
    if (!h) return HZ_E_ALLOC;
    h->N = channels;
    h->Np = ((long)channels + kThreads - 1) / kThreads * kThreads;
    h->G = h->Np / kThreads;
    h->device = device;
    h->width = width;
    h->W1 = width + 1;
    h->thresh = thresh;
    h->ratio = ratio;
    h->dry = dry;
    h->gain = gain;
    h->sorder = std::max(1, stick_order);
    h->sgain = std::pow(1 + stick_rad, h->sorder);
    stick_coefficients(h->sorder, stick_rad, h->back);
    for (int b = 0; b < 2; ++b) {
        h->w[b].assign(2 * h->Np, 0.0);
        for (long i = 0; i < h->Np; ++i) h->w[b][2 * i] = 1.0;   // setOnes
    }
    h->act.assign(2 * h->Np, 0);
    h->chunk = std::max(1L, std::min(1L << 20, kPartBytes / (long)sizeof(double) / h->G));
    if (const char* e = std::getenv("HZ_HET_CHUNK"))   // test hook: force launch splits
        h->chunk = std::max(1L, std::min(h->chunk, std::atol(e)));
    const size_t ring_bytes = sizeof(double) * (size_t)h->W1 * h->Np;
    bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMalloc(&h->d_st, sizeof(double) * F_COUNT * h->Np) == hipSuccess;
    ok = ok && hipMalloc(&h->d_ring, ring_bytes) == hipSuccess;
    ok = ok && hipMalloc(&h->d_act, 2 * h->Np) == hipSuccess;
    ok = ok && hipMalloc(&h->d_latch, h->Np) == hipSuccess;
    ok = ok && hipMalloc(&h->d_part, sizeof(double) * h->G * h->chunk) == hipSuccess;
    ok = ok && hipMemset(h->d_st, 0, sizeof(double) * F_COUNT * h->Np) == hipSuccess;
    ok = ok && hipMemset(h->d_ring, 0, ring_bytes) == hipSuccess;
    ok = ok && hipMemset(h->d_act, 0, 2 * h->Np) == hipSuccess;
    ok = ok && hipMemset(h->d_latch, 0, h->Np) == hipSuccess;
    if (!ok) {
        hz::set_error("hz_het_create: device allocation failed (ring %zu bytes)", ring_bytes);
        hz_het_destroy(h);
        return HZ_E_ALLOC;
    }
    h->own_stream = true;
    {   // phases and frequencies start at 1 (oscbank.h:44-45)
        std::vector<double> ones(h->Np, 1.0);
        int rc = HZ_OK;
        for (int f : {F_ZAR, F_WAR, F_ZSR, F_WSR})
            if (rc == HZ_OK) rc = upload_field(h, f, ones.data());
        if (rc == HZ_OK) rc = het_setup(h, order, radii);
        if (rc != HZ_OK) {
            hz_het_destroy(h);
            return rc;
        }
    }
    *out = h;
    return HZ_OK;
}

int hz_het_destroy(hz_het* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->d_st, (void*)h->d_ring, (void*)h->d_act, (void*)h->d_latch, (void*)h->d_part,
                    (void*)h->d_in, (void*)h->d_out})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_het_setup(hz_het* h, int order, const double* radii) {
    HZ_TRY(het_check(h));
    if (!radii) return HZ_E_INVALID;
    return het_setup(h, order, radii);
}

int hz_het_freqmod(hz_het* h, int bank, const int* index, const double* hz, int count) {
    HZ_TRY(het_check(h));
    if ((bank != 0 && bank != 1) || count < 0 || (count && (!index || !hz))) return HZ_E_INVALID;
    for (int k = 0; k < count; ++k) {
        const int i = index[k];
        if (0 <= i && i < h->N) {   // oscbank.h:51 (out-of-range indices ignored)
            // two libm calls as written (through pointers: a merged sincos can differ in the last bit)
            static double (*volatile cos_fn)(double) = ::cos;
            static double (*volatile sin_fn)(double) = ::sin;
            h->w[bank][2 * i] = cos_fn(2 * hz::kPI * hz[k] / hz::kSR);
            h->w[bank][2 * i + 1] = sin_fn(2 * hz::kPI * hz[k] / hz::kSR);
        }
    }
    h->w_dirty = h->w_dirty || count > 0;
    return HZ_OK;
}

int hz_het_activate(hz_het* h, int bank, const int* index, int count, int on) {
    HZ_TRY(het_check(h));
    if ((bank != 0 && bank != 1) || count < 0 || (count && !index)) return HZ_E_INVALID;
    for (int k = 0; k < count; ++k)
        if (0 <= index[k] && index[k] < h->N) h->act[bank * h->Np + index[k]] = on ? 1 : 0;
    h->act_dirty = h->act_dirty || count > 0;
    return HZ_OK;
}

int hz_het_open(hz_het* h, int bank, int on) {
    HZ_TRY(het_check(h));
    if (bank != 0 && bank != 1) return HZ_E_INVALID;
    for (int i = 0; i < h->N; ++i) h->act[bank * h->Np + i] = on ? 1 : 0;
    h->act_dirty = true;
    return HZ_OK;
}

int hz_het_process_device(hz_het* h, const double* d_in, double* d_out, size_t n) {
    HZ_TRY(het_check(h));
    if (n && (!d_in || !d_out)) return HZ_E_INVALID;
    return het_run(h, d_in, d_out, (long)n);
}

int hz_het_process(hz_het* h, const double* in, double* out, size_t n) {
    HZ_TRY(het_check(h));
    if (n && (!in || !out)) return HZ_E_INVALID;
    if (n == 0) return HZ_OK;
    size_t cap_in = h->io_cap, cap_out = h->io_cap;
    HZ_TRY(ensure(&h->d_in, &cap_in, n));
    HZ_TRY(ensure(&h->d_out, &cap_out, n));
    h->io_cap = std::min(cap_in, cap_out);
    HZ_TRY_HIP(hipMemcpyAsync(h->d_in, in, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
    HZ_TRY(het_run(h, h->d_in, h->d_out, (long)n));
    HZ_TRY_HIP(hipMemcpyAsync(out, h->d_out, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_het_state(hz_het* h, int what, double* dst) {
    HZ_TRY(het_check(h));
    if (!dst || what < 0 || what > HZ_HET_STATE_HISTORY) return HZ_E_INVALID;
    HZ_TRY(het_flush(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    const long N = h->N, Np = h->Np;
    auto field = [&](int f, std::vector<double>& v) -> int {
        v.resize(Np);
        HZ_TRY_HIP(hipMemcpy(v.data(), h->d_st + (long)f * Np, sizeof(double) * Np, hipMemcpyDeviceToHost));
        return HZ_OK;
    };
    std::vector<double> re, im;
    if (what == HZ_HET_STATE_ANALYSIS || what == HZ_HET_STATE_SYNTHESIS) {
        const int f = what == HZ_HET_STATE_ANALYSIS ? F_ZAR : F_ZSR;
        HZ_TRY(field(f, re));
        HZ_TRY(field(f + 1, im));
        for (long i = 0; i < N; ++i) {
            dst[2 * i] = re[i];
            dst[2 * i + 1] = im[i];
        }
    } else if (what == HZ_HET_STATE_SLIDE || what == HZ_HET_STATE_STICK) {
        const int K = what == HZ_HET_STATE_SLIDE ? h->order : h->sorder;
        const int f0 = what == HZ_HET_STATE_SLIDE ? F_SLIDE : F_STICK;
        for (int q = 0; q < K; ++q) {
            HZ_TRY(field(f0 + 2 * q, re));
            HZ_TRY(field(f0 + 2 * q + 1, im));
            for (long i = 0; i < N; ++i) {
                dst[(i * K + q) * 2] = re[i];
                dst[(i * K + q) * 2 + 1] = im[i];
            }
        }
    } else if (what == HZ_HET_STATE_RMS) {
        HZ_TRY(field(F_RSUM, re));
        std::memcpy(dst, re.data(), sizeof(double) * N);
    } else if (what == HZ_HET_STATE_LATCH) {
        std::vector<unsigned char> l(Np);
        HZ_TRY_HIP(hipMemcpy(l.data(), h->d_latch, Np, hipMemcpyDeviceToHost));
        for (long i = 0; i < N; ++i) {
            dst[2 * i] = (l[i] & 1) ? 1.0 : 0.0;
            dst[2 * i + 1] = (l[i] & 2) ? 1.0 : 0.0;
        }
    } else {   // history, newest first: slot (r + 1 + k) mod W1
        std::vector<double> row(Np);
        for (unsigned k = 0; k < h->width; ++k) {
            const long s = ((long)h->r + 1 + k) % h->W1;
            HZ_TRY_HIP(hipMemcpy(row.data(), h->d_ring + s * Np, sizeof(double) * Np, hipMemcpyDeviceToHost));
            for (long i = 0; i < N; ++i) dst[i * h->width + k] = row[i];
        }
    }
    return HZ_OK;
}

int hz_het_set_stream(hz_het* h, void* stream) {
    HZ_TRY(het_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) HZ_TRY_HIP(hipStreamDestroy(h->stream));
    h->stream = (hipStream_t)stream;
    h->own_stream = false;
    return HZ_OK;
}

int hz_het_synchronize(hz_het* h) {
    HZ_TRY(het_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_het_profile(hz_het* h, int enable) {
    HZ_TRY(het_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    h->prof = enable != 0;
    h->ev_used = 0;
    h->launches = 0;
    h->channel_samples = 0;
    return HZ_OK;
}

int hz_het_profile_read(hz_het* h, double* ms, long* launches, long* channel_samples) {
    HZ_TRY(het_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    double tot = 0.0;
    for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
        float t = 0.f;
        HZ_TRY_HIP(hipEventElapsedTime(&t, h->ev[i], h->ev[i + 1]));
        tot += t;
    }
    if (ms) *ms = tot;
    if (launches) *launches = h->launches;
    if (channel_samples) *channel_samples = h->channel_samples;
    h->ev_used = 0;
    h->launches = 0;
    h->channel_samples = 0;
    return HZ_OK;
}

}  // extern "C"
