// hz_bowl.hip -- Bowl<T> modal resonance bank for MI355X (gfx950).
//
// Replaces src/bowl.h:10-74:  s(n) = sum_i a_i pow(E, -d_i n/SR) form(f_i n/SR), n = the
// `phase` counter (T), reset by trigger(); fill(float*, bsize) writes float.
//
// Bowl<double>, form = cycle: every mode is a decaying phasor, so
//     a_i E^{-d_i n/SR} sin(2 PI f_i n/SR) = a_i Im(w_i^n),  w_i = E^{-d_i/SR} e^{i 2 PI f_i/SR}
// (the reference's own truncated PI), evaluated by rotation: lanes are TIME (16-sample
// chunks), a wave walks up to 64 modes per 1024-sample tile, chunk seeds from per-mode
// tables w^(16p), w^(256r), tile seeds z(t0) w^1024 kept in LDS; no transcendental in the
// loop.
// Bowl<float>, form = a Wave<float> lambda sin(2 PI p) (double in, float out): the
// reference rounds p = f n / SR and x = -d n / SR in float, which moves the phase by up to
// ulp(p)/2 (0.008 cycles at n ~ 5e5) -- that rounding is part of its output, so the float
// model is evaluated per mode-sample: float mul + correctly rounded float divide (FMA
// residual form, div_sr), then sin(2 PI p) in double with p split exactly as k + r
// (k = floor p), r folded to a quarter period and an odd polynomial (sin2pi_ref), rounded
// to float -- no library sin or IEEE divide sequence in the loop; the decay E^x uses a
// per-chunk exp seed and a per-sample factor (x's float rounding changes the term by
// < 2.5e-8 a_i).  The sum is kept in double (the reference rounds it to float after every
// mode; that accumulation differs by ~1e-7 relative, see tests).  The float counter
// saturates at 2^24 (phase++ stops incrementing), as in the reference.
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "hz_chain.h"
#include "hz_common.h"

namespace {

constexpr int kL = 16;
constexpr int kTile = 64 * kL;
constexpr int kWaves = 8;
constexpr int kMaxPerWave = 64;
constexpr int kPad = 66;
constexpr double kPiM = 3.141592653589793115997963468544185161590576171875;  // M_PI (double)

// per-mode record: a, W1 (2), T1[16] (32), T2[4] (8), WT (2), f, d, |w|  (48 doubles)
struct BRec {
    static constexpr int AMP = 0;
    static constexpr int W1 = 1;
    static constexpr int T1 = 3;
    static constexpr int T2 = T1 + 32;
    static constexpr int WT = T2 + 8;
    static constexpr int F = WT + 2;     // 45
    static constexpr int D = F + 1;      // 46
    static constexpr int R = D + 1;      // 47  per-sample decay factor E^{-d/SR}
    static constexpr int SIZE = 48;
};

struct BowlArgs {
    double* partial;  // [G][n_pad]
    long n, n_pad, seg_len;
    double n0;        // phase counter at call start
    int M, nseg, per_wave, is_float;
};

__device__ __forceinline__ void cmul(double ar, double ai, double br, double bi, double& cr, double& ci) {
    const double r = fma(ar, br, -ai * bi);
    const double i = fma(ar, bi, ai * br);
    cr = r;
    ci = i;
}

// x / 48000 correctly rounded (binary32) without the IEEE divide sequence: q = x * RN(1/SR),
// then one FMA residual step (Markstein).  Checked exhaustively against x / 48000.0f over all
// positive finite floats on the host: the only mismatches have subnormal quotients (x < 2^-110),
// and the phase / exponent arguments here are 0 or >= 20 * 1.
__device__ __forceinline__ float div_sr(float x) {
    const float inv = 1.0f / 48000.0f;
    const float q = x * inv;
    const float r = __builtin_fmaf(-q, 48000.0f, x);
    return __builtin_fmaf(r, inv, q);
}

// sin(2 PI p) in double for the reference's PI = 3.14159265359 (src/includes.h:30) and a float
// p >= 0: 2 PI p = 2 pi (p + p e) with e = PI / pi - 1, so with k = floor(p), r = p - k
// (exact) the value is sin(2 pi (r + p e)).  r is folded into [-1/4, 1/4] by exact float
// reflections (tracking the sign of the p e term), then an odd degree-11 polynomial in r
// (|error| < 1.4e-11) -- far below the float rounding that follows.
__device__ __forceinline__ double sin2pi_ref(float p) {
    constexpr double kE = 3.14159265359 / kPiM - 1.0;
    const float k = floorf(p);
    float u = p - k;                      // [0, 1), exact
    u = u >= 0.5f ? u - 1.0f : u;         // [-1/2, 1/2), exact
    // reflect |u| > 1/4 about +-1/2 (exact, Sterbenz); selects, not branches
    const bool refl = fabsf(u) > 0.25f;
    u = refl ? copysignf(0.5f, u) - u : u;
    const double y = fma(refl ? -kE : kE, (double)p, (double)u);   // revolutions, |y| <= 1/4 + 1e-7
    // sin(2 pi y) = y P(y^2), P a degree-5 least-squares (near-minimax) fit on |y| <= 1/4:
    // max |error| 1.35e-11
    const double z = y * y;
    double s = -14.337175761608114;
    s = fma(s, z, 42.000013938078347);
    s = fma(s, z, -76.703669216302146);
    s = fma(s, z, 81.605209465741268);
    s = fma(s, z, -41.341701930121658);
    s = fma(s, z, 6.2831853064884768);
    return y * s;
}

// float phase counter after t increments from n0 (saturates at 2^24)
__device__ __forceinline__ float phase_f(double n0, long t) {
    const double v = n0 + (double)t;
    return (float)(v < 16777216.0 ? v : 16777216.0);
}

__global__ __launch_bounds__(64 * kWaves) void bowl_mix_kernel(const double* __restrict__ rec, BowlArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* part = lds;                     // [W][16][66]
    double* zt = lds + kWaves * kL * kPad;  // [W][64][2]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p16 = lane & 15, r4 = lane >> 4;
    const int seg = blockIdx.y;
    const long seg_t0 = (long)seg * a.seg_len;
    const long seg_end = min(seg_t0 + a.seg_len, a.n);
    const int ntiles = (int)((seg_end - seg_t0 + kTile - 1) / kTile);
    const int first = (blockIdx.x * kWaves + wave) * a.per_wave;
    const int count = max(0, min(a.per_wave, a.M - first));
    double* myzt = zt + wave * (2 * kMaxPerWave);

    if (!a.is_float) {
        // tile-start phasors w^(n0 + seg_t0) by binary powering (n0: the phase counter)
        const unsigned long long e0 = (unsigned long long)(a.n0 + (double)seg_t0);
        for (int q = 0; q < count; ++q) {
            const double* rr = rec + (long)(first + q) * BRec::SIZE;
            double zr = 1.0, zi = 0.0, br = rr[BRec::W1], bi = rr[BRec::W1 + 1];
            for (unsigned long long e = e0; e > 0; e >>= 1) {
                if (e & 1) cmul(zr, zi, br, bi, zr, zi);
                cmul(br, bi, br, bi, br, bi);
            }
            if (lane == 0) {
                myzt[2 * q] = zr;
                myzt[2 * q + 1] = zi;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }

    for (int tile = 0; tile < ntiles; ++tile) {
        const long t0 = seg_t0 + (long)tile * kTile;
        const long tc = t0 + (long)kL * lane;
        double acc[kL];
#pragma unroll
        for (int j = 0; j < kL; ++j) acc[j] = 0.0;
        if (!a.is_float) {
            for (int q = 0; q < count; ++q) {
                const double* rr = rec + (long)(first + q) * BRec::SIZE;
                const double sr = myzt[2 * q], si = myzt[2 * q + 1];
                double nr, ni;
                cmul(sr, si, rr[BRec::WT], rr[BRec::WT + 1], nr, ni);
                if (lane == 0) {
                    myzt[2 * q] = nr;
                    myzt[2 * q + 1] = ni;
                }
                __builtin_amdgcn_wave_barrier();
                double ur, ui, zr, zi;
                cmul(rr[BRec::T1 + 2 * p16], rr[BRec::T1 + 2 * p16 + 1], rr[BRec::T2 + 2 * r4],
                     rr[BRec::T2 + 2 * r4 + 1], ur, ui);
                cmul(sr, si, ur, ui, zr, zi);
                const double amp = rr[BRec::AMP], wr = rr[BRec::W1], wi = rr[BRec::W1 + 1];
#pragma unroll
                for (int j = 0; j < kL; ++j) {
                    acc[j] = fma(amp, zi, acc[j]);
                    cmul(zr, zi, wr, wi, zr, zi);
                }
            }
        } else {
            // the float phase counter of the chunk's samples (mode-independent)
            float ph[kL];
#pragma unroll
            for (int j = 0; j < kL; ++j) ph[j] = phase_f(a.n0, tc + j);
            for (int q = 0; q < count; ++q) {
                const double* rr = rec + (long)(first + q) * BRec::SIZE;
                const float fq = (float)rr[BRec::F], dq = (float)rr[BRec::D], aq = (float)rr[BRec::AMP];
                // decay magnitude: exp seed at the chunk start (from the float exponent, as
                // the reference), advanced by E^{-d/SR} per sample
                const float x0 = div_sr(-dq * ph[0]);
                double amag = (double)aq * exp((double)x0);
                const double rstep = rr[BRec::R];
#pragma unroll
                for (int j = 0; j < kL; ++j) {
                    const float p = div_sr(fq * ph[j]);   // float mul, correctly rounded float divide
                    const float wv = (float)sin2pi_ref(p);  // Wave<float>: sin in double, float out
                    acc[j] = fma(amag, (double)wv, acc[j]);
                    amag *= rstep;
                }
            }
        }
        double* my = part + wave * (kL * kPad);
#pragma unroll
        for (int j = 0; j < kL; ++j) my[j * kPad + lane] = acc[j];
        __syncthreads();
        for (int tl = threadIdx.x; tl < kTile; tl += blockDim.x) {
            const int src = tl >> 4, j = tl & 15;
            double s0 = 0.0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) s0 += part[w * (kL * kPad) + j * kPad + src];
            const long t = t0 + tl;
            if (t < a.n) a.partial[(long)blockIdx.x * a.n_pad + t] = s0;
        }
        __syncthreads();
    }
}

template <typename OutT>
__global__ __launch_bounds__(256) void bowl_reduce_kernel(const double* __restrict__ partial, long n_pad, int G,
                                                          long n, OutT* __restrict__ out) {
    __shared__ double red[4][64];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const long t = (long)blockIdx.x * 64 + tx;
    double s = 0.0;
    if (t < n)
        for (int g = ty; g < G; g += 4) s += partial[(long)g * n_pad + t];
    red[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && t < n) out[t] = (OutT)((red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]));
}

// short calls (a streamed 1024-sample block): 16 row slices per 64 samples, the loads of a
// slice issued 8 at a time, then a fixed-order LDS sum over the slices
constexpr int kShortSlices = 16;
constexpr long kShortMax = 16384;

template <typename OutT>
__global__ __launch_bounds__(64 * kShortSlices) void bowl_reduce_short_kernel(const double* __restrict__ partial,
                                                                              long n_pad, int G, long n,
                                                                              OutT* __restrict__ out) {
    __shared__ double red[kShortSlices][64];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const long t = (long)blockIdx.x * 64 + tx;
    double s = 0.0;
    if (t < n) {
        const double* col = partial + t;
        int g = ty;
        for (; g + 7 * kShortSlices < G; g += 8 * kShortSlices) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = col[(long)(g + u * kShortSlices) * n_pad];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += v[u];
        }
        for (; g < G; g += kShortSlices) s += col[(long)g * n_pad];
    }
    red[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && t < n) {
        double m = red[0][tx];
#pragma unroll
        for (int k = 1; k < kShortSlices; ++k) m += red[k][tx];
        out[t] = (OutT)m;
    }
}

// ---- Bowl<float>::fill into a Delaybank<float> in one launch (hz_chain.h) ----------------------
// A workgroup owns kChainSpw consecutive samples: the float modal model of every mode for them
// (bowl_mix_kernel's per-sample arithmetic, the decay seeded at the workgroup's first sample), the
// mode sum in double rounded to float (the fill buffer), then every line of the bank for those
// samples (dly_line_kernel's tap arithmetic: age-0 reads take the new sample, all others ring
// slots no sample of the block writes -- loaded before the modal sums, so their latency hides
// under them), the ring commit and the mixdown in line order / N.  Modes come from a compact
// table (float f, d, a + the double decay step), one coalesced load per mode and thread.
constexpr int kChainSpw = 4;
constexpr int kChainThreads = 512;
constexpr int kChainMaxLines = kChainThreads / kChainSpw;   // one (line, sample) per thread
constexpr long kChainMaxN = 8192;

struct ChainArgs {
    const float4* fda;     // [M] {f, d, a, 0} (Bowl<float>'s float coefficients)
    const double* rstep;   // [M] E^{-d/SR} (BRec::R)
    int M;
    double n0;
    long n;
    float* buf;            // the fill buffer [n]
    hz_chain::DlyBlock d;
    float* out;            // mix: [n] (line sum / N); else [N][n] line outputs
    int mix;
};

template <int SPW>
__global__ __launch_bounds__(kChainThreads) void bowl_dly_chain_kernel(ChainArgs a) {
    constexpr int kW = kChainThreads / 64;
    __shared__ double wsum[kW][SPW];
    __shared__ float xs[SPW];
    __shared__ float ly[(kChainThreads / SPW) * SPW];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long t0 = (long)blockIdx.x * SPW;
    const hz_chain::DlyBlock& d = a.d;
    const int S = d.S;
    // ---- the bank's ring reads for this thread's (line, sample), issued first
    const int l = tid / SPW, sl = tid % SPW;
    const long j = t0 + sl;
    const bool live = l < d.N && j < a.n;
    const unsigned o = live ? (unsigned)((d.o0 + (unsigned long)j) % d.size) : 0u;
    float rxv[hz_chain::kMaxTaps], ryv[hz_chain::kMaxTaps], fg[hz_chain::kMaxTaps], bg[hz_chain::kMaxTaps];
    unsigned af_[hz_chain::kMaxTaps], ab_[hz_chain::kMaxTaps];
#pragma unroll
    for (int i = 0; i < hz_chain::kMaxTaps; ++i) {
        rxv[i] = ryv[i] = fg[i] = bg[i] = 0.0f;
        af_[i] = ab_[i] = 0u;
        if (live && i < S) {
            const int4* tp = d.taps + (long)l * 2 * S;
            const float* gn = d.gains + (long)l * 2 * S;
            const int4 qf = tp[i], qb = tp[S + i];
            fg[i] = gn[i];
            bg[i] = gn[S + i];
            af_[i] = ((int)o < qf.x) ? (unsigned)qf.z : (unsigned)qf.y;
            ab_[i] = ((int)o < qb.x) ? (unsigned)qb.z : (unsigned)qb.y;
            if (af_[i] != 0u) rxv[i] = d.rx[(long)l * d.size + (o >= af_[i] ? o - af_[i] : o + d.size - af_[i])];
            if (bg[i] != 0.0f && ab_[i] != 0u)
                ryv[i] = d.ry[(long)l * d.size + (o >= ab_[i] ? o - ab_[i] : o + d.size - ab_[i])];
        }
    }
    // ---- generator: acc[s] = sum over this thread's modes
    float ph[SPW];
#pragma unroll
    for (int s = 0; s < SPW; ++s) ph[s] = phase_f(a.n0, t0 + s);
    double acc[SPW];
#pragma unroll
    for (int s = 0; s < SPW; ++s) acc[s] = 0.0;
    // kPre modes per thread per pass, their table entries loaded together (a mode past M is
    // all zeros: amplitude 0 adds an exact 0)
    constexpr int kPre = 4;
    for (int m0 = tid; m0 < a.M; m0 += kPre * kChainThreads) {
        float4 q[kPre];
        double rs[kPre];
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
            const int m = m0 + u * kChainThreads;
            q[u] = m < a.M ? a.fda[m] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            rs[u] = m < a.M ? a.rstep[m] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < kPre; ++u) {
            const float x0 = div_sr(-q[u].y * ph[0]);
            double amag = (double)q[u].z * exp((double)x0);
#pragma unroll
            for (int s = 0; s < SPW; ++s) {
                const float p = div_sr(q[u].x * ph[s]);
                const float wv = (float)sin2pi_ref(p);
                acc[s] = fma(amag, (double)wv, acc[s]);
                amag *= rs[u];
            }
        }
    }
#pragma unroll
    for (int s = 0; s < SPW; ++s) {
        double v = acc[s];
#pragma unroll
        for (int w = 32; w; w >>= 1) v += __shfl_xor(v, w);
        if (lane == 0) wsum[wave][s] = v;
    }
    __syncthreads();
    if (tid < SPW) {
        double v = wsum[0][tid];
#pragma unroll
        for (int w = 1; w < kW; ++w) v += wsum[w][tid];
        const float x = (float)v;
        xs[tid] = x;
        if (t0 + tid < a.n) a.buf[t0 + tid] = x;
    }
    __syncthreads();
    // ---- the bank (fp contraction off: every product and sum rounds as the reference's)
    {
#pragma clang fp contract(off)
        if (live) {
            const float x = xs[sl];
            float accd = 0.0f;
#pragma unroll
            for (int i = 0; i < hz_chain::kMaxTaps; ++i) {
                if (i < S) {
                    const float xv = af_[i] == 0u ? x : rxv[i];
                    const float yv = bg[i] != 0.0f ? (ab_[i] == 0u ? accd : ryv[i]) : 0.0f;
                    const float fx = fg[i] * xv;
                    const float by = bg[i] * yv;
                    accd = accd + (fx - by);
                }
            }
            d.rx[(long)l * d.size + o] = x;
            d.ry[(long)l * d.size + o] = accd;
            if (a.mix) ly[l * SPW + sl] = accd;
            else a.out[(long)l * a.n + j] = accd;
        }
        if (a.mix) {
            __syncthreads();
            if (tid < SPW && t0 + tid < a.n) {
                float m = 0.0f;   // line order; the LDS reads of 16 lines issue together
#pragma unroll 16
                for (int k = 0; k < d.N; ++k) m = m + ly[k * SPW + tid];
                a.out[t0 + tid] = m / (float)d.N;
            }
        }
    }
}

void build_brec(double f, double amp, double d, bool is_float, double* rec) {
    using C = std::complex<long double>;
    std::memset(rec, 0, sizeof(double) * BRec::SIZE);
    const long double PIr = 3.14159265359L;  // src/includes.h:30
    const long double E = 2.718281828459045L;
    const long double mag = powl(E, -(long double)d / 48000.0L);
    const long double th = 2.0L * PIr * (long double)f / 48000.0L;
    const C w(mag * cosl(th), mag * sinl(th));
    rec[BRec::AMP] = amp;
    rec[BRec::W1] = (double)w.real();
    rec[BRec::W1 + 1] = (double)w.imag();
    C w16(1, 0);
    for (int k = 0; k < 16; ++k) w16 *= w;
    C acc(1, 0);
    for (int p = 0; p < 16; ++p) {
        rec[BRec::T1 + 2 * p] = (double)acc.real();
        rec[BRec::T1 + 2 * p + 1] = (double)acc.imag();
        acc *= w16;
    }
    const C w256 = acc;
    acc = C(1, 0);
    for (int r = 0; r < 4; ++r) {
        rec[BRec::T2 + 2 * r] = (double)acc.real();
        rec[BRec::T2 + 2 * r + 1] = (double)acc.imag();
        acc *= w256;
    }
    rec[BRec::WT] = (double)acc.real();
    rec[BRec::WT + 1] = (double)acc.imag();
    rec[BRec::F] = f;
    rec[BRec::D] = d;
    // float model: per-sample decay factor from the float decay constant
    rec[BRec::R] = (double)expl(-(long double)(is_float ? (float)d : d) / 48000.0L);
}

}  // namespace

struct hz_bowl {
    int M = 0, device = 0, is_float = 0;
    double n0 = 0;  // phase counter (T) at the next call
    double *d_rec = nullptr, *d_partial = nullptr;
    void* d_chain = nullptr;   // (float Bowls) [M] float4 {f, d, a, 0} then [M] double decay steps
    void* d_out = nullptr;
    size_t partial_cap = 0, out_cap = 0;
    int target_groups = 256;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool prof = false;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    long launches = 0;
    // per-sample calls (renders shorter than kLookMin: the drop-in's operator() / tick()) come
    // from a speculative block of kLook samples rendered at once; the state is the phase counter
    // alone, so a rollback sets it to the consumed sample (huygens_hip.h, hz_add_fill)
    static constexpr long kLook = 1024, kLookMin = 64;
    double* la_buf = nullptr;
    long la_n = 0, la_pos = 0;
    double n0_snap = 0;
};

namespace {

int bowl_check(hz_bowl* h) {
    if (!h) {
        hz::set_error("null hz_bowl handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    return HZ_OK;
}

// out_kind: 0 = float samples (fill), 1 = double samples (operator() in T's precision)
int bowl_launch(hz_bowl* h, void* d_dst, long n, int out_kind) {
    if (n <= 0) return HZ_OK;
    const int M = h->M;
    const long ntiles = (n + kTile - 1) / kTile;
    // modes per wave: up to 64 when time segments alone fill the chip; fewer (down to one)
    // for short calls so that modes x segments still give ~2 workgroups per CU
    int per_wave = std::min(kMaxPerWave, std::max(1, (M + kWaves * 32 - 1) / (kWaves * 32)));
    const long par = (long)M * ntiles / ((long)kWaves * 2 * h->target_groups);
    if (par < per_wave) per_wave = (int)std::max<long>(1, par);
    const int G = std::max(1, (M + kWaves * per_wave - 1) / (kWaves * per_wave));
    long nseg = std::max<long>(1, std::min<long>(ntiles, (h->target_groups + G - 1) / G));
    const long seg_tiles = (ntiles + nseg - 1) / nseg;
    nseg = (ntiles + seg_tiles - 1) / seg_tiles;
    const long n_pad = ntiles * kTile;
    const size_t need = (size_t)G * n_pad;
    if (need > h->partial_cap) {
        if (h->d_partial) HZ_TRY_HIP(hipFree(h->d_partial));
        h->d_partial = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_partial, sizeof(double) * need));
        h->partial_cap = need;
    }
    const size_t lds = sizeof(double) * (kWaves * kL * kPad + kWaves * 2 * kMaxPerWave);
    static bool attr = false;
    if (!attr) {
        HZ_TRY_HIP(hipFuncSetAttribute((const void*)bowl_mix_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds));
        attr = true;
    }
    hipEvent_t* e = nullptr;
    if (h->prof) {
        if (h->ev_used + 2 > h->ev.size())
            for (int q = 0; q < 128; ++q) {
                hipEvent_t ne;
                HZ_TRY_HIP(hz::prof_event_create(&ne));
                h->ev.push_back(ne);
            }
        e = &h->ev[h->ev_used];
        h->ev_used += 2;
        HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
    }
    BowlArgs args;
    args.partial = h->d_partial;
    args.n = n;
    args.n_pad = n_pad;
    args.seg_len = seg_tiles * kTile;
    args.n0 = h->n0;
    args.M = M;
    args.nseg = (int)nseg;
    args.per_wave = per_wave;
    args.is_float = h->is_float;
    hipLaunchKernelGGL(bowl_mix_kernel, dim3(G, (unsigned)nseg), dim3(64 * kWaves), lds, h->stream,
                       (const double*)h->d_rec, args);
    HZ_TRY_HIP(hipGetLastError());
    if (e) HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
    if (n <= kShortMax) {
        if (out_kind == 0)
            hipLaunchKernelGGL(bowl_reduce_short_kernel<float>, dim3((unsigned)((n + 63) / 64)),
                               dim3(64 * kShortSlices), 0, h->stream, (const double*)h->d_partial, n_pad, G, n,
                               (float*)d_dst);
        else
            hipLaunchKernelGGL(bowl_reduce_short_kernel<double>, dim3((unsigned)((n + 63) / 64)),
                               dim3(64 * kShortSlices), 0, h->stream, (const double*)h->d_partial, n_pad, G, n,
                               (double*)d_dst);
    } else if (out_kind == 0)
        hipLaunchKernelGGL(bowl_reduce_kernel<float>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, h->stream,
                           (const double*)h->d_partial, n_pad, G, n, (float*)d_dst);
    else
        hipLaunchKernelGGL(bowl_reduce_kernel<double>, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, h->stream,
                           (const double*)h->d_partial, n_pad, G, n, (double*)d_dst);
    HZ_TRY_HIP(hipGetLastError());
    // phase counter: T = double counts exactly; T = float saturates at 2^24
    h->n0 += (double)n;
    if (h->is_float && h->n0 > 16777216.0) h->n0 = 16777216.0;
    h->launches += h->prof ? 1 : 0;
    return HZ_OK;
}

// roll a speculative block back to its consumed sample (the counter saturates as bowl_launch's)
void bowl_settle(hz_bowl* h) {
    if (h->la_pos < h->la_n) {
        h->n0 = h->n0_snap + (double)h->la_pos;
        if (h->is_float && h->n0 > 16777216.0) h->n0 = 16777216.0;
    }
    h->la_n = h->la_pos = 0;
}

int bowl_host(hz_bowl* h, void* out, size_t elem, long n, int kind);

int bowl_look_ahead(hz_bowl* h) {
    if (!h->la_buf) HZ_TRY_HIP(hipHostMalloc((void**)&h->la_buf, sizeof(double) * hz_bowl::kLook));
    h->n0_snap = h->n0;
    HZ_TRY(bowl_host(h, h->la_buf, sizeof(double), hz_bowl::kLook, 1));
    h->la_n = hz_bowl::kLook;
    h->la_pos = 0;
    return HZ_OK;
}

int bowl_host(hz_bowl* h, void* out, size_t elem, long n, int kind) {
    if (n <= 0) return HZ_OK;
    if ((size_t)n * elem > h->out_cap) {
        if (h->d_out) HZ_TRY_HIP(hipFree(h->d_out));
        h->d_out = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_out, elem * n));
        h->out_cap = elem * n;
    }
    HZ_TRY(bowl_launch(h, h->d_out, n, kind));
    HZ_TRY_HIP(hipMemcpyAsync(out, h->d_out, elem * n, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

}  // namespace

extern "C" {

int hz_bowl_create(int overtones, const double* f, const double* a, const double* d, int count, int is_float,
                   int device, hz_bowl** out) {
    if (!out || overtones <= 0 || count < 0 || (count > 0 && (!f || !a || !d))) {
        hz::set_error("hz_bowl_create: invalid arguments");
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_bowl* h = new (std::nothrow) hz_bowl();
    if (!h) return HZ_E_ALLOC;
    h->M = overtones;
    h->device = device;
    h->is_float = is_float ? 1 : 0;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        h->target_groups = prop.multiProcessorCount;
    std::vector<double> rec((size_t)overtones * BRec::SIZE, 0.0);
    for (int i = 0; i < overtones; ++i) {  // vectors resized to `overtones`, padded with 0 (bowl.h:19-22)
        const bool have = i < count;
        double fi = have ? f[i] : 0.0, ai = have ? a[i] : 0.0, di = have ? d[i] : 0.0;
        if (h->is_float) {  // Bowl<float> stores float coefficients
            fi = (float)fi;
            ai = (float)ai;
            di = (float)di;
        }
        build_brec(fi, ai, di, h->is_float, &rec[(size_t)i * BRec::SIZE]);
    }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&h->d_rec, sizeof(double) * rec.size()) != hipSuccess ||
        hipMemcpy(h->d_rec, rec.data(), sizeof(double) * rec.size(), hipMemcpyHostToDevice) != hipSuccess) {
        hz::set_error("hz_bowl_create: device allocation failed");
        if (h->stream) (void)hipStreamDestroy(h->stream);
        if (h->d_rec) (void)hipFree(h->d_rec);
        delete h;
        return HZ_E_ALLOC;
    }
    h->own_stream = true;
    if (h->is_float) {   // the fused block's compact mode table (hz_bowl_fill_delaybank)
        std::vector<float> fda((size_t)overtones * 4, 0.0f);
        std::vector<double> rs((size_t)overtones);
        for (int i = 0; i < overtones; ++i) {
            const double* r = &rec[(size_t)i * BRec::SIZE];
            fda[4 * (size_t)i] = (float)r[BRec::F];
            fda[4 * (size_t)i + 1] = (float)r[BRec::D];
            fda[4 * (size_t)i + 2] = (float)r[BRec::AMP];
            rs[i] = r[BRec::R];
        }
        const size_t fb = sizeof(float) * fda.size();
        if (hipMalloc(&h->d_chain, fb + sizeof(double) * rs.size()) != hipSuccess ||
            hipMemcpy(h->d_chain, fda.data(), fb, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy((char*)h->d_chain + fb, rs.data(), sizeof(double) * rs.size(), hipMemcpyHostToDevice) !=
                hipSuccess) {
            hz::set_error("hz_bowl_create: device allocation failed");
            (void)hz_bowl_destroy(h);
            return HZ_E_ALLOC;
        }
    }
    *out = h;
    return HZ_OK;
}

int hz_bowl_destroy(hz_bowl* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->d_rec, (void*)h->d_partial, h->d_out, h->d_chain})
        if (p) (void)hipFree(p);
    if (h->la_buf) (void)hipHostFree(h->la_buf);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_bowl_trigger(hz_bowl* h) {   // bowl.h:25-28
    if (!h) return HZ_E_INVALID;
    bowl_settle(h);
    h->n0 = 0;
    return HZ_OK;
}

int hz_bowl_fill(hz_bowl* h, float* buffer, size_t bsize) {   // bowl.h:50-63
    HZ_TRY(bowl_check(h));
    if (bsize && !buffer) return HZ_E_INVALID;
    bowl_settle(h);
    return bowl_host(h, buffer, sizeof(float), (long)bsize, 0);
}

int hz_bowl_fill_device(hz_bowl* h, float* d_buffer, size_t bsize) {
    HZ_TRY(bowl_check(h));
    if (bsize && !d_buffer) return HZ_E_INVALID;
    bowl_settle(h);
    return bowl_launch(h, d_buffer, (long)bsize, 0);
}

// n x { out[j] = operator()(); tick(); }  bowl.h:30-48, samples widened to double
int hz_bowl_render(hz_bowl* h, double* out, size_t n) {
    HZ_TRY(bowl_check(h));
    if (n && !out) return HZ_E_INVALID;
    if ((long)n < hz_bowl::kLookMin) {   // per-sample calls: from the speculative block
        for (size_t i = 0; i < n; ++i) {
            if (h->la_pos == h->la_n) HZ_TRY(bowl_look_ahead(h));
            out[i] = h->la_buf[h->la_pos++];
        }
        return HZ_OK;
    }
    bowl_settle(h);
    return bowl_host(h, out, sizeof(double), (long)n, 1);
}

int hz_bowl_render_device(hz_bowl* h, double* d_out, size_t n) {
    HZ_TRY(bowl_check(h));
    if (n && !d_out) return HZ_E_INVALID;
    bowl_settle(h);
    return bowl_launch(h, d_out, (long)n, 1);
}

int hz_bowl_phase(hz_bowl* h, double* phase) {
    if (!h || !phase) return HZ_E_INVALID;
    bowl_settle(h);
    *phase = h->n0;
    return HZ_OK;
}

int hz_bowl_set_stream(hz_bowl* h, void* s) {
    HZ_TRY(bowl_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) HZ_TRY_HIP(hipStreamDestroy(h->stream));
    if (s) {
        h->stream = (hipStream_t)s;
        h->own_stream = false;
    } else {
        HZ_TRY_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->own_stream = true;
    }
    return HZ_OK;
}

int hz_bowl_set_target_groups(hz_bowl* h, int groups) {
    if (!h || groups < 1) return HZ_E_INVALID;
    h->target_groups = groups;
    return HZ_OK;
}

int hz_bowl_profile(hz_bowl* h, int enable) {
    HZ_TRY(bowl_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    h->prof = enable != 0;
    h->ev_used = 0;
    h->launches = 0;
    return HZ_OK;
}

int hz_bowl_profile_read(hz_bowl* h, double* ms, long* launches) {
    HZ_TRY(bowl_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    double m = 0;
    for (size_t i = 0; i + 2 <= h->ev_used; i += 2) {
        float x = 0;
        HZ_TRY_HIP(hipEventElapsedTime(&x, h->ev[i], h->ev[i + 1]));
        m += x;
    }
    if (ms) *ms = m;
    if (launches) *launches = h->launches;
    return HZ_OK;
}

// Bowl<float>::fill(buf, n) then Delaybank<float>::process(buf, out, n, mix) (bowl.h:50-63,
// delay.h:71-97) as one launch when the bank's taps allow it (hz_chain.h), else
// the two block calls.  Both objects on one stream.
int hz_bowl_fill_delaybank(hz_bowl* h, float* d_buf, hz_dly* bank, void* d_out, size_t bsize, int mix) {
    HZ_TRY(bowl_check(h));
    if (!bank || (bsize && (!d_buf || !d_out))) return HZ_E_INVALID;
    bowl_settle(h);
    const long n = (long)bsize;
    hz_chain::DlyBlock d;
    bool fusable = false;
    HZ_TRY(hz_chain::dly_block_begin(bank, n, &d, &fusable));
    HZ_TRY(bowl_check(h));
    if (d.stream != h->stream) {
        hz::set_error("hz_bowl_fill_delaybank: the bowl and the bank run on different streams (set_stream both)");
        return HZ_E_INVALID;
    }
    if (n == 0) return HZ_OK;
    if (!fusable || !h->is_float || !h->d_chain || n > kChainMaxN || d.N > kChainMaxLines) {
        HZ_TRY(bowl_launch(h, d_buf, n, 0));
        return hz_dly_process_device(bank, d_buf, d_out, bsize, 0, mix);
    }
    hipEvent_t* e = nullptr;
    if (h->prof) {
        if (h->ev_used + 2 > h->ev.size())
            for (int q = 0; q < 128; ++q) {
                hipEvent_t ne;
                HZ_TRY_HIP(hz::prof_event_create(&ne));
                h->ev.push_back(ne);
            }
        e = &h->ev[h->ev_used];
        h->ev_used += 2;
        HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
    }
    ChainArgs a;
    a.fda = (const float4*)h->d_chain;
    a.rstep = (const double*)((const char*)h->d_chain + sizeof(float4) * h->M);
    a.M = h->M;
    a.n0 = h->n0;
    a.n = n;
    a.buf = d_buf;
    a.d = d;
    a.out = (float*)d_out;
    a.mix = mix ? 1 : 0;
    // samples per workgroup (env HZ_CHAIN_SPW = 2 / 4 / 8 for A/B; lines must fit kChainThreads / SPW)
    int spw = kChainSpw;
    if (const char* e = std::getenv("HZ_CHAIN_SPW")) {
        const int v = std::atoi(e);
        if ((v == 2 || v == 4 || v == 8) && d.N <= kChainThreads / v) spw = v;
    }
    const unsigned grid = (unsigned)((n + spw - 1) / spw);
    if (spw == 2) hipLaunchKernelGGL(bowl_dly_chain_kernel<2>, dim3(grid), dim3(kChainThreads), 0, h->stream, a);
    else if (spw == 8) hipLaunchKernelGGL(bowl_dly_chain_kernel<8>, dim3(grid), dim3(kChainThreads), 0, h->stream, a);
    else hipLaunchKernelGGL(bowl_dly_chain_kernel<kChainSpw>, dim3(grid), dim3(kChainThreads), 0, h->stream, a);
    HZ_TRY_HIP(hipGetLastError());
    if (e) HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
    h->n0 += (double)n;
    if (h->n0 > 16777216.0) h->n0 = 16777216.0;
    h->launches += h->prof ? 1 : 0;
    hz_chain::dly_block_end(bank, n);
    return HZ_OK;
}

}  // extern "C"
