// hz_fb_resp.hip -- the stationary Filterbank<double> engine (bank response convolution).
//
// Once a bank has run converged (pre = pin, gain = gin: hz_fb_lti.hip) with unchanged
// coefficients for K samples, K = its horizon (||M^K||_inf < 2^-53 for every band's state
// transition M, fb_lti_horizon, rounded up to 8192), every band's state is the zero-state response
// of the last K input samples to below an ulp of itself, and the bank's mixdown
// (src/filterbank.h:130,178-179) is ONE linear filter of the input:
//     out[t] = sum_n gin_n y_n[t] = sum_{tau < K} h[tau] x[t - tau],   h[tau] = sum_n gin_n r_n[tau]
// with r_n band n's impulse response at pre = pin_n.  A call then runs as a uniformly partitioned
// overlap-save convolution on FP64 FFTs (P = 2048-sample partitions, 4096-point transforms):
//   resp_fwd_kernel   one 4096-point FFT per pair of input windows W_i = u[(i-1)P, (i+1)P) of
//                     u = [last K inputs | call input]: windows i and i + D share a transform
//                     (real + i imag; h is real, so their products with H stay separable)
//   resp_mac_kernel   Y_b = sum_{p < Q} H_p Z_{b+Q-1-p} per bin (Q = K / P partition spectra)
//   resp_inv_kernel   one inverse FFT per output-block pair: Re -> block b, Im -> block b + D
// Per output sample that is O(Q + log F) work whatever the number of bands; the bands enter once,
// through h, when coefficients or targets change (resp_h_kernel: each band's response by the
// reference's own recurrence, summed in a fixed order).
//
// The per-band state is kept exact: the last K inputs are the handle's history (updated by every
// converged long call the engine could take, whatever engine ran it), and the band states at the
// call end are their zero-state response over those K samples (the chunk-128 LTI state kernel in
// its prepass mode, fb_lti_zero_start_end) -- after every call (HZ_FB_RESP_EAGER, default) or only
// when a later call, get_state, tick or a setter needs them (HZ_FB_RESP_LAZY).
// Multi-GPU: time-range shards (hz_fb_set_bank_response + hz_fb_set_time_shard) convolve one
// rank's run of output blocks with the whole bank's response; DESIGN.md 3.6 and 5.
#include <cstdlib>

#include "hz_fb_impl.h"
#include "hz_fft.h"

namespace {

constexpr int kLgP = 11, kP = 1 << kLgP;       // partition / output block (samples)
constexpr int kLgF = kLgP + 1, kF = 2 * kP;    // transform size
constexpr int kRmax = 3;                       // radix-8 passes (hz_fft.h)
constexpr int kFftThreads = kF >> kRmax;       // 512: one radix-8 group per thread
constexpr int kMacR = 8;                       // output blocks per MAC thread (partitions padded to it)
// (A/B) HZ_FB_RESP_MAC_R = 4 / 8 / 16 output blocks per MAC thread
int mac_r() {
    static const int r = [] {
        const int v = std::getenv("HZ_FB_RESP_MAC_R") ? std::atoi(std::getenv("HZ_FB_RESP_MAC_R")) : kMacR;
        return v == 4 || v == 16 ? v : kMacR;
    }();
    return r;
}
constexpr long kMinCall = 16384;               // shortest call that keeps the history

size_t fft_lds() { return sizeof(double) * 2 * (size_t)hz::padded_len(kF) + sizeof(double2) * hz::twc_len(kLgF); }

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

__device__ __forceinline__ void load_tw(double2* T, const double2* __restrict__ tw) {
    for (int k = threadIdx.x; k < hz::twc_len(kLgF); k += blockDim.x) T[k] = tw[k];
}

// the compact twiddle table in two register loads per thread (threads >= twc_len / 2), issued
// with the data loads and stored with them: one memory latency before the first pass, not two
template <int NT>
struct TwRegs {
    static_assert(2 * NT >= hz::twc_len(kLgF), "two twiddles per thread");
    double2 a, b;
    __device__ __forceinline__ void load(const double2* __restrict__ tw) {
        constexpr int TL = hz::twc_len(kLgF);
        a = threadIdx.x < TL ? tw[threadIdx.x] : make_double2(0.0, 0.0);
        b = threadIdx.x + NT < TL ? tw[threadIdx.x + NT] : make_double2(0.0, 0.0);
    }
    __device__ __forceinline__ void store(double2* T) const {
        constexpr int TL = hz::twc_len(kLgF);
        if (threadIdx.x < TL) T[threadIdx.x] = a;
        if (threadIdx.x + NT < TL) T[threadIdx.x + NT] = b;
    }
};

// Partition spectra H_p = FFT(h[pP, (p+1)P) zero-padded to F) / F (the inverse is unnormalised;
// 1/F is a power of two), bins in the transforms' storage (bit-reversed) order
__global__ __launch_bounds__(kFftThreads) void resp_hspec_kernel(const double* __restrict__ h, long K,
                                                                 const double2* __restrict__ tw,
                                                                 double2* __restrict__ H) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + hz::padded_len(kF);
    double2* T = (double2*)(im + hz::padded_len(kF));
    load_tw(T, tw);
    const long p0 = (long)blockIdx.x * kP;
    for (int k = threadIdx.x; k < kF; k += blockDim.x) {
        re[hz::pad16(k)] = (k < kP && p0 + k < K) ? h[p0 + k] * (1.0 / kF) : 0.0;
        im[hz::pad16(k)] = 0.0;
    }
    __syncthreads();
    hz::fft_fwd_lead<kRmax>(re, im, kLgF, T, true);
    double2* o = H + (long)blockIdx.x * kF;
    for (int q = threadIdx.x; q < kF; q += blockDim.x) o[q] = make_double2(re[hz::pad16(q)], im[hz::pad16(q)]);
}

struct RespArgs {
    const double* hist;   // [K] the K inputs before the call
    const double* x;      // [n] the call's input
    long K, n;            // horizon; the call's length
    long off, n_out;      // outputs of this launch: out[off, off + n_out) (time-range shards)
    int Q, D;             // partitions; packed output-block pairs
    const double2* tw;
    double2* Z;           // [Q + D - 1 (+ pad)][F] packed window spectra
    const double2* Y;     // [D][F] packed output spectra
    double* out;          // [n]
    // state upkeep, done by the inverse kernel's threads: the history after the call (the last K
    // samples of [hist | x]), the smoothers' closed form, the x history (the last O inputs)
    double* hist_next;
    const double *pg, *pin, *gin;
    double* pg_next;
    double sp_n, sg_n;
    double* xhist_next;
    int N, O;
};

// u = [hist | x | 0 ...], indexed from the launch's first output block (off)
__device__ __forceinline__ double resp_u(const RespArgs& a, long m) {
    m += a.off;
    if (m < a.K) return a.hist[m];
    m -= a.K;
    return m < a.off + a.n_out ? a.x[m] : 0.0;
}

// Z_j = FFT(W_{j+1} + i W_{j+1+D}), W_i = u[(i-1)P, (i+1)P)
// (ABL, diagnostics HZ_FB_RESP_ABL=1: no FFT passes -- wrong results, timed by rocprof)
template <int ABL = 0, int RM = kRmax>
__global__ __launch_bounds__(kF >> RM) void resp_fwd_kernel(RespArgs a) {
    constexpr int kFftThreads = kF >> RM;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + hz::padded_len(kF);
    double2* T = (double2*)(im + hz::padded_len(kF));
    const long j = blockIdx.x;
    const long m0 = j * kP, m1 = (j + a.D) * kP;
    // every load of the thread (twiddles included) issued before the first LDS store
    constexpr int PT = kF / kFftThreads;
    TwRegs<kFftThreads> tr;
    tr.load(a.tw);
    double vr[PT], vi[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) {
        const int k = threadIdx.x + i * kFftThreads;
        vr[i] = resp_u(a, m0 + k);
        vi[i] = resp_u(a, m1 + k);
    }
    tr.store(T);
#pragma unroll
    for (int i = 0; i < PT; ++i) {
        const int k = threadIdx.x + i * kFftThreads;
        re[hz::pad16(k)] = vr[i];
        im[hz::pad16(k)] = vi[i];
    }
    __syncthreads();
    if constexpr (ABL == 0) hz::fft_fwd_lead<RM>(re, im, kLgF, T, true);
    double2* z = a.Z + j * kF;
    for (int q = threadIdx.x; q < kF; q += blockDim.x) z[q] = make_double2(re[hz::pad16(q)], im[hz::pad16(q)]);
}

// Y_b[q] = sum_{p < Q} H_p[q] Z_{b+Q-1-p}[q] for b in [b0, b0 + R): thread = bin q x R output
// blocks.  The R Z values of step p sit in a register ring (element r in slot (r - p) mod R): each
// step brings one new Z value and one H value for R complex MACs.  Partitions are padded to a
// multiple of R with zero spectra (Qp), so every block of R steps loads unguarded, and the next
// block's 2R loads are issued before this block's MACs (latency once per call, not per step).
template <int R>
__global__ __launch_bounds__(256) void resp_mac_kernel(const double2* __restrict__ H, const double2* __restrict__ Z,
                                                       double2* __restrict__ Y, int Q, int Qp, int D) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;   // bin (grid.x = F / 256)
    const int b0 = blockIdx.y * R;
    double ar[R], ai[R], zr[R], zi[R];
    const long base = (long)b0 + Q - 1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        ar[r] = ai[r] = 0.0;
        const double2 z = Z[(base + r) * kF + q];
        zr[r] = z.x;
        zi[r] = z.y;
    }
    double2 hb[R], zb[R];
    auto fetch = [&](int p0) {
#pragma unroll
        for (int u = 0; u < R; ++u) {
            hb[u] = H[(long)(p0 + u) * kF + q];
            const long zi_ = base - (p0 + u) - 1;   // < 0 only past Q (zero H rows)
            zb[u] = Z[(zi_ > 0 ? zi_ : 0) * kF + q];
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
        for (int u = 0; u < R; ++u) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sl = ((r - u) % R + R) % R;
                ar[r] = fma(hc[u].x, zr[sl], ar[r]);
                ar[r] = fma(-hc[u].y, zi[sl], ar[r]);
                ai[r] = fma(hc[u].x, zi[sl], ai[r]);
                ai[r] = fma(hc[u].y, zr[sl], ai[r]);
            }
            // element 0 of step p + 1 = Z[base - p - 1] into the slot element R - 1 leaves
            const int sl = ((-(u + 1)) % R + R) % R;
            zr[sl] = zc[u].x;
            zi[sl] = zc[u].y;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
        if (b0 + r < D) Y[(long)(b0 + r) * kF + q] = make_double2(ar[r], ai[r]);
}

// The same MACs with the operands shared through LDS: workgroup = 64 bins x 4 waves, wave w owns
// output blocks b0 + w R .. + R - 1 of the workgroup's 4 R; the Qp partition spectra and the
// 4 R + Qp window spectra of the 64 bins are staged once (24 + 57 KB at C2) instead of read by
// every thread from L2, then each thread runs the register ring of resp_mac_kernel from LDS.
template <int R>
__global__ __launch_bounds__(256) void resp_mac_lds_kernel(const double2* __restrict__ H, const double2* __restrict__ Z,
                                                           double2* __restrict__ Y, int Q, int Qp, int D, int zrows) {
    extern __shared__ __attribute__((aligned(16))) double mac_lds[];
    double2* hs = (double2*)mac_lds;   // [Qp][64]
    double2* zs = hs + Qp * 64;        // [4 R + Qp][64]
    const int bin = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int q = blockIdx.x * 64 + bin;
    const int bw = blockIdx.y * 4 * R;            // first output block of the workgroup
    const int nz = 4 * R + Qp;                    // window rows bw .. bw + nz - 1 (clamped)
    // staging in batches of 8 loads per thread issued before their stores (few memory latencies)
    constexpr int SB = 8;
    for (int i0 = threadIdx.x; i0 < Qp * 64; i0 += SB * 256) {
        double2 v[SB];
#pragma unroll
        for (int k = 0; k < SB; ++k) {
            const int i = i0 + k * 256;
            v[k] = i < Qp * 64 ? H[(long)(i >> 6) * kF + blockIdx.x * 64 + (i & 63)] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int k = 0; k < SB; ++k)
            if (i0 + k * 256 < Qp * 64) hs[i0 + k * 256] = v[k];
    }
    for (int i0 = threadIdx.x; i0 < nz * 64; i0 += SB * 256) {
        double2 v[SB];
#pragma unroll
        for (int k = 0; k < SB; ++k) {
            const int i = i0 + k * 256;
            const int row = min(bw + (i >> 6), zrows - 1);
            v[k] = i < nz * 64 ? Z[(long)row * kF + blockIdx.x * 64 + (i & 63)] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int k = 0; k < SB; ++k)
            if (i0 + k * 256 < nz * 64) zs[i0 + k * 256] = v[k];
    }
    __syncthreads();
    // thread's outputs b = bw + w R + r; Y_b = sum_p H_p Z_{b+Q-1-p}: local row w R + r + Q - 1 - p
    double ar[R], ai[R], zr[R], zi[R];
    const int base = w * R + Q - 1;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        ar[r] = ai[r] = 0.0;
        const double2 z = zs[(base + r) * 64 + bin];
        zr[r] = z.x;
        zi[r] = z.y;
    }
    for (int p0 = 0; p0 < Qp; p0 += R) {
#pragma unroll
        for (int u = 0; u < R; ++u) {
            const int p = p0 + u;
            const double2 hv = hs[p * 64 + bin];
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int sl = ((r - u) % R + R) % R;
                ar[r] = fma(hv.x, zr[sl], ar[r]);
                ar[r] = fma(-hv.y, zi[sl], ar[r]);
                ai[r] = fma(hv.x, zi[sl], ai[r]);
                ai[r] = fma(hv.y, zr[sl], ai[r]);
            }
            const int zrow = base - p - 1;   // < 0 only past Q (zero H rows)
            const double2 z = zs[(zrow > 0 ? zrow : 0) * 64 + bin];
            const int sl = ((-(u + 1)) % R + R) % R;
            zr[sl] = z.x;
            zi[sl] = z.y;
        }
    }
    (void)q;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int b = bw + w * R + r;
        if (b < D) Y[(long)b * kF + blockIdx.x * 64 + bin] = make_double2(ar[r], ai[r]);
    }
}

// out[bP + r] = Re IFFT(Y_b)[P + r], out[(b + D)P + r] = Im ...
template <int ABL = 0, int RM = kRmax>
__global__ __launch_bounds__(kF >> RM) void resp_inv_kernel(RespArgs a) {
    constexpr int kFftThreads = kF >> RM;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + hz::padded_len(kF);
    double2* T = (double2*)(im + hz::padded_len(kF));
    const long b = blockIdx.x;
    const double2* y = a.Y + b * kF;
    constexpr int PT = kF / kFftThreads;
    TwRegs<kFftThreads> tr;
    tr.load(a.tw);
    double2 v[PT];
#pragma unroll
    for (int i = 0; i < PT; ++i) v[i] = y[threadIdx.x + i * kFftThreads];
    tr.store(T);
#pragma unroll
    for (int i = 0; i < PT; ++i) {
        const int q = threadIdx.x + i * kFftThreads;
        re[hz::pad16(q)] = v[i].x;
        im[hz::pad16(q)] = v[i].y;
    }
    __syncthreads();
    if constexpr (ABL == 0) hz::fft_inv_tail<RM>(re, im, kLgF, T, true);
    for (int r = threadIdx.x; r < kP; r += blockDim.x) {
        const long t0 = b * kP + r, t1 = (b + a.D) * kP + r;
        if (t0 < a.n_out) a.out[a.off + t0] = re[hz::pad16(kP + r)];
        if (t1 < a.n_out) a.out[a.off + t1] = im[hz::pad16(kP + r)];
    }
    // state upkeep (the forward kernel, the last reader of hist, has finished)
    const long g = b * blockDim.x + threadIdx.x, stride = (long)gridDim.x * blockDim.x;
    // a time-range shard leaves zeros outside its range: the ranks' outputs sum to the call's
    for (long t = g; t < a.n - a.n_out; t += stride) a.out[t < a.off ? t : t + a.n_out] = 0.0;
    for (long i = g; i < a.K; i += stride) {
        const long m = a.n + i;
        a.hist_next[i] = m < a.K ? a.hist[m] : a.x[m - a.K];
    }
    for (long n = g; n < a.N; n += stride) {
        const double P0 = a.pg[2 * n], G0 = a.pg[2 * n + 1], pb = a.pin[n], gb = a.gin[n];
        a.pg_next[2 * n] = pb + a.sp_n * (P0 - pb);
        a.pg_next[2 * n + 1] = gb + a.sg_n * (G0 - gb);
    }
    if (g < a.O) a.xhist_next[g] = a.x[a.n - 1 - g];
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

// per-bank setup: horizon, history buffers, twiddles
int resp_setup(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    if (R.K == -2) {
        // ||M^K|| < 2^-53 (env HZ_FB_RESP_HORIZON_LOG2, e.g. -64): older inputs reach a band state
        // below one unit in the last place of it, and the bank response's tail below 2^-53 of its
        // l1 norm; then a whole number of the chunk-128 state kernel's 8192-sample tiles
        static const int lb = std::getenv("HZ_FB_RESP_HORIZON_LOG2") ? std::atoi(std::getenv("HZ_FB_RESP_HORIZON_LOG2"))
                                                                      : -53;
        R.K = hz_fbi::fb_horizon(h, lb);
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
    if (!R.d_tw) {
        std::vector<double2> tw(kF / 2);
        const long double pi = acosl(-1.0L);
        for (int k = 0; k < kF / 2; ++k) {
            const long double ang = -2.0L * pi * k / kF;
            tw[k] = make_double2((double)cosl(ang), (double)sinl(ang));
        }
        HZ_TRY_HIP(hipMalloc((void**)&R.d_tw, sizeof(double2) * tw.size()));
        HZ_TRY_HIP(hipMemcpy(R.d_tw, tw.data(), sizeof(double2) * tw.size(), hipMemcpyHostToDevice));
        for (const void* k : {(const void*)resp_hspec_kernel, (const void*)resp_fwd_kernel<0>, (const void*)resp_inv_kernel<0>,
                              (const void*)resp_fwd_kernel<1>, (const void*)resp_inv_kernel<1>})
            HZ_TRY(hz_fbi::fb_set_lds_attr(k));
    }
    return HZ_OK;
}

int resp_state_mode() {
    // (C2, 200 steps: 2 -> 0.0664 ms/step; 0 -> 0.0730, 1 -> 0.0776, 3 -> 0.0739: beside the
    // convolution the state work slows the FFT and MAC kernels by as much as it hides)
    static const int m = std::getenv("HZ_FB_RESP_STATE") ? std::atoi(std::getenv("HZ_FB_RESP_STATE")) : 2;
    return m >= 0 && m <= 3 ? m : 2;
}
bool resp_gemm_states() { return resp_state_mode() == 1 || resp_state_mode() == 3; }

// h and its partition spectra for the current coefficients / targets
int resp_build_h(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    if (R.h_valid) return HZ_OK;
    const int O = h->order, N = h->N;
    const long K = R.K;
    const int G = (N + 63) / 64;
    const int Q = (int)(K / kP);
    const int Qp = (Q + mac_r() - 1) / mac_r() * mac_r();   // zero spectra past Q (the MAC's unguarded blocks)
    HZ_TRY(resp_alloc(&R.d_coef, &R.coef_cap, (size_t)N * (2 * O + 1)));
    HZ_TRY_HIP(hipMemcpyAsync(R.d_coef, h->F.data(), sizeof(double) * N * (O + 1), hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipMemcpyAsync(R.d_coef + (size_t)N * (O + 1), h->B.data(), sizeof(double) * N * O,
                              hipMemcpyHostToDevice, h->stream));
    HZ_TRY(resp_alloc(&R.d_hpart, &R.hpart_cap, (size_t)G * K));
    HZ_TRY(resp_alloc(&R.d_h, &R.h_cap, (size_t)K));
    HZ_TRY(resp_alloc(&R.d_H, &R.H_cap, (size_t)2 * Qp * kF));
    HZ_TRY_HIP(hipMemsetAsync(R.d_H, 0, sizeof(double2) * (size_t)Qp * kF, h->stream));
    hipLaunchKernelGGL(pick_h(O), dim3(G), dim3(64), 0, h->stream, (const double*)R.d_coef,
                       (const double*)(R.d_coef + (size_t)N * (O + 1)), (const double*)h->d_pin,
                       (const double*)h->d_gin, N, K, R.d_hpart);
    HZ_TRY_HIP(hipGetLastError());
    hipLaunchKernelGGL(resp_hsum_kernel, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, h->stream,
                       (const double*)R.d_hpart, G, K, R.d_h);
    HZ_TRY_HIP(hipGetLastError());
    if (R.over_valid)   // the whole bank's response (time-range shards)
        HZ_TRY_HIP(hipMemcpyAsync(R.d_h, R.h_over.data(), sizeof(double) * K, hipMemcpyHostToDevice, h->stream));
    hipLaunchKernelGGL(resp_hspec_kernel, dim3((unsigned)Q), dim3(kFftThreads), fft_lds(), h->stream,
                       (const double*)R.d_h, K, (const double2*)R.d_tw, (double2*)R.d_H);
    HZ_TRY_HIP(hipGetLastError());
    if (resp_gemm_states()) {   // end-state GEMM operands for these coefficients and pre-amps
        HZ_TRY(resp_alloc(&R.d_eg, &R.eg_cap, (size_t)hz_fbi::fb_end_rows(O) * hz_fbi::fb_end_cols(N, O)));
        HZ_TRY(resp_alloc(&R.d_epart, &R.epart_cap, hz_fbi::fb_end_scratch(N, O, K)));
        HZ_TRY(hz_fbi::fb_end_operands(h, R.d_eg));
    } else {
        HZ_TRY(hz_fbi::fb_lti_prepare_end(h, K));   // the state kernel's records, for LAZY too
    }
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // pageable coefficient sources
    R.h_valid = true;
    return HZ_OK;
}

// zero-start band states over the history's K samples -> ystate (the end state of the last
// stationary call: after it (EAGER) or when needed (LAZY))
int resp_states(hz_fb* h, double* ystate) {
    hz_fb::Resp& R = h->resp;
    if (resp_gemm_states() && R.d_eg)   // operands of the coefficients the history ran with
        return hz_fbi::fb_end_state_gemm(h, R.d_hist[R.hcur], nullptr, 0, R.K, R.d_eg, R.d_epart, ystate, h->stream);
    return hz_fbi::fb_lti_zero_start_end(h, R.d_hist[R.hcur], R.K, R.d_zero, R.d_zero, ystate);
}

long resp_min_call(const hz_fb* h) { return h->resp.min_call > 0 ? h->resp.min_call : kMinCall; }

int resp_mode_default() {
    static const int m = [] {
        const char* e = std::getenv("HZ_FB_RESP");   // 0 off, 1 eager (default), 2 lazy
        const int v = e ? std::atoi(e) : HZ_FB_RESP_EAGER;
        return v >= HZ_FB_RESP_OFF && v <= HZ_FB_RESP_LAZY ? v : HZ_FB_RESP_EAGER;
    }();
    return m;
}

}  // namespace

namespace hz_fbi {

void fb_resp_init(hz_fb* h) { h->resp.mode = resp_mode_default(); }

void fb_resp_invalidate(hz_fb* h, bool coefficients) {
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
    static const long per_env = std::getenv("HZ_FB_RESP_BANDS") ? std::atol(std::getenv("HZ_FB_RESP_BANDS")) : 256;
    const long per = R.bands_per_sample >= 0 ? R.bands_per_sample : per_env;
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

int fb_resp_materialize(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    if (!R.implicit) return HZ_OK;
    HZ_TRY(resp_states(h, h->d_ystate[h->scur]));
    R.implicit = false;
    return HZ_OK;
}

// after a call on any engine: the history keeps the last K inputs while the bank stays converged
int fb_resp_track(hz_fb* h, const double* d_in, long n, bool conv) {
    hz_fb::Resp& R = h->resp;
    // (handles pinned to the general engine never run stationary: no history upkeep; a
    // distortion functor keeps it, the engine resumes when the functor is cleared)
    if (R.mode == HZ_FB_RESP_OFF || !conv || h->order == 0 || n < resp_min_call(h) ||
        h->path_mode != HZ_FB_PATH_AUTO) {
        R.run = 0;
        return HZ_OK;
    }
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
    HZ_TRY(resp_build_h(h));
    const long K = R.K;
    const int Q = (int)(K / kP);
    const int Qp = (Q + mac_r() - 1) / mac_r() * mac_r();
    // time-range shard (hz_fb_set_time_shard, with the whole bank's response): this rank's run of
    // whole output blocks
    long off = 0, n_out = n;
    if (R.shard_world > 1 && R.over_valid) {
        const long Ball = (n + kP - 1) / kP;
        const long lo = Ball * R.shard_rank / R.shard_world, hi = Ball * (R.shard_rank + 1) / R.shard_world;
        off = std::min(n, lo * kP);
        n_out = std::min(n, hi * kP) - off;
    }
    const long B = std::max<long>(1, (n_out + kP - 1) / kP);
    const int D = (int)((B + 1) / 2);
    const int nz = Q + D - 1;
    // rows the MACs may read: the last register window (padded to 4 R output blocks, Qp partitions)
    const int zrows = (D + 64 - 1) / 64 * 64 + Qp;   // >= every MAC variant's last window
    if ((size_t)zrows * kF * 2 > R.Z_cap) {
        HZ_TRY(resp_alloc(&R.d_Z, &R.Z_cap, (size_t)zrows * kF * 2));
        HZ_TRY_HIP(hipMemsetAsync(R.d_Z, 0, sizeof(double2) * (size_t)zrows * kF, h->stream));
    }
    HZ_TRY(resp_alloc(&R.d_Y, &R.Y_cap, (size_t)D * kF * 2));
    hipEvent_t* e = nullptr;
    if (h->prof) {
        HZ_TRY(fb_prof_events(h, &e));
        HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        h->ev_skip[(e - h->ev.data()) / 5] |= 2 | 8;   // no segment phase; reduce start = mix end
    }
    RespArgs a;
    a.hist = R.d_hist[R.hcur];
    a.x = d_in;
    a.K = K;
    a.n = n;
    a.off = off;
    a.n_out = n_out;
    a.Q = Q;
    a.D = D;
    a.tw = (const double2*)R.d_tw;
    a.Z = (double2*)R.d_Z;
    a.Y = (const double2*)R.d_Y;
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
    // EAGER: the band states after this call (the last K samples of [hist | x]) do not depend on
    // the convolution -- the end-state GEMM runs on a side stream beside it, joined at the end
    const bool lazy = R.mode == HZ_FB_RESP_LAZY;
    // where the band states are computed (HZ_FB_RESP_STATE, A/B): 2 (default) the chunk-128 state
    // kernel in prepass mode after the convolution; 0 that kernel over x's last K samples on a
    // side stream beside the convolution (calls n >= K; else as 2), 1 the end-state GEMM on the
    // side stream, 3 the end-state GEMM after the convolution
    const int smode = resp_state_mode() == 0 && n < K ? 2 : resp_state_mode();
    const bool side = !lazy && (smode == 0 || smode == 1);
    if (side) {
        if (!R.side) {
            HZ_TRY_HIP(hipStreamCreateWithFlags(&R.side, hipStreamNonBlocking));
            HZ_TRY_HIP(hipEventCreateWithFlags(&R.ev_fork, hipEventDisableTiming));
            HZ_TRY_HIP(hipEventCreateWithFlags(&R.ev_join, hipEventDisableTiming));
        }
        HZ_TRY_HIP(hipEventRecord(R.ev_fork, h->stream));
        HZ_TRY_HIP(hipStreamWaitEvent(R.side, R.ev_fork, 0));
        if (smode == 0)
            HZ_TRY(hz_fbi::fb_lti_zero_start_end_on(h, d_in + (n - K), K, R.d_zero, R.d_zero,
                                                    h->d_ystate[h->scur ^ 1], R.side));
        else
            HZ_TRY(hz_fbi::fb_end_state_gemm(h, R.d_hist[R.hcur], d_in, n, K, R.d_eg, R.d_epart,
                                             h->d_ystate[h->scur ^ 1], R.side));
        HZ_TRY_HIP(hipEventRecord(R.ev_join, R.side));
    }
    static const int abl = std::getenv("HZ_FB_RESP_ABL") ? std::atoi(std::getenv("HZ_FB_RESP_ABL")) : 0;
    // (A/B) HZ_FB_RESP_RADIX=4: radix-4 passes on 1024 threads per transform instead of radix 8 on 512
    static const bool r4 = std::getenv("HZ_FB_RESP_RADIX") && std::atoi(std::getenv("HZ_FB_RESP_RADIX")) == 4;
    if (r4) {
        HZ_TRY(fb_set_lds_attr((const void*)resp_fwd_kernel<0, 2>));
        HZ_TRY(fb_set_lds_attr((const void*)resp_inv_kernel<0, 2>));
    }
    typedef void (*RespFftKernel)(RespArgs);
    const RespFftKernel kfwd = r4 ? resp_fwd_kernel<0, 2> : abl == 1 ? resp_fwd_kernel<1> : resp_fwd_kernel<0>;
    const RespFftKernel kinv = r4 ? resp_inv_kernel<0, 2> : abl == 1 ? resp_inv_kernel<1> : resp_inv_kernel<0>;
    hipLaunchKernelGGL(kfwd, dim3((unsigned)nz), dim3(r4 ? kF >> 2 : kFftThreads), fft_lds(), h->stream, a);
    HZ_TRY_HIP(hipGetLastError());
    // MAC straight from L2 (default) or through LDS (HZ_FB_RESP_MAC=1; C2: 8.4 vs 8.0 us -- the
    // L2 reads were not its bound)
    static const bool mac_lds = std::getenv("HZ_FB_RESP_MAC") && std::getenv("HZ_FB_RESP_MAC")[0] == '1';
    const size_t mac_bytes = sizeof(double2) * 64 * (size_t)(Qp + 4 * kMacR + Qp);
    if (mac_lds && mac_bytes <= 160 * 1024) {
        HZ_TRY(fb_set_lds_attr((const void*)resp_mac_lds_kernel<kMacR>));
        hipLaunchKernelGGL(resp_mac_lds_kernel<kMacR>, dim3(kF / 64, (unsigned)((D + 4 * kMacR - 1) / (4 * kMacR))),
                           dim3(256), mac_bytes, h->stream, (const double2*)R.d_H, (const double2*)R.d_Z,
                           (double2*)R.d_Y, Q, Qp, D, zrows);
    } else {
        const int mr = mac_r();
        auto km = mr == 4 ? resp_mac_kernel<4> : mr == 16 ? resp_mac_kernel<16> : resp_mac_kernel<8>;
        hipLaunchKernelGGL(km, dim3(kF / 256, (unsigned)((D + mr - 1) / mr)), dim3(256), 0,
                           h->stream, (const double2*)R.d_H, (const double2*)R.d_Z, (double2*)R.d_Y, Q, Qp, D);
    }
    HZ_TRY_HIP(hipGetLastError());
    hipLaunchKernelGGL(kinv, dim3((unsigned)D), dim3(r4 ? kF >> 2 : kFftThreads), fft_lds(), h->stream, a);
    HZ_TRY_HIP(hipGetLastError());
    if (e) HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
    R.hcur ^= 1;   // the inverse kernel wrote the history after the call
    R.run = std::min(R.run + n, 1L << 60);
    // end state: band states joined from the side stream (EAGER) or computed when needed (LAZY);
    // smoothers and x history were written by the inverse kernel
    if (lazy) {
        R.implicit = true;
    } else if (side) {
        HZ_TRY_HIP(hipStreamWaitEvent(h->stream, R.ev_join, 0));
        R.implicit = false;
    } else {
        HZ_TRY(resp_states(h, h->d_ystate[h->scur ^ 1]));
        R.implicit = false;
    }
    if (e) HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
    h->scur ^= 1;
    h->xcur ^= 1;
    h->prof_launches += h->prof ? 1 : 0;
    ++R.calls;
    fb_mirror_advance(h, n);
    return HZ_OK;
}

void fb_resp_free(hz_fb* h) {
    hz_fb::Resp& R = h->resp;
    if (R.side) (void)hipStreamSynchronize(R.side);
    for (double* p : {R.d_hist[0], R.d_hist[1], R.d_h, R.d_hpart, R.d_coef, R.d_zero, R.d_H, R.d_Z, R.d_Y, R.d_tw,
                      R.d_eg, R.d_epart})
        if (p) (void)hipFree(p);
    if (R.ev_fork) (void)hipEventDestroy(R.ev_fork);
    if (R.ev_join) (void)hipEventDestroy(R.ev_join);
    if (R.side) (void)hipStreamDestroy(R.side);
    R = hz_fb::Resp();
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
