// hz_freezer.hip -- Freezer<N> (spectral freeze) on MI355X (gfx950).
//
// Replaces src/fourier.h:389-562 (Freezer) with its FFrame / IFrame / DFrame helpers
// (236-387) and the Delay<double>(1, N) dry path.  Per sample the reference does
//     write(x): frames i = 0..M-1 write their windowed spot; frame i at spot 0 processes
//               frame (i-1) mod M (FFT, norms = |X|^2, phases = arg X);
//     frozen:   out = sum over slots i of Re(IFrame[iqueue[i]][spot_i]) * halfhann(spot_i / N),
//               the slot at spot 0 drawing next = rand() % (M-2) (+2 past `excluded`) and
//               repopulating IFrame[next] = IFFT(polar(sqrt(dnorm), fmod(dphase, 2 PI)));
//               out /= N;
//     else:     out = Delay(N)(x) (its input ring written only while unfrozen).
//
// MI355X design.  Everything sequential is host bookkeeping: writehead / readhead /
// iqueue / iindex / rand() draws follow the reference exactly, and because the DFrames only
// change at a freeze, every repopulation of IFrame k in one frozen period yields the same
// frame.  So the device work per freeze is one batched pass -- the M frames' last
// processing states gathered from the input history (with the reference's write/process
// order inside write()), forward FFTs, polarization, the M-2 DFrames and their inverse
// FFTs -- and the output is a block-parallel gather: thread per sample, its run (frozen /
// dry) and slot map (IFrame index, which version) found by binary search.  The dry path
// reads x(t - N) or the Delay ring as it stood when the current unfrozen stretch began.
//
// Layout in HBM: input history ring [H]; window [N]; per freeze norms/phases [M][N]
// (bit-reversed bins) and IFrames [M][N] (Re only: the output takes the real part; stored times
// the output window);
// IFrame state [M][N]; Delay ring snapshots [S][N+1]; runs and slot maps per call.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "hz_common.h"
#include "hz_fft.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxN = 8192;
constexpr long kChunk = 1L << 20;   // samples per chunk: a 10 s call at 48 kHz is one output launch

struct FrzRun {
    long t0;        // first sample of the run (absolute)
    long u0;        // dry run: start of its unfrozen stretch
    int frozen;     // 1 frozen, 0 dry
    int rh0;        // frozen: readhead at t0
    int map;        // frozen: slot map index (M entries)
    int snap;       // dry: Delay ring snapshot index
};

struct SlotSrc {
    int k;          // IFrame index
    int src;        // -1: IFrame state at chunk start, 0: the open period's frames (frozen
                    // since an earlier chunk), q >= 1: the q-th freeze of this chunk
};

// x(tau) for a time within reach: the call's input or the history ring
__device__ __forceinline__ double hist_at(const double* in, long T0, const double* ring, long mask, long tau) {
    return tau >= T0 ? in[tau - T0] : ring[tau & mask];
}

// One workgroup per frame j: its data at its last process() before the freeze at tf
// (fourier.h:448-466 incl. the write/process order), FFT, norms and phases (bit-reversed)
__global__ __launch_bounds__(kThreads) void frz_frame_kernel(const double* in, long T0, const double* ring, long mask,
                                                             const double* win, const double2* tw, int N, int lg,
                                                             int stride, int M, int size, long tf, double* norm,
                                                             double* phase) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + N;
    const int j = blockIdx.x;
    const long r = (long)((j + 1) % M) * stride;                   // processed when frame j+1 hits spot 0
    const long tp = (tf - 1) - ((((tf - 1 - r) % size) + size) % size);
    for (int s = threadIdx.x; s < N; s += blockDim.x) {
        double v = 0.0;
        if (tp >= 0 && s < size) {
            long tau = tp - ((((tp - (long)j * stride - s) % size) + size) % size);
            if (j == M - 1 && tau == tp) tau -= size;   // frame M-1 is processed before its own write
            if (tau >= 0) v = hist_at(in, T0, ring, mask, tau);
        }
        re[s] = win[s] * v;
        im[s] = win[s] * 0.0;
    }
    __syncthreads();
    hz::lds_fft_fwd(re, im, N, lg, tw);
    for (int p = threadIdx.x; p < N; p += blockDim.x) {
        const double a = re[p], b = im[p];
        norm[(long)j * N + p] = tp >= 0 ? a * a + b * b : 0.0;   // never processed: zero (reference: uninitialised)
        phase[(long)j * N + p] = tp >= 0 ? atan2(b, a) : 0.0;
    }
}

// One workgroup per DFrame d: freeze() refreshes d = (excluded + i) mod M, i = 1..M-2
// (norms of frame d+1, phases[d+1] - phases[d]); the others keep their state from earlier
// freezes -- and the frame draw can pick excluded - 1, one of those (fourier.h:473-474 vs
// 503-505).  Then the IFrame IFFT(polar(sqrt(dnorm), fmod(dphase, 2 PI))), Re part.
__global__ __launch_bounds__(kThreads) void frz_iframe_kernel(const double* norm, const double* phase,
                                                              double* dnorm, double* dphase, const double2* tw,
                                                              const double* win, int N, int lg, int M, int excluded,
                                                              double* ifr) {
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* re = lds;
    double* im = lds + N;
    const int d = blockIdx.x, s = (d + 1) % M;
    const int i = (d - excluded + M) % M;
    const bool refresh = i >= 1 && i <= M - 2;
    for (int p = threadIdx.x; p < N; p += blockDim.x) {
        double dn, dph;
        if (refresh) {   // DFrame::populate (fourier.h:371-378)
            dn = norm[(long)s * N + p];
            dph = phase[(long)s * N + p] - phase[(long)d * N + p];
            dnorm[(long)d * N + p] = dn;
            dphase[(long)d * N + p] = dph;
        } else {
            dn = dnorm[(long)d * N + p];
            dph = dphase[(long)d * N + p];
        }
        const double voc = fmod(dph, 2 * hz::kPI);
        const double rr = sqrt(dn);
        re[p] = rr * cos(voc);   // std::polar
        im[p] = rr * sin(voc);
    }
    __syncthreads();
    hz::lds_fft_inv(re, im, N, lg, tw);
    // stored times the output window: the output's product Re(IFrame[spot]) * halfhann(spot)
    // (fourier.h:516), one rounding as there, made once per frame instead of per sample and slot
    for (int k = threadIdx.x; k < N; k += blockDim.x) ifr[(long)d * N + k] = re[k] * win[k];
}

// Delay ring snapshots: snap[q+1] = snap[q] after the writes of dry stretch q = [a_q, b_q)
__global__ void frz_snap_kernel(const double* in, long T0, const double* ring, long mask, const long* stretch,
                                int nst, int N, double* snap) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int S = N + 1;
    if (s >= S) return;
    double v = snap[s];
    for (int q = 0; q < nst; ++q) {
        const long a = stretch[2 * q], b = stretch[2 * q + 1];
        // latest tau in [a, b) with tau = s (mod N+1)
        const long tau = (b - 1) - ((((b - 1 - s) % S) + S) % S);
        if (tau >= a && tau >= 0) v = hist_at(in, T0, ring, mask, tau);
        snap[(long)(q + 1) * S + s] = v;
    }
}

struct OutArgs {
    const double* in;
    double* out;
    double* ring;
    long mask, T0, n;
    const FrzRun* runs;
    const int* blk_run;      // [workgroups + 1] the run holding each workgroup's first sample
    int nruns;
    const SlotSrc* maps;
    const double* ifstate;   // [M][N]
    const double* ifopen;    // [M][N]
    const double* ifnew;     // [P][M][N]
    const double* snaps;     // [S][N+1]
    int N, M, stride, readsize;
};

__global__ __launch_bounds__(kThreads) void frz_out_kernel(OutArgs a) {
#pragma clang fp contract(off)
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n) return;
    const long t = a.T0 + j;
    // last run with t0 <= t, within this workgroup's runs (host table: one dependent load or two
    // instead of a search over the chunk's ~2 runs per stride)
    int lo = a.blk_run[blockIdx.x], hi = a.blk_run[blockIdx.x + 1];
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.runs[mid].t0 <= t) lo = mid;
        else hi = mid - 1;
    }
    const FrzRun r = a.runs[lo];
    const int N = a.N;
    double output = 0;
    if (r.frozen) {
        // frozen runs end at the next populate point (<= stride samples), so rh0 + (t - t0) and
        // rh - i stride stay within one readsize of [0, readsize): a compare instead of a division
        const long d = t - r.t0;
        int rh = d < a.readsize ? r.rh0 + (int)d : (int)((r.rh0 + d) % a.readsize);
        if (rh >= a.readsize) rh -= a.readsize;
        const SlotSrc* map = a.maps + (long)r.map * a.M;
        for (int i = 0; i < a.M; ++i) {   // fourier.h:493-521, slot order
            int spot = rh - i * a.stride;   // (rh - i stride + readsize) mod readsize, i stride < readsize
            if (spot < 0) spot += a.readsize;
            if (spot < N) {
                const SlotSrc m = map[i];
                const double* f = m.src < 0    ? a.ifstate
                                  : m.src == 0 ? a.ifopen
                                               : a.ifnew + (long)(m.src - 1) * a.M * N;
                output += f[(long)m.k * N + spot];   // (IFrames stored windowed: frz_iframe_kernel)
            }
        }
        output /= N;
    } else {   // Delay<double>(1, N): the input ring's slot (t + 1) mod (N + 1)
        const double v = t - N >= r.u0 ? hist_at(a.in, a.T0, a.ring, a.mask, t - N)
                                       : a.snaps[(long)r.snap * (N + 1) + (t + 1) % (N + 1)];
        output = 0.0 + v;
    }
    a.out[j] = output;
    a.ring[t & a.mask] = a.in[j];   // the history ring is >= 2 size + 2 N + chunk: no reader of this slot
}

// IFrame state <- the latest content of each frame (src[q]: -1 unchanged, 0 the open period's
// frames, p >= 1 the p-th freeze of the chunk), one launch for all M frames
// (row M: Delay ring snapshot 0 <- the last one, when the chunk ended dry stretches)
__global__ __launch_bounds__(256) void frz_carry_kernel(double* ifstate, const double* ifopen, const double* ifnew,
                                                         const int* src, int M, int N, double* snap, int nsnap) {
    const int q = blockIdx.y, e = blockIdx.x * blockDim.x + threadIdx.x;
    if (q == M) {
        if (nsnap > 1 && e <= N) snap[e] = snap[(size_t)(nsnap - 1) * (N + 1) + e];
        return;
    }
    const int sq = src[q];
    if (sq < 0 || e >= N) return;
    const double* f = sq == 0 ? ifopen : ifnew + (size_t)(sq - 1) * M * N;
    ifstate[(size_t)q * N + e] = f[(size_t)q * N + e];
}

int ilog2(int N) {
    int lg = 0;
    while ((1 << lg) < N) ++lg;
    return lg;
}

}  // namespace

struct hz_frz {
    int N = 0, laps = 0, stride = 0, M = 0, size = 0, lg = 0, device = 0;
    long T = 0;
    bool frozen = false;
    int readhead = 0, iindex = 0, excluded = 0;
    std::vector<int> iqueue;
    long u0 = 0;                  // start of the current unfrozen stretch (the Delay ring snapshot is at u0)
    long mask = 0;
    long chunk = 0;               // samples per chunk (kChunk; env HZ_FRZ_CHUNK at create, tests)
    double *d_ring = nullptr, *d_win = nullptr, *d_norm = nullptr, *d_phase = nullptr, *d_ifstate = nullptr;
    double* d_ifopen = nullptr;   // [M][N] IFrames of the freeze period open at chunk start
    double *d_dnorm = nullptr, *d_dphase = nullptr;   // [M][N] DFrame state (persists across freezes)
    double* d_ifnew = nullptr;    // [P][M][N] IFrames of the chunk's freezes
    size_t ifnew_cap = 0;         // periods
    double* d_snap = nullptr;     // [S][N+1]; snapshot 0 = the ring at u0
    size_t snap_cap = 0;
    double2* d_tw = nullptr;
    void* d_tab = nullptr;        // runs + maps + stretches of one chunk
    // host side of the chunk tables, kept across chunks (capacity reused: no regrowth copies); the
    // upload goes from pinned staging (an async DMA, no bounce copy)
    std::vector<FrzRun> v_runs;
    std::vector<SlotSrc> v_maps;
    char* h_tab = nullptr;        // pinned
    size_t h_tab_cap = 0;
    size_t tab_cap = 0;
    double *d_in = nullptr, *d_out = nullptr;
    size_t in_cap = 0, out_cap = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool prof = false;                 // HIP events around each frz_out_kernel launch
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    long launches = 0;
};

namespace {

int frz_check(hz_frz* h) {
    if (!h) {
        hz::set_error("null hz_frz handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    return HZ_OK;
}

int grow(void** p, size_t* cap, size_t bytes, hipStream_t st) {
    if (bytes <= *cap) return HZ_OK;
    HZ_TRY_HIP(hipStreamSynchronize(st));
    if (*p) HZ_TRY_HIP(hipFree(*p));
    *p = nullptr;
    HZ_TRY_HIP(hipMalloc(p, bytes));
    *cap = bytes;
    return HZ_OK;
}

// One chunk [T0, T0 + n) with its events (at relative to T0, ascending).
int frz_chunk(hz_frz* h, const double* d_in, double* d_out, long n, const hz_frz_event* ev, int nev) {
    const int N = h->N, M = h->M;
    const long T0 = h->T;
    std::vector<FrzRun>& runs = h->v_runs;
    std::vector<SlotSrc>& maps = h->v_maps;
    runs.clear();
    maps.clear();
    std::vector<long> stretch;         // dry stretches ended in this chunk: [a, b) pairs
    std::vector<long> period_tf;       // freeze transitions in this chunk
    std::vector<int> period_excl;
    std::vector<int> last_src(M, -1);  // latest IFrame content source in this chunk
    int snap_idx = 0;                  // current dry stretch's snapshot (0 = carried in)

    auto map_now = [&]() {
        const int idx = (int)(maps.size() / M);
        for (int i = 0; i < M; ++i) maps.push_back({h->iqueue[i], last_src[h->iqueue[i]]});
        return idx;
    };
    auto open_run = [&](long t) {
        FrzRun r{};
        r.t0 = t;
        r.frozen = h->frozen ? 1 : 0;
        r.rh0 = h->readhead;
        r.u0 = h->u0;
        r.snap = snap_idx;
        r.map = h->frozen ? map_now() : 0;
        runs.push_back(r);
    };
    auto apply = [&](const hz_frz_event& e, long t) {
        if (e.kind == HZ_FRZ_FREEZE) {   // fourier.h:468-479
            if (!h->frozen) {
                stretch.push_back(h->u0);
                stretch.push_back(t);
                ++snap_idx;
                h->excluded = (int)((t % h->size) / h->stride);   // origin / stride
                period_tf.push_back(t);
                period_excl.push_back(h->excluded);
            }
            h->readhead = 0;
            h->frozen = true;
        } else {   // fourier.h:481-485
            if (h->frozen) h->u0 = t;
            h->frozen = false;
        }
    };

    // the freeze transitions depend on the events alone (fourier.h:468-479): their frame / DFrame /
    // IFrame passes are launched first and run on the device while the host builds the runs below
    std::vector<long> pre_tf;
    std::vector<int> pre_excl;
    {
        bool fz = h->frozen;
        for (int e = 0; e < nev; ++e) {
            const long te = T0 + ev[e].at;
            if (ev[e].kind == HZ_FRZ_FREEZE) {
                if (!fz) {
                    pre_tf.push_back(te);
                    pre_excl.push_back((int)((te % h->size) / h->stride));
                }
                fz = true;
            } else {
                fz = false;
            }
        }
    }
    const int P = (int)pre_tf.size();
    HZ_TRY(grow((void**)&h->d_ifnew, &h->ifnew_cap, sizeof(double) * (size_t)std::max(1, P) * M * N, h->stream));
    const size_t lds = sizeof(double) * 2 * N;
    const int ft = std::min(kThreads, std::max(64, N / 4));   // within the kernels' launch bounds
    for (int q = 0; q < P; ++q) {   // new period q is source q + 1
        hipLaunchKernelGGL(frz_frame_kernel, dim3(M), dim3(ft), lds, h->stream, d_in, T0, (const double*)h->d_ring,
                           h->mask, (const double*)h->d_win, (const double2*)h->d_tw, N, h->lg, h->stride, M, h->size,
                           pre_tf[q], h->d_norm, h->d_phase);
        HZ_TRY_HIP(hipGetLastError());
        hipLaunchKernelGGL(frz_iframe_kernel, dim3(M), dim3(ft), lds, h->stream, (const double*)h->d_norm,
                           (const double*)h->d_phase, h->d_dnorm, h->d_dphase, (const double2*)h->d_tw,
                           (const double*)h->d_win, N, h->lg, M, pre_excl[q], h->d_ifnew + (size_t)q * M * N);
        HZ_TRY_HIP(hipGetLastError());
    }

    std::vector<SlotSrc> before(M);
    int k = 0;
    long t = T0;
    const long T1 = T0 + n;
    while (t < T1) {
        for (; k < nev && T0 + ev[k].at == t; ++k) apply(ev[k], t);
        const long t_ev = k < nev ? T0 + ev[k].at : T1;
        if (!h->frozen) {
            open_run(t);
            t = t_ev;
            continue;
        }
        // frozen: one run per populate sample (its split map) and one until the next
        const int p = (int)period_tf.size();   // this period's frames: 0 open (earlier chunk), q >= 1 new
        while (t < t_ev) {
            const int rh = h->readhead;
            if (rh % h->stride == 0 && rh / h->stride < M) {   // slot i = rh / stride at spot 0
                const int i = rh / h->stride;
                // before the populate: slots <= i; after: slots > i
                for (int q = 0; q < M; ++q) before[q] = {h->iqueue[q], last_src[h->iqueue[q]]};
                int next = std::rand() % (M - 2);   // fourier.h:503-509
                if (next >= h->excluded) next += 2;
                h->iindex = (h->iindex + 1) % M;
                h->iqueue[h->iindex] = next;
                last_src[next] = p;
                FrzRun r{};
                r.t0 = t;
                r.frozen = 1;
                r.rh0 = rh;
                r.map = (int)(maps.size() / M);
                for (int q = 0; q < M; ++q)
                    maps.push_back(q <= i ? before[q] : SlotSrc{h->iqueue[q], last_src[h->iqueue[q]]});
                runs.push_back(r);
                h->readhead = (h->readhead + 1) % h->size;
                ++t;
                continue;
            }
            // no populate until readhead reaches the next multiple of stride
            const long to_next = h->stride - (rh % h->stride);
            const long len = std::min(t_ev - t, to_next);
            open_run(t);
            h->readhead = (int)((h->readhead + len) % h->size);
            t += len;
        }
    }
    for (; k < nev; ++k) apply(ev[k], T1);   // events at the chunk end (at == n)

    if (period_tf != pre_tf || period_excl != pre_excl) {   // (the pre-pass restates apply())
        hz::set_error("hz_frz: freeze transitions disagree with the pre-pass");
        return HZ_E_STATE;
    }
    // tables: runs, maps, stretches, each output workgroup's first run, the carry sources
    const size_t b_runs = runs.size() * sizeof(FrzRun), b_maps = std::max<size_t>(1, maps.size()) * sizeof(SlotSrc);
    const size_t b_st = std::max<size_t>(2, stretch.size()) * sizeof(long);
    const size_t nsnap = stretch.size() / 2 + 1;
    const long nb = (n + kThreads - 1) / kThreads;
    const size_t b_blk = sizeof(int) * (size_t)(nb + 1), b_src = sizeof(int) * (size_t)M;
    HZ_TRY(grow(&h->d_tab, &h->tab_cap, b_runs + b_maps + b_st + b_blk + b_src + 64, h->stream));
    const size_t b_tab = b_runs + b_maps + b_st + b_blk + b_src;
    if (b_tab > h->h_tab_cap) {   // (the previous chunk's upload finished: every chunk ends synchronised)
        if (h->h_tab) HZ_TRY_HIP(hipHostFree(h->h_tab));
        h->h_tab = nullptr;
        h->h_tab_cap = 0;
        HZ_TRY_HIP(hipHostMalloc((void**)&h->h_tab, b_tab * 2));
        h->h_tab_cap = b_tab * 2;
    }
    char* hb = h->h_tab;
    std::memcpy(hb, runs.data(), b_runs);
    if (!maps.empty()) std::memcpy(hb + b_runs, maps.data(), maps.size() * sizeof(SlotSrc));
    if (!stretch.empty()) std::memcpy(hb + b_runs + b_maps, stretch.data(), stretch.size() * sizeof(long));
    int* blk = (int*)(hb + b_runs + b_maps + b_st);
    for (long b = 0, r = 0; b < nb; ++b) {   // runs ascend in t0: the run at each workgroup start
        const long tb = T0 + b * kThreads;
        while (r + 1 < (long)runs.size() && runs[r + 1].t0 <= tb) ++r;
        blk[b] = (int)r;
    }
    // a workgroup's runs lie in [blk[b], blk[b + 1]] (the run at the next workgroup's start)
    blk[nb] = runs.empty() ? 0 : (int)runs.size() - 1;
    std::memcpy(hb + b_runs + b_maps + b_st + b_blk, last_src.data(), b_src);
    HZ_TRY_HIP(hipMemcpyAsync(h->d_tab, hb, b_tab, hipMemcpyHostToDevice, h->stream));
    const char* tab = (const char*)h->d_tab;
    // Delay ring snapshots after each dry stretch that ended here
    if (nsnap > h->snap_cap / (sizeof(double) * (N + 1))) {
        double* ns = nullptr;
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        HZ_TRY_HIP(hipMalloc(&ns, sizeof(double) * (N + 1) * nsnap));
        HZ_TRY_HIP(hipMemcpy(ns, h->d_snap, sizeof(double) * (N + 1), hipMemcpyDeviceToDevice));
        HZ_TRY_HIP(hipFree(h->d_snap));
        h->d_snap = ns;
        h->snap_cap = sizeof(double) * (N + 1) * nsnap;
    }
    if (nsnap > 1) {
        hipLaunchKernelGGL(frz_snap_kernel, dim3((N + 1 + 255) / 256), dim3(256), 0, h->stream, d_in, T0,
                           (const double*)h->d_ring, h->mask, (const long*)(tab + b_runs + b_maps),
                           (int)(nsnap - 1), N, h->d_snap);
        HZ_TRY_HIP(hipGetLastError());
    }
    OutArgs a;
    a.in = d_in;
    a.out = d_out;
    a.ring = h->d_ring;
    a.mask = h->mask;
    a.T0 = T0;
    a.n = n;
    a.runs = (const FrzRun*)tab;
    a.blk_run = (const int*)(tab + b_runs + b_maps + b_st);
    a.nruns = (int)runs.size();
    a.maps = (const SlotSrc*)(tab + b_runs);
    a.ifstate = h->d_ifstate;
    a.ifopen = h->d_ifopen;
    a.ifnew = h->d_ifnew;
    a.snaps = h->d_snap;
    a.N = N;
    a.M = M;
    a.stride = h->stride;
    a.readsize = h->size;
    if (n > 0) {
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
        hipLaunchKernelGGL(frz_out_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                           h->stream, a);
        HZ_TRY_HIP(hipGetLastError());
        if (e) {
            HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
            ++h->launches;
        }
    }
    // carry: IFrame state <- latest content (before the open period's frames are replaced)
    // (and snapshot 0 <- the Delay ring at the start of the current or next dry stretch: row M)
    if (nsnap > 1 || std::any_of(last_src.begin(), last_src.end(), [](int v) { return v >= 0; })) {
        hipLaunchKernelGGL(frz_carry_kernel, dim3((unsigned)((N + 1 + 255) / 256), (unsigned)M + 1), dim3(256), 0,
                           h->stream, h->d_ifstate, (const double*)h->d_ifopen, (const double*)h->d_ifnew,
                           (const int*)(tab + b_runs + b_maps + b_st + b_blk), M, N, h->d_snap, (int)nsnap);
        HZ_TRY_HIP(hipGetLastError());
    }
    // a period still open at the chunk end: its frames for later chunks
    if (h->frozen && P > 0)
        HZ_TRY_HIP(hipMemcpyAsync(h->d_ifopen, h->d_ifnew + (size_t)(P - 1) * M * N, sizeof(double) * M * N,
                                  hipMemcpyDeviceToDevice, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // the pinned tables are rewritten by the next chunk
    h->T += n;
    return HZ_OK;
}

}  // namespace

extern "C" {

int hz_frz_create(int N, int laps, double width, int device, hz_frz** out) {
    if (!out || N < 4 || N > kMaxN || (N & (N - 1)) != 0) {
        hz::set_error("hz_frz_create: N must be a power of two in [4, %d]", kMaxN);
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_frz* h = new (std::nothrow) hz_frz();
    if (!h) return HZ_E_ALLOC;
    width = std::max(width, 1.0);   // fourier.h:397-402
    laps = std::max(laps, 2);
    h->N = N;
    h->laps = laps;
    h->stride = N / laps;
    h->M = (int)(width * laps) + 1;
    h->size = h->M * h->stride;
    h->lg = ilog2(N);
    h->device = device;
    h->iqueue.assign(h->M, 0);
    if (h->stride < 1 || h->M < 3 || h->M > 4096) {
        delete h;
        hz::set_error("hz_frz_create: unsupported geometry (laps %d, width %g)", laps, width);
        return HZ_E_INVALID;
    }
    long H = 1;
    h->chunk = kChunk;
    if (const char* e = std::getenv("HZ_FRZ_CHUNK")) {   // (tests: the launch split at a shorter length)
        const long c = std::atol(e);
        if (c >= 4096 && c <= kChunk) h->chunk = c;
    }
    while (H < 2L * h->size + 2L * N + h->chunk + 2) H <<= 1;
    h->mask = H - 1;
    std::vector<double> win(N);
    for (int k = 0; k < N; ++k) win[k] = std::sqrt(0.5 * (1 - std::cos(2 * hz::kPI * (k / (double)N))));   // halfhann
    std::vector<double2> tw(N / 2);
    const long double pi = acosl(-1.0L);
    for (int k = 0; k < N / 2; ++k) {
        const long double ang = -2.0L * pi * k / N;
        tw[k] = make_double2((double)cosl(ang), (double)sinl(ang));
    }
    const size_t MN = (size_t)h->M * N;
    bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMalloc(&h->d_ring, sizeof(double) * H) == hipSuccess;
    ok = ok && hipMalloc(&h->d_win, sizeof(double) * N) == hipSuccess;
    ok = ok && hipMalloc(&h->d_tw, sizeof(double2) * (N / 2)) == hipSuccess;
    ok = ok && hipMalloc(&h->d_norm, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMalloc(&h->d_phase, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMalloc(&h->d_ifstate, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMalloc(&h->d_ifopen, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMalloc(&h->d_dnorm, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMalloc(&h->d_dphase, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMemset(h->d_dnorm, 0, sizeof(double) * MN) == hipSuccess;   // reference: uninitialised
    ok = ok && hipMemset(h->d_dphase, 0, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMalloc(&h->d_snap, sizeof(double) * (N + 1)) == hipSuccess;
    if (ok) h->snap_cap = sizeof(double) * (N + 1);
    ok = ok && hipMemset(h->d_ring, 0, sizeof(double) * H) == hipSuccess;
    ok = ok && hipMemset(h->d_ifstate, 0, sizeof(double) * MN) == hipSuccess;   // IFrame data zeroed (fourier.h:308)
    ok = ok && hipMemset(h->d_ifopen, 0, sizeof(double) * MN) == hipSuccess;
    ok = ok && hipMemset(h->d_snap, 0, sizeof(double) * (N + 1)) == hipSuccess;   // Buffer zeroed
    ok = ok && hipMemcpy(h->d_win, win.data(), sizeof(double) * N, hipMemcpyHostToDevice) == hipSuccess;
    ok = ok && hipMemcpy(h->d_tw, tw.data(), sizeof(double2) * (N / 2), hipMemcpyHostToDevice) == hipSuccess;
    static bool attr = false;
    if (ok && !attr) {
        const int lds = (int)(sizeof(double) * 2 * kMaxN);
        ok = hipFuncSetAttribute((const void*)frz_frame_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds) ==
                 hipSuccess &&
             hipFuncSetAttribute((const void*)frz_iframe_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds) ==
                 hipSuccess;
        attr = ok;
    }
    if (!ok) {
        hz::set_error("hz_frz_create: device allocation failed");
        for (void* p : {(void*)h->d_ring, (void*)h->d_win, (void*)h->d_tw, (void*)h->d_norm, (void*)h->d_phase,
                        (void*)h->d_ifstate, (void*)h->d_ifopen, (void*)h->d_dnorm, (void*)h->d_dphase,
                        (void*)h->d_snap})
            if (p) (void)hipFree(p);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        delete h;
        return HZ_E_ALLOC;
    }
    h->own_stream = true;
    *out = h;
    return HZ_OK;
}

int hz_frz_destroy(hz_frz* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->d_ring, (void*)h->d_win, (void*)h->d_tw, (void*)h->d_norm, (void*)h->d_phase,
                    (void*)h->d_ifstate, (void*)h->d_ifopen, (void*)h->d_dnorm, (void*)h->d_dphase,
                    (void*)h->d_ifnew, (void*)h->d_snap, h->d_tab, (void*)h->d_in,
                    (void*)h->d_out})
        if (p) (void)hipFree(p);
    if (h->h_tab) (void)hipHostFree(h->h_tab);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_frz_profile(hz_frz* h, int enable) {
    HZ_TRY(frz_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    h->prof = enable != 0;
    h->ev_used = 0;
    h->launches = 0;
    return HZ_OK;
}

int hz_frz_profile_read(hz_frz* h, double* ms, long* launches) {
    HZ_TRY(frz_check(h));
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

int hz_frz_info(hz_frz* h, int* stride, int* frames, int* frozen) {
    if (!h) return HZ_E_INVALID;
    if (stride) *stride = h->stride;
    if (frames) *frames = h->M;
    if (frozen) *frozen = h->frozen ? 1 : 0;
    return HZ_OK;
}

int hz_frz_process_device(hz_frz* h, const double* d_in, double* d_out, size_t n, const hz_frz_event* ev, int nev) {
    HZ_TRY(frz_check(h));
    if ((n && (!d_in || !d_out)) || nev < 0 || (nev && !ev)) return HZ_E_INVALID;
    for (int k = 0; k < nev; ++k)
        if (ev[k].at < 0 || ev[k].at > (long)n || (k && ev[k].at < ev[k - 1].at) ||
            (ev[k].kind != HZ_FRZ_FREEZE && ev[k].kind != HZ_FRZ_UNFREEZE)) {
            hz::set_error("hz_frz_process: event %d invalid (0 <= at <= n ascending, kind freeze/unfreeze)", k);
            return HZ_E_INVALID;
        }
    long done = 0;
    int k0 = 0;
    do {
        const long m = std::min<long>((long)n - done, h->chunk);
        int k1 = k0;
        while (k1 < nev && (ev[k1].at < done + m || (done + m == (long)n && ev[k1].at <= done + m))) ++k1;
        std::vector<hz_frz_event> local(ev + k0, ev + k1);
        for (auto& e : local) e.at -= done;
        HZ_TRY(frz_chunk(h, d_in + done, d_out + done, m, local.data(), (int)local.size()));
        done += m;
        k0 = k1;
    } while (done < (long)n);
    return HZ_OK;
}

int hz_frz_process(hz_frz* h, const double* in, double* out, size_t n, const hz_frz_event* ev, int nev) {
    HZ_TRY(frz_check(h));
    if ((n && (!in || !out)) || nev < 0 || (nev && !ev)) return HZ_E_INVALID;
    if (n) {
        HZ_TRY(grow((void**)&h->d_in, &h->in_cap, sizeof(double) * n, h->stream));
        HZ_TRY(grow((void**)&h->d_out, &h->out_cap, sizeof(double) * n, h->stream));
        HZ_TRY_HIP(hipMemcpyAsync(h->d_in, in, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
    }
    HZ_TRY(hz_frz_process_device(h, h->d_in, h->d_out, n, ev, nev));
    if (n) HZ_TRY_HIP(hipMemcpyAsync(out, h->d_out, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_frz_freeze(hz_frz* h) {
    const hz_frz_event e{0, HZ_FRZ_FREEZE};
    return hz_frz_process_device(h, nullptr, nullptr, 0, &e, 1);
}

int hz_frz_unfreeze(hz_frz* h) {
    const hz_frz_event e{0, HZ_FRZ_UNFREEZE};
    return hz_frz_process_device(h, nullptr, nullptr, 0, &e, 1);
}

int hz_frz_set_stream(hz_frz* h, void* stream) {
    HZ_TRY(frz_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) HZ_TRY_HIP(hipStreamDestroy(h->stream));
    h->stream = (hipStream_t)stream;
    h->own_stream = false;
    return HZ_OK;
}

int hz_frz_synchronize(hz_frz* h) {
    HZ_TRY(frz_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

}  // extern "C"
