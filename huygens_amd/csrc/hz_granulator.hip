// hz_granulator.hip -- Granulator<double> on MI355X (gfx950).
//
// Replaces src/granulator.h:12-127 (request 51-79, tick 81-86, operator() 88-104) with
// its Buffer<double> source (src/buffer.h:9-86) and the FUNCTIONAL hann window
// (src/wave.h:65-70,148), in the per-sample order of tests/granny.cpp:34-56:
//     source.write(x); y = sum over active voices v (ascending):
//         gains_v * source(offsets_v + (1 - speeds_v) ticks_v) * hann(ticks_v / sizes_v),
//     deactivating v after its read once ticks_v >= sizes_v;  <requests>;  ticks++.
//
// Host/device split.  Voice allocation (first inactive voice) and every grain's lifetime
// are closed-form: a grain requested after the read of sample t first reads at t+1 with
// ticks0 (1 if the tick of t follows the request, else 0) and reads until the first
// ticks with (double)ticks >= sizes, so the host keeps a grain list {voice, t_first,
// t_end, ticks0, parameters} and knows exactly which voices are free at any request.
// The device then evaluates a block with no sequential dependence: thread per output
// sample, looping over the block's grains in voice order (the reference's summation
// order), each an interpolated ring read and a hann weight.
//
// Source ring.  The reference reads slot (origin - c + size) mod 2^32 mod size of a
// `size`-slot ring whose slot s, at time t, holds the latest sample written at a time
// tau <= t with tau = t - ((origin_t - s) mod size) (0 if tau < 0).  The device keeps a
// time-indexed ring of C >= size + kChunk samples (a power of two); a launch's input is
// copied into it first, so every read is ring[tau mod C]: a read reaches back less than `size`
// samples, so slot tau mod C still holds x(tau) (its next writer, tau + C, lies past the
// launch), and a tau < 0 slot is still the ring's initial zero.  The uint32 index arithmetic
// is kept verbatim (bit-exact) where it can wrap; for 0 <= center < size it reduces to
// tau = t - center (tau = t - center - 1, or t when center + 1 = size, for the second tap).
//
// Layout in HBM: ring [C] doubles; grains [G] x 64 B per block (uploaded once per call).
#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <cmath>
#include <cstring>
#include <deque>
#include <limits>
#include <new>
#include <vector>

#include "hz_common.h"
#include "hz_rt.h"

namespace {

constexpr int kThreads = 256;
constexpr long kChunk = 1L << 18;             // samples per launch
constexpr long kTile = 4096;                  // samples sharing one grain list (multiple of kThreads)
constexpr long kNever = 1L << 62;             // t_end of a grain that never finishes (NaN/inf size)

typedef hz_rt::Grain GrainDev;   // one 64-B line (shared with the per-sample server)

struct GranArgs {
    double* out;
    double* ring;         // time-indexed source ring (C = mask + 1 samples)
    const GrainDev* g;    // the call's grains, voice-major
    const int* tile_off;  // per kTile samples of the call: [tile_off[k], tile_off[k+1]) in tile_idx
    const int* tile_idx;  // grains overlapping the tile, in voice order
    long tile_base;       // tile index of this launch's first sample
    long T0, n, mask;
    unsigned size, o0;    // Buffer size and origin at time T0
    unsigned long fm;     // fastmod multiplier for `size`: 2^64 / size rounded up (0 for size 1)
    unsigned wrap1;       // (2^32 - 1) % size: the second tap's slot when the first index is 0 mod 2^32
    int fastcos;          // cos_0_2pi for the window (HZ_GRAN_LIBCOS=1: the library cos, A/B)
};

// x mod size for any uint32 x, without a divide (Lemire, Kaser & Kurz 2019, "fastmod")
__device__ __forceinline__ unsigned fastmod(unsigned x, unsigned long fm, unsigned size) {
    const unsigned long low = fm * (unsigned long)x;
    return (unsigned)__umul64hi(low, (unsigned long)size);
}

constexpr int kUnroll = 4;   // grains in flight per thread: their 2 x 4 gathers issue together

__global__ __launch_bounds__(kThreads) void gran_kernel(GranArgs a) {
#pragma clang fp contract(off)
    // the wave's first sample: grains that miss the wave's 64 samples are skipped (scalar branch)
    const long tw = a.T0 + (long)blockIdx.x * blockDim.x + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63);
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n) return;
    const long t = a.T0 + j;
    const unsigned size = a.size;
    const unsigned origin = (unsigned)(((unsigned long)a.o0 + (unsigned long)j) % size);
    double out = 0;
    const long k = a.tile_base + (long)blockIdx.x * blockDim.x / kTile;
    const int i0 = a.tile_off[k], ng = a.tile_off[k + 1] - i0;
    const int* idx = a.tile_idx + i0;
    for (int e0 = 0; e0 < ng; e0 += kUnroll) {
        bool wv[kUnroll], act[kUnroll];
        unsigned ticks[kUnroll];
        double disp[kUnroll], v0[kUnroll], v1[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {   // phase 1: indices and gathers of kUnroll grains
            const GrainDev g = a.g[idx[e0 + u < ng ? e0 + u : ng - 1]];   // block-uniform: scalar loads
            wv[u] = e0 + u < ng && g.t_first < tw + 64 && g.t_end > tw;   // wave-uniform
            act[u] = wv[u] && t >= g.t_first && t < g.t_end;
            disp[u] = 0.0;
            v0[u] = v1[u] = 0.0;
            ticks[u] = 0u;
            if (!wv[u]) continue;
            // inactive lanes use ticks 0: their (discarded) cos stays on the short argument path
            ticks[u] = act[u] ? g.ticks0 + (unsigned)(t - g.t_first) : 0u;
            const double position = g.offsets + (1 - g.speeds) * ticks[u];
            // buffer.h:40-47 with its unsigned wrap; the second tap reads center + 1
            const int center = (int)position;
            disp[u] = position - center;
            long tau0, tau1;
            if (center >= 0 && (unsigned)center < size) {   // no uint32 wrap: x0 in [1, 2 size)
                tau0 = t - center;
                tau1 = (unsigned)center + 1u < size ? tau0 - 1 : t;
            } else {
                const unsigned x0 = origin - (unsigned)center + size;
                const unsigned s0 = fastmod(x0, a.fm, size);
                // x1 = x0 - 1 (mod 2^32), so x1 % size follows from s0 unless x0 wrapped to 0
                const unsigned s1 = x0 == 0u ? a.wrap1 : (s0 == 0u ? size - 1u : s0 - 1u);
                tau0 = t - (long)(origin >= s0 ? origin - s0 : origin + size - s0);
                tau1 = t - (long)(origin >= s1 ? origin - s1 : origin + size - s1);
            }
            v0[u] = a.ring[tau0 & a.mask];
            v1[u] = a.ring[tau1 & a.mask];
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {   // phase 2: weights, in voice order
            if (!wv[u]) continue;
            const GrainDev& g = a.g[idx[e0 + u < ng ? e0 + u : ng - 1]];
            const double src = v0[u] * (1 - disp[u]) + v1[u] * disp[u];
            const double tk = (double)ticks[u];
            double phase;
            if (g.rsizes != 0.0) {   // tk / sizes: reciprocal product + one residual step (within an ulp)
                const double q0 = tk * g.rsizes;
                phase = __builtin_fma(__builtin_fma(-q0, g.sizes, tk), g.rsizes, q0);
            } else {
                phase = tk / g.sizes;
            }
            const double arg = 2 * hz::kPI * phase;
            const double cv = hz_rt::hann_cos(arg, a.fastcos != 0);
            const double term = g.gains * src * (0.5 * (1 - cv));   // wave.h:148
            if (act[u]) out += term;
        }
    }
    a.out[j] = out;
}

}  // namespace

struct hz_gran {
    long uid = 0;                     // unique per handle (the per-sample server's grain-cache key)
    unsigned polyphony = 0, size = 0;
    int device = 0;
    long T = 0;                       // samples processed
    std::vector<long> busy_until;     // per voice: t_end of its latest grain
    std::vector<long> tree;           // min-segment tree over busy_until (first free voice in O(log P))
    unsigned leaves = 1;
    std::vector<std::deque<GrainDev>> vg;   // per voice, its grains that may still read, in time order
    long mask = 0;
    double* d_ring = nullptr;
    GrainDev* d_g = nullptr;          // the call's grains + tile lists (bytes)
    size_t g_cap = 0;
    GrainDev* h_g = nullptr;          // pinned staging of the same (bytes)
    size_t hg_cap = 0;
    hipEvent_t up_ev = nullptr;
    bool up_pending = false;
    double *d_in = nullptr, *d_out = nullptr;
    size_t io_cap = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool prof = false;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    long launches = 0, grain_samples = 0;
    bool pending = false;             // block work queued on the stream since the last synchronisation
    // per-sample calls (hz_gran_sample): the grains that may still read, in voice order, in pinned
    // memory for the server (which caches them by version)
    GrainDev* h_list = nullptr;
    size_t list_cap = 0;
    int list_count = 0;
    long list_version = 0, list_min_end = 0;
    bool list_dirty = true;
};

namespace {

int gran_check(hz_gran* h) {
    if (!h) {
        hz::set_error("null hz_gran handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    return HZ_OK;
}

// granulator.h:51-79 made at the position "after the read of sample t"; ticks0 = 1 when
// the tick of t follows the request.  Returns the voice or -1.
int gran_alloc(hz_gran* h, long t, unsigned ticks0, double offset, double size, double speed, double gain) {
    if (size == 0) return -1;
    const double lo = size * (speed - 1);
    offset = (offset < lo) ? lo : offset;   // std::max(offset, size * (speed - 1))
    // first voice whose last read was at or before t (granulator.h:58-63's first inactive voice)
    if (h->polyphony == 0 || h->tree[1] > t + 1) return -1;
    unsigned node = 1;
    while (node < h->leaves) node = h->tree[2 * node] <= t + 1 ? 2 * node : 2 * node + 1;
    const int voice = (int)(node - h->leaves);
    GrainDev g{};
    g.offsets = hz::kSR * offset;
    g.sizes = hz::kSR * size;
    g.speeds = speed;
    g.gains = gain;
    g.ticks0 = ticks0;
    {   // RN(1/sizes) when the reciprocal and the quotients stay normal; else the device divides
        const double r = 1.0 / g.sizes;
        g.rsizes = (std::isnormal(r) && std::fabs(g.sizes) < 0x1p+900 && std::fabs(g.sizes) > 0x1p-900) ? r : 0.0;
    }
    g.t_first = t + 1;
    // last read: the first ticks >= ticks0 with (double)ticks >= sizes
    long m;
    if (std::isnan(g.sizes) || g.sizes >= 4294967295.0) m = kNever;   // never (or past the uint ticks range)
    else if (!(g.sizes > (double)ticks0)) m = 1;
    else m = (long)std::ceil(g.sizes) - ticks0 + 1;
    g.t_end = m >= kNever - g.t_first ? kNever : g.t_first + m;
    h->busy_until[voice] = g.t_end;
    h->list_dirty = true;
    h->tree[node] = g.t_end;
    for (unsigned q = node >> 1; q >= 1; q >>= 1) h->tree[q] = std::min(h->tree[2 * q], h->tree[2 * q + 1]);
    h->vg[voice].push_back(g);
    return voice;
}

int ensure(double** p, size_t* cap, size_t n) {
    if (n <= *cap) return HZ_OK;
    if (*p) HZ_TRY_HIP(hipFree(*p));
    *p = nullptr;
    HZ_TRY_HIP(hipMalloc(p, n * sizeof(double)));
    *cap = n;
    return HZ_OK;
}

int gran_run(hz_gran* h, const double* d_in, double* d_out, long n, const hz_grain_req* reqs, int nreq, int* voices) {
    if (n <= 0 && nreq > 0) {
        hz::set_error("hz_gran_process: requests need n > 0 (use hz_gran_request between calls)");
        return HZ_E_INVALID;
    }
    if (n <= 0) return HZ_OK;
    for (int k = 0; k < nreq; ++k)
        if (reqs[k].at < 0 || reqs[k].at >= n || (k && reqs[k].at < reqs[k - 1].at)) {
            hz::set_error("hz_gran_process: request %d has at = %ld (need 0 <= at < n, ascending)", k, reqs[k].at);
            return HZ_E_INVALID;
        }
    // drop finished grains, then apply the call's requests in order (closed-form lifetimes)
    for (auto& q : h->vg)
        while (!q.empty() && q.front().t_end <= h->T) q.pop_front();
    for (int k = 0; k < nreq; ++k) {
        const hz_grain_req& r = reqs[k];
        const int v = gran_alloc(h, h->T + r.at, 1u, r.offset, r.size, r.speed, r.gain);
        if (voices) voices[k] = v;
    }
    // the call's grains (voice-major) and per-tile lists in voice order (CSR), staged in
    // one pinned buffer and uploaded once
    const long nchunks = (n + kChunk - 1) / kChunk, ntiles = (n + kTile - 1) / kTile;
    std::vector<GrainDev> recs;
    std::vector<int> cnt(ntiles + 1, 0);
    for (const auto& q : h->vg)   // voice order (the reference's summation order)
        for (const GrainDev& g : q) {
            if (g.t_first >= h->T + n) break;   // a voice's grains are in time order
            if (g.t_end <= h->T) continue;
            recs.push_back(g);
            const long k0 = std::max(0L, (g.t_first - h->T) / kTile);
            const long k1 = std::min(ntiles, (g.t_end - 1 - h->T) / kTile + 1);
            for (long k = k0; k < k1; ++k) ++cnt[k + 1];
        }
    for (long k = 0; k < ntiles; ++k) cnt[k + 1] += cnt[k];
    std::vector<int> idx(cnt[ntiles]);
    {
        std::vector<int> fill(cnt.begin(), cnt.end() - 1);
        for (size_t r = 0; r < recs.size(); ++r) {
            const long k0 = std::max(0L, (recs[r].t_first - h->T) / kTile);
            const long k1 = std::min(ntiles, (recs[r].t_end - 1 - h->T) / kTile + 1);
            for (long k = k0; k < k1; ++k) idx[fill[k]++] = (int)r;
        }
    }
    const size_t b_rec = recs.size() * sizeof(GrainDev), b_off = cnt.size() * sizeof(int);
    const size_t bytes = b_rec + b_off + idx.size() * sizeof(int);
    if (h->up_pending) HZ_TRY_HIP(hipEventSynchronize(h->up_ev));   // staging buffer reuse
    if (bytes > h->hg_cap) {
        if (h->h_g) HZ_TRY_HIP(hipHostFree(h->h_g));
        h->h_g = nullptr;
        const size_t cap = std::max<size_t>(bytes, 2 * h->hg_cap);
        HZ_TRY_HIP(hipHostMalloc((void**)&h->h_g, cap));
        h->hg_cap = cap;
    }
    if (bytes > h->g_cap) {
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        if (h->d_g) HZ_TRY_HIP(hipFree(h->d_g));
        h->d_g = nullptr;
        const size_t cap = std::max<size_t>(bytes, 2 * h->g_cap);
        HZ_TRY_HIP(hipMalloc((void**)&h->d_g, cap));
        h->g_cap = cap;
    }
    char* hs = (char*)h->h_g;
    std::memcpy(hs, recs.data(), b_rec);
    std::memcpy(hs + b_rec, cnt.data(), b_off);
    std::memcpy(hs + b_rec + b_off, idx.data(), idx.size() * sizeof(int));
    HZ_TRY_HIP(hipMemcpyAsync(h->d_g, hs, bytes, hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipEventRecord(h->up_ev, h->stream));
    h->up_pending = true;
    const char* ds = (const char*)h->d_g;
    for (long c = 0; c < nchunks; ++c) {
        const long T0 = h->T + c * kChunk, m = std::min(n - c * kChunk, kChunk);
        {   // the launch's input into the time-indexed ring (slots T0 .. T0 + m - 1 mod C)
            const long C = h->mask + 1, s0 = T0 & h->mask, first = std::min(m, C - s0);
            HZ_TRY_HIP(hipMemcpyAsync(h->d_ring + s0, d_in + c * kChunk, sizeof(double) * first,
                                      hipMemcpyDeviceToDevice, h->stream));
            if (m > first)
                HZ_TRY_HIP(hipMemcpyAsync(h->d_ring, d_in + c * kChunk + first, sizeof(double) * (m - first),
                                          hipMemcpyDeviceToDevice, h->stream));
        }
        GranArgs a;
        a.out = d_out + c * kChunk;
        a.ring = h->d_ring;
        a.g = (const GrainDev*)ds;
        a.tile_off = (const int*)(ds + b_rec);
        a.tile_idx = (const int*)(ds + b_rec + b_off);
        a.tile_base = c * kChunk / kTile;
        a.T0 = T0;
        a.n = m;
        a.mask = h->mask;
        a.size = h->size;
        a.o0 = (unsigned)(T0 % (long)h->size);
        a.fm = h->size == 1u ? 0ul : ~0ul / h->size + 1ul;
        a.wrap1 = 0xffffffffu % h->size;
        static const bool libcos = std::getenv("HZ_GRAN_LIBCOS") != nullptr;
        a.fastcos = libcos ? 0 : 1;
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
        hipLaunchKernelGGL(gran_kernel, dim3((unsigned)((m + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                           h->stream, a);
        HZ_TRY_HIP(hipGetLastError());
        if (e) {
            HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
            ++h->launches;
            for (const GrainDev& g : recs)   // grain-samples of this launch
                h->grain_samples += std::max(0L, std::min(g.t_end, T0 + m) - std::max(g.t_first, T0));
        }
    }
    h->T += n;
    h->pending = true;
    h->list_dirty = true;
    return HZ_OK;
}

}  // namespace

extern "C" {

int hz_gran_create(unsigned polyphony, unsigned buffer_size, int device, hz_gran** out) {
    if (!out || buffer_size > (1u << 30)) {
        hz::set_error("hz_gran_create: invalid arguments (buffer_size <= 2^30)");
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_gran* h = new (std::nothrow) hz_gran();
    if (!h) return HZ_E_ALLOC;
    static std::atomic<long> next_uid{1};
    h->uid = next_uid++;
    h->polyphony = polyphony;
    h->size = buffer_size + (buffer_size == 0 ? 1u : 0u);   // buffer.h:21 (size zero disallowed)
    h->device = device;
    h->busy_until.assign(polyphony, 0);
    while (h->leaves < polyphony) h->leaves <<= 1;
    h->tree.assign(2 * (size_t)h->leaves, std::numeric_limits<long>::max());   // padding leaves never free
    for (unsigned v = 0; v < polyphony; ++v) h->tree[h->leaves + v] = 0;
    for (unsigned q = h->leaves - 1; q >= 1; --q) h->tree[q] = std::min(h->tree[2 * q], h->tree[2 * q + 1]);
    h->vg.resize(polyphony);
    long C = 1;
    while (C < (long)h->size + kChunk) C <<= 1;
    h->mask = C - 1;
    bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&h->up_ev, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipMalloc(&h->d_ring, sizeof(double) * C) == hipSuccess;
    ok = ok && hipMemset(h->d_ring, 0, sizeof(double) * C) == hipSuccess;   // Buffer: zeroed
    if (!ok) {
        hz::set_error("hz_gran_create: device allocation failed");
        if (h->up_ev) (void)hipEventDestroy(h->up_ev);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        if (h->d_ring) (void)hipFree(h->d_ring);
        delete h;
        return HZ_E_ALLOC;
    }
    h->own_stream = true;
    *out = h;
    return HZ_OK;
}

int hz_gran_destroy(hz_gran* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->d_ring, (void*)h->d_g, (void*)h->d_in, (void*)h->d_out})
        if (p) (void)hipFree(p);
    if (h->h_g) (void)hipHostFree(h->h_g);
    if (h->h_list) (void)hipHostFree(h->h_list);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->up_ev) (void)hipEventDestroy(h->up_ev);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_gran_request(hz_gran* h, double offset, double size, double speed, double gain, double pan, int ticked,
                    int* voice) {
    if (!h) return HZ_E_INVALID;
    (void)pan;   // stored but unused by the reference (granulator.h:71)
    // position: after the read of sample T-1; its tick follows unless `ticked` is 0
    const int v = gran_alloc(h, h->T - 1, ticked ? 1u : 0u, offset, size, speed, gain);
    if (voice) *voice = v;
    return HZ_OK;
}

int hz_gran_process_device(hz_gran* h, const double* d_in, double* d_out, size_t n, const hz_grain_req* reqs,
                           int nreq, int* voices) {
    HZ_TRY(gran_check(h));
    if ((n && (!d_in || !d_out)) || nreq < 0 || (nreq && !reqs)) return HZ_E_INVALID;
    return gran_run(h, d_in, d_out, (long)n, reqs, nreq, voices);
}

int hz_gran_process(hz_gran* h, const double* in, double* out, size_t n, const hz_grain_req* reqs, int nreq,
                    int* voices) {
    HZ_TRY(gran_check(h));
    if ((n && (!in || !out)) || nreq < 0 || (nreq && !reqs)) return HZ_E_INVALID;
    if (n == 0) return gran_run(h, nullptr, nullptr, 0, reqs, nreq, voices);
    size_t cap_in = h->io_cap, cap_out = h->io_cap;
    HZ_TRY(ensure(&h->d_in, &cap_in, n));
    HZ_TRY(ensure(&h->d_out, &cap_out, n));
    h->io_cap = std::min(cap_in, cap_out);
    HZ_TRY_HIP(hipMemcpyAsync(h->d_in, in, n * sizeof(double), hipMemcpyHostToDevice, h->stream));
    HZ_TRY(gran_run(h, h->d_in, h->d_out, (long)n, reqs, nreq, voices));
    HZ_TRY_HIP(hipMemcpyAsync(out, h->d_out, n * sizeof(double), hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

// one sample through the device's per-sample server (hz_rt.hip OP_GRAN): the reference's
// `source.write(x); y = granny(); granny.tick();` (tests/granny.cpp:36-56) without a launch per sample
int hz_gran_sample(hz_gran* h, double x, double* y) {
    HZ_TRY(gran_check(h));
    if (!y) return HZ_E_INVALID;
    if (h->pending) {   // the ring's block-call writes land before the server reads it
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        h->pending = false;
    }
    for (auto& q : h->vg)
        while (!q.empty() && q.front().t_end <= h->T) q.pop_front();
    if (h->list_dirty || h->list_min_end <= h->T) {   // grains started or ended: a new list version
        size_t cnt = 0;
        for (const auto& q : h->vg) cnt += q.size();
        // the server caches the grain list in LDS (kMaxGrains); a denser texture takes the
        // one-sample block call, which has no such cap (the list stays dirty until it fits)
        if (cnt > (size_t)hz_rt::kMaxGrains) return hz_gran_process(h, &x, y, 1, nullptr, 0, nullptr);
        if (cnt > h->list_cap || !h->h_list) {
            if (h->h_list) HZ_TRY_HIP(hipHostFree(h->h_list));
            h->h_list = nullptr;
            h->list_cap = std::max<size_t>(cnt, 64);
            HZ_TRY_HIP(hipHostMalloc((void**)&h->h_list, sizeof(GrainDev) * h->list_cap,
                                     hipHostMallocCoherent | hipHostMallocMapped));
        }
        long mn = kNever;
        int k = 0;
        for (const auto& q : h->vg)   // voice order (the reference's summation order)
            for (const GrainDev& g : q) {
                h->h_list[k++] = g;
                mn = std::min(mn, g.t_end);
            }
        h->list_count = k;
        h->list_min_end = mn;
        ++h->list_version;
        h->list_dirty = false;
    }
    hz_rt::Server* srv = hz_rt::server(h->device);
    if (!srv) return HZ_E_NODEV;
    hz_rt::GranArgs a{};
    a.ring = h->d_ring;
    a.grains = (const hz_rt::Grain*)hz_rt::dev(srv, h->h_list);
    a.mask = h->mask;
    a.t = h->T;
    a.key = h->uid;
    a.version = h->list_version;
    a.x = x;
    a.fm = h->size == 1u ? 0ul : ~0ul / h->size + 1ul;
    a.count = h->list_count;
    a.size = h->size;
    a.origin = (unsigned)(h->T % (long)h->size);
    a.wrap1 = 0xffffffffu % h->size;
    HZ_TRY(hz_rt::call(srv, hz_rt::OP_GRAN, &a, sizeof(a), 1, y));
    h->T += 1;
    return HZ_OK;
}

int hz_gran_activity(hz_gran* h, unsigned* activity) {
    if (!h || !activity) return HZ_E_INVALID;
    unsigned a = 0;
    for (long b : h->busy_until) a += b > h->T ? 1u : 0u;   // last read at or after T
    *activity = a;
    return HZ_OK;
}

int hz_gran_set_stream(hz_gran* h, void* stream) {
    HZ_TRY(gran_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) HZ_TRY_HIP(hipStreamDestroy(h->stream));
    h->stream = (hipStream_t)stream;
    h->own_stream = false;
    return HZ_OK;
}

int hz_gran_synchronize(hz_gran* h) {
    HZ_TRY(gran_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_gran_profile(hz_gran* h, int enable) {
    HZ_TRY(gran_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    h->prof = enable != 0;
    h->ev_used = 0;
    h->launches = 0;
    h->grain_samples = 0;
    return HZ_OK;
}

int hz_gran_profile_read(hz_gran* h, double* ms, long* launches, long* grain_samples) {
    HZ_TRY(gran_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    double tot = 0.0;
    for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
        float t = 0.f;
        HZ_TRY_HIP(hipEventElapsedTime(&t, h->ev[i], h->ev[i + 1]));
        tot += t;
    }
    if (ms) *ms = tot;
    if (launches) *launches = h->launches;
    if (grain_samples) *grain_samples = h->grain_samples;
    h->ev_used = 0;
    h->launches = 0;
    h->grain_samples = 0;
    return HZ_OK;
}

}  // extern "C"
