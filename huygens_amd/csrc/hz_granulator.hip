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
// time-indexed ring of C >= size + kChunk samples (a power of two), so no sample a block
// still needs is overwritten by the same block: tau >= T0 comes from the block's input,
// older ones from the ring.  The uint32 index arithmetic is kept verbatim (bit-exact).
//
// Layout in HBM: ring [C] doubles; grains [G] x 64 B per block (uploaded once per call).
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <new>
#include <vector>

#include "hz_common.h"

namespace {

constexpr int kThreads = 256;
constexpr long kChunk = 1L << 18;             // samples per launch
constexpr long kNever = 1L << 62;             // t_end of a grain that never finishes (NaN/inf size)

struct alignas(16) GrainDev {
    long t_first, t_end;                      // reads at t_first <= t < t_end
    double offsets, sizes, speeds, gains;     // granulator.h:67-70 (samples, samples, ratio, gain)
    unsigned ticks0, pad0;
    long pad1;
};
static_assert(sizeof(GrainDev) == 64, "grain record is one 64 B line");

struct GranArgs {
    const double* in;     // block input: time T0 + j
    double* out;
    double* ring;         // time-indexed source ring (C = mask + 1 samples)
    const GrainDev* g;
    int ng;
    long T0, n, mask;
    unsigned size, o0;    // Buffer size and origin at time T0
};

// x(tau) for tau <= t: the block input, the ring, or 0 before the first write
__device__ __forceinline__ double src_at(const GranArgs& a, long tau) {
    if (tau < 0) return 0.0;
    if (tau >= a.T0) return a.in[tau - a.T0];
    return a.ring[tau & a.mask];
}

__global__ __launch_bounds__(kThreads) void gran_kernel(GranArgs a) {
#pragma clang fp contract(off)
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= a.n) return;
    const long t = a.T0 + j;
    const unsigned size = a.size;
    const unsigned origin = (unsigned)(((unsigned long)a.o0 + (unsigned long)j) % size);
    double out = 0;
    for (int e = 0; e < a.ng; ++e) {
        const GrainDev g = a.g[e];   // wave-uniform: scalar loads
        if (t < g.t_first || t >= g.t_end) continue;
        const unsigned ticks = g.ticks0 + (unsigned)(t - g.t_first);
        const double phase = (double)ticks / g.sizes;
        const double position = g.offsets + (1 - g.speeds) * ticks;
        // buffer.h:40-47 with its unsigned wrap
        const int center = (int)position;
        const int before = center + 1;
        const double disp = position - center;
        const unsigned s0 = (origin - (unsigned)center + size) % size;
        const unsigned s1 = (origin - (unsigned)before + size) % size;
        const double v0 = src_at(a, t - (long)(origin >= s0 ? origin - s0 : origin + size - s0));
        const double v1 = src_at(a, t - (long)(origin >= s1 ? origin - s1 : origin + size - s1));
        const double src = v0 * (1 - disp) + v1 * disp;
        out += g.gains * src * (0.5 * (1 - cos(2 * hz::kPI * phase)));   // wave.h:148
    }
    a.out[j] = out;
    a.ring[t & a.mask] = a.in[j];   // no thread of this block reads this slot (C >= size + kChunk)
}

}  // namespace

struct hz_gran {
    unsigned polyphony = 0, size = 0;
    int device = 0;
    long T = 0;                       // samples processed
    std::vector<long> busy_until;     // per voice: t_end of its latest grain
    std::vector<GrainDev> grains;     // grains that may still read (t_end > T)
    std::vector<int> grain_voice;     // voice of each grain (sort key)
    long mask = 0;
    double* d_ring = nullptr;
    GrainDev* d_g = nullptr;
    size_t g_cap = 0;
    GrainDev* h_g = nullptr;          // pinned staging of the call's grain lists
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
    int voice = -1;
    for (unsigned v = 0; v < h->polyphony; ++v)
        if (h->busy_until[v] <= t + 1) {   // its last read was at or before t
            voice = (int)v;
            break;
        }
    if (voice < 0) return -1;
    GrainDev g{};
    g.offsets = hz::kSR * offset;
    g.sizes = hz::kSR * size;
    g.speeds = speed;
    g.gains = gain;
    g.ticks0 = ticks0;
    g.t_first = t + 1;
    // last read: the first ticks >= ticks0 with (double)ticks >= sizes
    long m;
    if (std::isnan(g.sizes) || g.sizes >= 4294967295.0) m = kNever;   // never (or past the uint ticks range)
    else if (!(g.sizes > (double)ticks0)) m = 1;
    else m = (long)std::ceil(g.sizes) - ticks0 + 1;
    g.t_end = m >= kNever - g.t_first ? kNever : g.t_first + m;
    h->busy_until[voice] = g.t_end;
    h->grains.push_back(g);
    h->grain_voice.push_back(voice);
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
    {
        size_t w = 0;
        for (size_t i = 0; i < h->grains.size(); ++i)
            if (h->grains[i].t_end > h->T) {
                h->grains[w] = h->grains[i];
                h->grain_voice[w++] = h->grain_voice[i];
            }
        h->grains.resize(w);
        h->grain_voice.resize(w);
    }
    for (int k = 0; k < nreq; ++k) {
        const hz_grain_req& r = reqs[k];
        const int v = gran_alloc(h, h->T + r.at, 1u, r.offset, r.size, r.speed, r.gain);
        if (voices) voices[k] = v;
    }
    // voice order (the reference's summation order); a voice's grains never overlap in time
    std::vector<int> order(h->grains.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
    std::sort(order.begin(), order.end(), [&](int x, int y) {
        return h->grain_voice[x] != h->grain_voice[y] ? h->grain_voice[x] < h->grain_voice[y]
                                                      : h->grains[x].t_first < h->grains[y].t_first;
    });
    // per-launch grain lists, staged in one pinned buffer and uploaded once
    const long nchunks = (n + kChunk - 1) / kChunk;
    std::vector<size_t> off(nchunks + 1, 0);
    std::vector<GrainDev> all;
    for (long c = 0; c < nchunks; ++c) {
        const long T0 = h->T + c * kChunk, T1 = std::min(h->T + n, T0 + kChunk);
        for (int i : order) {
            const GrainDev& g = h->grains[i];
            if (g.t_first < T1 && g.t_end > T0) all.push_back(g);
        }
        off[c + 1] = all.size();
    }
    if (h->up_pending) HZ_TRY_HIP(hipEventSynchronize(h->up_ev));   // staging buffer reuse
    if (all.size() > h->hg_cap) {
        if (h->h_g) HZ_TRY_HIP(hipHostFree(h->h_g));
        h->h_g = nullptr;
        const size_t cap = std::max<size_t>(all.size(), 2 * h->hg_cap);
        HZ_TRY_HIP(hipHostMalloc((void**)&h->h_g, cap * sizeof(GrainDev)));
        h->hg_cap = cap;
    }
    if (all.size() > h->g_cap) {
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        if (h->d_g) HZ_TRY_HIP(hipFree(h->d_g));
        h->d_g = nullptr;
        const size_t cap = std::max<size_t>(all.size(), 2 * h->g_cap);
        HZ_TRY_HIP(hipMalloc(&h->d_g, cap * sizeof(GrainDev)));
        h->g_cap = cap;
    }
    if (!all.empty()) {
        std::memcpy(h->h_g, all.data(), all.size() * sizeof(GrainDev));
        HZ_TRY_HIP(hipMemcpyAsync(h->d_g, h->h_g, all.size() * sizeof(GrainDev), hipMemcpyHostToDevice, h->stream));
        HZ_TRY_HIP(hipEventRecord(h->up_ev, h->stream));
        h->up_pending = true;
    }
    for (long c = 0; c < nchunks; ++c) {
        const long T0 = h->T + c * kChunk, m = std::min(n - c * kChunk, kChunk);
        GranArgs a;
        a.in = d_in + c * kChunk;
        a.out = d_out + c * kChunk;
        a.ring = h->d_ring;
        a.g = h->d_g + off[c];
        a.ng = (int)(off[c + 1] - off[c]);
        a.T0 = T0;
        a.n = m;
        a.mask = h->mask;
        a.size = h->size;
        a.o0 = (unsigned)(T0 % (long)h->size);
        hipEvent_t* e = nullptr;
        if (h->prof) {
            if (h->ev_used + 2 > h->ev.size())
                for (int q = 0; q < 64; ++q) {
                    hipEvent_t ne;
                    HZ_TRY_HIP(hipEventCreate(&ne));
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
            for (size_t i = off[c]; i < off[c + 1]; ++i)   // grain-samples of this launch
                h->grain_samples += std::min(all[i].t_end, T0 + m) - std::max(all[i].t_first, T0);
        }
    }
    h->T += n;
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
    h->polyphony = polyphony;
    h->size = buffer_size + (buffer_size == 0 ? 1u : 0u);   // buffer.h:21 (size zero disallowed)
    h->device = device;
    h->busy_until.assign(polyphony, 0);
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
