// hz_fb_rt.hip -- the per-sample ("real-time") Filterbank<double> path.
//
// The reference's operator API is per sample: `y = F(x); F.tick();` inside a PortAudio callback
// (src/filterbank.h:125-148, tests/resynthesis.cpp:35-39), and callers may feed y back into the
// next x (tests/spectral.cpp:94-104), so a sample cannot wait for a block.  A kernel launch plus
// two copies per sample costs tens of microseconds; at 48 kHz a sample has 20.8 us.
//
// Per-sample calls go to the device's per-sample server (hz_rt.hip: one resident kernel serving
// every handle through a pinned-host mailbox) as OP_FB requests over the handle's state in device
// memory.  Entering per-sample mode converts the block engines' state into ring rows in ring
// order, R[0..O-1] = y[t-1 .. t-O] and R[O] = the row at `origin` (filterbank.h:52, duplicated
// there; rotated here so a tick is a rotation):
//   compute(x)  (filterbank.h:170-187, the restatement's operation order, no FMA contraction):
//               pre, gain smoothed; y = pre (F0 x + sum_i F_i x[t-i]) - sum_k B_k R[k]; R[O] = y
//   tick()      (filterbank.h:142-148) origin - 1: R rotates right by one (R[0] <- R[O]) -- the
//               same for a tick after a compute and a bare tick (the stale row O+1 samples back
//               becomes the newest history row), so bare ticks are exact
//   mixdown     sum_n dist(R[O][n] g[n]) (filterbank.h:130, 138)
// The input ring is mirrored on the host and sent with each request.  Any block call, get/set_state
// or tick-rotation converts back (the rows and the spare row into ystate / xhist).
//
// Setters while samples run (the reference's MIDI thread, tests/filterbank.cpp:217-252 against
// the audio thread's 200-210): every entry point takes the handle's lock; a boost / mix / open or a
// coefficients() call reaches the next sample's request as a payload the server copies into the
// device arrays (no conversion, no restart), so it applies from the next operator() on -- the
// documented application point.
#include <algorithm>
#include <chrono>
#include <memory>
#include <mutex>
#include <cstring>
#include <thread>

#include "hz_fb_impl.h"
#include "hz_rt.h"

namespace {

// R[b][k] = ystate[b][k] (k < O), R[b][O] = the spare row (ystate_other[b][O-1]) or 0
__global__ __launch_bounds__(256) void fb_rt_enter_kernel(const double* __restrict__ ys, const double* __restrict__ yo,
                                                          double* __restrict__ R, int N, int O, int spare) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= N) return;
    for (int k = 0; k < O; ++k) R[(long)b * (O + 1) + k] = ys[(long)b * O + k];
    R[(long)b * (O + 1) + O] = (O > 0 && spare) ? yo[(long)b * O + O - 1] : 0.0;
}

__global__ __launch_bounds__(256) void fb_rt_leave_kernel(const double* __restrict__ R, double* __restrict__ ys,
                                                          double* __restrict__ yo, int N, int O) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= N || O == 0) return;
    for (int k = 0; k < O; ++k) ys[(long)b * O + k] = R[(long)b * (O + 1) + k];
    yo[(long)b * O + O - 1] = R[(long)b * (O + 1) + O];
}

int groups_for(int N) { return std::max(1, std::min(hz_rt::kGroups, (N + hz_rt::kThreads - 1) / hz_rt::kThreads)); }

}  // namespace

namespace hz_fbi {

bool fb_rt_supported(const hz_fb*) { return true; }   // the server loops over any number of bands

// sparse reloads: at most this many triples (beyond it both arrays are cheaper to send)
static size_t sparse_cap(int N) { return std::max<size_t>(16, (size_t)N / 8); }

static void sparse_clear(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    for (int l : T.dirty) T.mark[l] = 0;
    T.dirty.clear();
    T.sp_base = T.sp_gen = h->pg_gen;
}

void fb_rt_target_setter(hz_fb* h, int l) {
    hz_fb::Rt& T = h->rt;
    const bool track = l != kAllBands && T.sp_gen == h->pg_gen;
    ++h->pg_gen;
    if (!track) return;
    if (l >= 0 && !T.mark[l]) {
        if (T.dirty.size() >= sparse_cap(h->N)) return;   // the list stops covering: both arrays
        T.mark[l] = 1;
        T.dirty.push_back(l);
    }
    T.sp_gen = h->pg_gen;
}

// the state into ring rows, the coefficients into the op's layout, the input ring to the host
static int rt_enter(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    const int O = h->order, N = h->N;
    HZ_TRY(fb_upload_staged(h));
    HZ_TRY(fb_resp_materialize(h));
    const size_t nc = (size_t)N * (2 * O + 1), nr = (size_t)N * (O + 1);
    if (nc + nr > T.coef_cap) {
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        if (T.d_coef) HZ_TRY_HIP(hipFree(T.d_coef));
        T.d_coef = nullptr;
        HZ_TRY_HIP(hipMalloc(&T.d_coef, sizeof(double) * (nc + nr)));
        T.coef_cap = nc + nr;
    }
    if (!T.pin1) HZ_TRY_HIP(hipHostMalloc((void**)&T.pin1, sizeof(double) * 16));
    T.h_coef.resize(nc);
    for (int n = 0; n < N; ++n) {
        for (int i = 0; i <= O; ++i) T.h_coef[(size_t)n * (2 * O + 1) + i] = h->F[(size_t)n * (O + 1) + i];
        for (int k = 0; k < O; ++k) T.h_coef[(size_t)n * (2 * O + 1) + O + 1 + k] = h->B[(size_t)n * O + k];
    }
    HZ_TRY_HIP(hipMemcpyAsync(T.d_coef, T.h_coef.data(), sizeof(double) * nc, hipMemcpyHostToDevice, h->stream));
    const int spare = h->spare_ok ? 1 : 0;
    hipLaunchKernelGGL(fb_rt_enter_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, h->stream,
                       (const double*)h->d_ystate[h->scur], (const double*)h->d_ystate[h->scur ^ 1], T.d_coef + nc, N,
                       O, spare);
    HZ_TRY_HIP(hipGetLastError());
    double xh[hz_fbi::kMaxOrder + 1] = {}, xo[hz_fbi::kMaxOrder + 1] = {};
    if (O > 0) {
        HZ_TRY_HIP(hipMemcpyAsync(T.pin1, h->d_xhist[h->xcur], sizeof(double) * O, hipMemcpyDeviceToHost, h->stream));
        HZ_TRY_HIP(hipMemcpyAsync(T.pin1 + 8, h->d_xhist[h->xcur ^ 1], sizeof(double) * O, hipMemcpyDeviceToHost,
                                  h->stream));
    }
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // pageable sources; block work drained before the server
    for (int k = 0; k < O; ++k) {
        xh[k] = T.pin1[k];
        xo[k] = T.pin1[8 + k];
    }
    for (int k = 0; k < O; ++k) T.xr[k] = xh[k];
    T.xr[O] = (O > 0 && spare) ? xo[O - 1] : 0.0;
    T.pg_gen = h->pg_gen;
    T.coef_gen = h->coef_gen;
    sparse_clear(h);
    T.active = true;
    T.spare_known = h->spare_ok;
    // per-sample calls own the state from here; the stationary history no longer follows it
    h->resp.run = 0;
    fb_stream_reset(h);
    return HZ_OK;
}

// back to the block engines' layout (stream-ordered on the handle's stream)
int fb_rt_stop(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    if (T.active) {
        const int O = h->order, N = h->N;
        const size_t nc = (size_t)N * (2 * O + 1);
        hipLaunchKernelGGL(fb_rt_leave_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, h->stream,
                           (const double*)(T.d_coef + nc), h->d_ystate[h->scur], h->d_ystate[h->scur ^ 1], N, O);
        HZ_TRY_HIP(hipGetLastError());
        if (O > 0) {
            for (int k = 0; k < O; ++k) T.pin1[k] = T.xr[k];
            T.pin1[8] = T.xr[O];
            HZ_TRY_HIP(hipMemcpyAsync(h->d_xhist[h->xcur], T.pin1, sizeof(double) * O, hipMemcpyHostToDevice, h->stream));
            HZ_TRY_HIP(hipMemcpyAsync(h->d_xhist[h->xcur ^ 1] + (O - 1), T.pin1 + 8, sizeof(double), hipMemcpyHostToDevice,
                                      h->stream));
            HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // the pinned staging is reused
        }
        T.active = false;
        h->spare_ok = T.spare_known;
    }
    // ticks since the last served sample: the block engines' ring rotation
    const int O = h->order;
    const long rot = O > 0 ? T.pending_ticks % (O + 1) : 0;
    T.pending_ticks = 0;
    for (long i = 0; i < rot; ++i) HZ_TRY(fb_tick_rotate(h));
    return HZ_OK;
}

static int sample_locked(hz_fb* h, double x, int dist_id, double param, double* y);
static void tick_locked(hz_fb* h);

int fb_rt_resolve(hz_fb* h, double* y0) {
    if (!h->rt.computed) return 0;
    HZ_TRY(sample_locked(h, 0.0, h->dist_id, h->dist_param, y0));   // (the caller holds the handle)
    tick_locked(h);
    HZ_TRY(fb_rt_stop(h));
    return 1;
}

double* fb_rt_cached_slot(hz_fb* h) { return h->rt.pin1 + 15; }

void fb_rt_free(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    if (T.pin1) (void)hipHostFree(T.pin1);
    if (T.d_coef) (void)hipFree(T.d_coef);
    T.pin1 = nullptr;
    T.d_coef = nullptr;
    T.active = false;
}

// operator() with the handle held (the entry point below, or a block call resolving a cached sample)
static int sample_locked(hz_fb* h, double x, int dist_id, double param, double* y) {
    HZ_TRY_HIP(hipSetDevice(h->device));
    hz_fb::Rt& T = h->rt;
    const int O = h->order, N = h->N;
    const long ticks = O > 0 ? T.pending_ticks % (O + 1) : 0;
    const bool spare_known = T.active ? T.spare_known : h->spare_ok;   // the ring row a bare tick exposes
    if (!T.computed && ticks > 0 && !spare_known) {
        hz::set_error("hz_fb_sample: tick() without operator() after a block call or set_state: the ring row "
                      "it would reuse (O+1 samples back) is not kept");
        return HZ_E_STATE;
    }
    hz_rt::Server* srv = hz_rt::server(h->device);
    if (!srv) {
        hz::set_error("hz_fb_sample: no per-sample server on device %d", h->device);
        return HZ_E_NODEV;
    }
    if (T.many) {   // the rows were served by other workgroups (OP_FB_MANY): a fresh instance
        hz_rt::quiesce(srv);
        T.many = false;
    }
    if (!T.active || h->tv_pending) {
        if (T.active) {   // a coefficient stream call left a row staged: convert back and in again
            const long keep = T.pending_ticks;
            T.pending_ticks = 0;
            HZ_TRY(hz_fbi::fb_rt_stop(h));
            T.pending_ticks = keep;
        }
        HZ_TRY(hz_fbi::rt_enter(h));
    }
    hz_rt::FbArgs a{};
    const size_t nc = (size_t)N * (2 * O + 1);
    a.R = T.d_coef + nc;
    a.pg = h->d_pg[h->scur];
    a.coef = T.d_coef;
    a.pin = h->d_pin;
    a.gin = h->d_gin;
    a.reload = nullptr;
    a.reload_coef = nullptr;
    a.sparse = nullptr;
    a.nsparse = 0;
    std::lock_guard<std::recursive_mutex> slk(hz_rt::lock(srv));
    if (T.pg_gen != h->pg_gen || T.coef_gen != h->coef_gen) {
        // setters since the last sample: the new targets / coefficients ride in the payload and the
        // server writes them into the device arrays (block calls upload them again: dirty flags stay)
        const bool tg = T.pg_gen != h->pg_gen, cf = T.coef_gen != h->coef_gen;
        // one-band setters only (the list covers every change since the server's copy): triples
        const bool sparse = tg && T.sp_base == T.pg_gen && T.sp_gen == h->pg_gen;
        const size_t nt = !tg ? 0 : sparse ? 3 * T.dirty.size() : 2 * (size_t)N;
        double* p = hz_rt::payload(srv, std::max<size_t>(1, nt + (cf ? nc : 0)));
        if (!p) return HZ_E_ALLOC;
        const size_t at = nt;
        if (sparse) {
            for (size_t j = 0; j < T.dirty.size(); ++j) {
                const int l = T.dirty[j];
                p[3 * j] = (double)l;
                p[3 * j + 1] = h->pin[l];
                p[3 * j + 2] = h->gin[l];
            }
            a.sparse = (const double*)hz_rt::dev(srv, p);
            a.nsparse = (int)T.dirty.size();
        } else if (tg) {
            std::memcpy(p, h->pin.data(), sizeof(double) * N);
            std::memcpy(p + N, h->gin.data(), sizeof(double) * N);
            a.reload = (const double*)hz_rt::dev(srv, p);
        }
        if (tg) hz_fbi::sparse_clear(h);
        if (cf) {
            HZ_TRY(hz_fbi::fb_tv_materialize(h));
            for (int n = 0; n < N; ++n) {
                double* r = p + at + (size_t)n * (2 * O + 1);
                for (int i = 0; i <= O; ++i) r[i] = h->F[(size_t)n * (O + 1) + i];
                for (int k = 0; k < O; ++k) r[O + 1 + k] = h->B[(size_t)n * O + k];
            }
            a.reload_coef = (const double*)hz_rt::dev(srv, p + at);
        }
        T.pg_gen = h->pg_gen;
        T.coef_gen = h->coef_gen;
    }
    // the input ring after the bare ticks (ring order; rotated right per tick)
    for (long q = 0; q < ticks; ++q) {
        const double t0 = T.xr[O];
        for (int k = O; k >= 1; --k) T.xr[k] = T.xr[k - 1];
        T.xr[0] = t0;
    }
    const bool compute = !T.computed;
    a.x = x;
    a.param = param;
    a.sp = h->sp;
    a.sg = h->sg;
    for (int k = 0; k <= O; ++k) a.xr[k] = T.xr[k];
    a.N = N;
    a.O = O;
    a.ticks = (int)ticks;
    a.compute = compute ? 1 : 0;
    a.dist = dist_id;
    double s = 0.0;
    HZ_TRY(hz_rt::call(srv, hz_rt::OP_FB, &a, sizeof(a), groups_for(N), &s));
    if (compute) T.xr[O] = x;
    *y = s;
    T.pending_ticks = 0;
    if (compute) {
        T.computed = true;
        T.spare_known = true;   // the row at origin now holds this sample's outputs
        T.cached = s;
        hz_fbi::fb_mirror_advance(h, 1);
    }
    T.cached_dist = dist_id;
    ++T.seq;
    return HZ_OK;
}

static void tick_locked(hz_fb* h) {
    ++h->rt.pending_ticks;
    h->rt.computed = false;
}

// ---- several handles per request (OP_FB_MANY) ------------------------------------------------
// The chunk table of the last group served on each device (rebuilt when a member's arrays move)
struct ManyCache {
    std::vector<hz_fb*> hs;
    std::vector<hz_rt::ManyChunk> chunks;
    hz_rt::ManyChunk* d = nullptr;
    size_t cap = 0;
};
static ManyCache g_many[64];
static std::mutex g_many_mu;

// *changed: the table differs from the last group's -- a member's chunks move to other workgroups
// (the chunk -> workgroup map follows the group's order and size), so the caller quiesces the server
static int many_table(int device, hz_fb* const* hs, int H, int* nchunks, const hz_rt::ManyChunk** d, bool* changed) {
    std::vector<hz_rt::ManyChunk> ch;
    for (int m = 0; m < H; ++m) {
        hz_fb* h = hs[m];
        const int O = h->order, N = h->N;
        const size_t nc = (size_t)N * (2 * O + 1);
        double* R = h->rt.d_coef + nc;
        for (int b0 = 0; b0 < N; b0 += 64) {
            hz_rt::ManyChunk c{};
            c.R = R + (size_t)b0 * (O + 1);
            c.pg = h->d_pg[h->scur] + 2 * (size_t)b0;
            c.coef = h->rt.d_coef + (size_t)b0 * (2 * O + 1);
            c.pin = h->d_pin + b0;
            c.gin = h->d_gin + b0;
            c.n = std::min(64, N - b0);
            c.m = m;
            c.sp = h->sp;
            c.sg = h->sg;
            ch.push_back(c);
        }
    }
    ManyCache& C = g_many[device];
    const bool same = C.hs.size() == (size_t)H && std::equal(C.hs.begin(), C.hs.end(), hs) &&
                      C.chunks.size() == ch.size() &&
                      std::memcmp(C.chunks.data(), ch.data(), sizeof(hz_rt::ManyChunk) * ch.size()) == 0;
    if (!same) {
        if (ch.size() > C.cap) {
            if (C.d) HZ_TRY_HIP(hipFree(C.d));
            C.d = nullptr;
            HZ_TRY_HIP(hipMalloc(&C.d, sizeof(hz_rt::ManyChunk) * ch.size()));
            C.cap = ch.size();
        }
        HZ_TRY_HIP(hipMemcpy(C.d, ch.data(), sizeof(hz_rt::ManyChunk) * ch.size(), hipMemcpyHostToDevice));
        C.hs.assign(hs, hs + H);
        C.chunks = std::move(ch);
    }
    *nchunks = (int)C.chunks.size();
    *d = C.d;
    *changed = !same;
    return HZ_OK;
}

// setters staged on a member since the server's copy: with the server out, straight into the
// device arrays (targets, and the per-sample layout's coefficients)
static int many_apply_setters(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    if (T.pg_gen == h->pg_gen && T.coef_gen == h->coef_gen) return HZ_OK;
    const int O = h->order, N = h->N;
    if (T.pg_gen != h->pg_gen) {
        HZ_TRY_HIP(hipMemcpy(h->d_pin, h->pin.data(), sizeof(double) * N, hipMemcpyHostToDevice));
        HZ_TRY_HIP(hipMemcpy(h->d_gin, h->gin.data(), sizeof(double) * N, hipMemcpyHostToDevice));
        sparse_clear(h);
    }
    if (T.coef_gen != h->coef_gen) {
        HZ_TRY(fb_tv_materialize(h));
        const size_t nc = (size_t)N * (2 * O + 1);
        T.h_coef.resize(nc);
        for (int n = 0; n < N; ++n) {
            for (int i = 0; i <= O; ++i) T.h_coef[(size_t)n * (2 * O + 1) + i] = h->F[(size_t)n * (O + 1) + i];
            for (int k = 0; k < O; ++k) T.h_coef[(size_t)n * (2 * O + 1) + O + 1 + k] = h->B[(size_t)n * O + k];
        }
        HZ_TRY_HIP(hipMemcpy(T.d_coef, T.h_coef.data(), sizeof(double) * nc, hipMemcpyHostToDevice));
    }
    T.pg_gen = h->pg_gen;
    T.coef_gen = h->coef_gen;
    return HZ_OK;
}

static int sample_many_locked(hz_fb* const* hs, int H, const double* x, int dist_id, double param, double* y) {
    const int O = hs[0]->order, dev = hs[0]->device;
    HZ_TRY_HIP(hipSetDevice(dev));
    hz_rt::Server* srv = hz_rt::server(dev);
    if (!srv) {
        hz::set_error("hz_fb_sample_many: no per-sample server on device %d", dev);
        return HZ_E_NODEV;
    }
    std::lock_guard<std::recursive_mutex> slk(hz_rt::lock(srv));
    // members entering the per-sample layout, members last served one by one (other workgroups),
    // members with staged setters: all handled with the resident instance out
    bool fresh = false;
    for (int m = 0; m < H; ++m) {
        hz_fb::Rt& T = hs[m]->rt;
        const long ticks = O > 0 ? T.pending_ticks % (O + 1) : 0;
        const bool spare_known = T.active ? T.spare_known : hs[m]->spare_ok;
        if (!T.computed && ticks > 0 && !spare_known) {
            hz::set_error("hz_fb_sample_many: tick() without operator() after a block call or set_state (member %d)", m);
            return HZ_E_STATE;
        }
        if (!T.active || hs[m]->tv_pending || !T.many || T.pg_gen != hs[m]->pg_gen || T.coef_gen != hs[m]->coef_gen)
            fresh = true;
    }
    if (fresh) {
        hz_rt::quiesce(srv);
        for (int m = 0; m < H; ++m) {
            hz_fb* h = hs[m];
            hz_fb::Rt& T = h->rt;
            if (!T.active || h->tv_pending) {
                if (T.active) {
                    const long keep = T.pending_ticks;
                    T.pending_ticks = 0;
                    HZ_TRY(fb_rt_stop(h));
                    T.pending_ticks = keep;
                }
                HZ_TRY(rt_enter(h));
            }
            HZ_TRY(many_apply_setters(h));
            T.many = true;
        }
    }
    int nch = 0;
    const hz_rt::ManyChunk* d = nullptr;
    bool changed = false;
    {
        std::lock_guard<std::mutex> lk(g_many_mu);
        HZ_TRY(many_table(dev, hs, H, &nch, &d, &changed));
    }
    // another group (other members, order or size) than the last request's: its band rows were
    // served by other workgroups, possibly on another XCD -- a kernel boundary first
    if (changed && !fresh) hz_rt::quiesce(srv);
    const int groups = std::max(1, std::min(hz_rt::kGroups, (nch + hz_rt::kThreads / 64 - 1) / (hz_rt::kThreads / 64)));
    double* res = hz_rt::result(srv, (size_t)hz_rt::kGroups * hz_rt::kMaxMany);
    if (!res) return HZ_E_ALLOC;
    long long w[hz_rt::kArgWords] = {};
    hz_rt::ManyArgs* a = (hz_rt::ManyArgs*)w;
    a->chunks = d;
    a->out = (double*)hz_rt::dev(srv, res);
    a->param = param;
    a->H = H;
    a->nchunks = nch;
    a->O = O;
    a->dist = dist_id;
    a->meta = 0;
    double* xv = (double*)(w + hz_rt::kManyHeader);
    for (int m = 0; m < H; ++m) {
        hz_fb::Rt& T = hs[m]->rt;
        const long ticks = O > 0 ? T.pending_ticks % (O + 1) : 0;
        for (long q = 0; q < ticks; ++q) {   // the input ring after the bare ticks
            const double t0 = T.xr[O];
            for (int k = O; k >= 1; --k) T.xr[k] = T.xr[k - 1];
            T.xr[0] = t0;
        }
        const bool compute = !T.computed;
        a->meta |= (unsigned long long)(ticks | (compute ? 8 : 0)) << (4 * m);
        xv[m * (O + 2)] = x[m];
        for (int k = 0; k <= O; ++k) xv[m * (O + 2) + 1 + k] = T.xr[k];
    }
    const size_t bytes = sizeof(long long) * (hz_rt::kManyHeader + (size_t)H * (O + 2));
    HZ_TRY(hz_rt::call(srv, hz_rt::OP_FB_MANY, w, bytes, groups, nullptr));
    for (int m = 0; m < H; ++m) {
        double v = 0.0;
        for (int g = 0; g < groups; ++g) v += res[g * H + m];   // workgroups in order
        hz_fb* h = hs[m];
        hz_fb::Rt& T = h->rt;
        const bool compute = ((a->meta >> (4 * m)) & 8) != 0;
        if (compute) {
            T.xr[O] = x[m];
            T.computed = true;
            T.spare_known = true;
            T.cached = v;
            fb_mirror_advance(h, 1);
        }
        T.pending_ticks = 0;
        T.cached_dist = dist_id;
        ++T.seq;
        y[m] = v;
    }
    return HZ_OK;
}

}  // namespace hz_fbi

extern "C" {

int hz_fb_sample(hz_fb* h, double x, int dist_id, double param, double* y) {
    if (!h || !y || dist_id < HZ_DIST_NONE || dist_id > HZ_DIST_LIMITER) {
        hz::set_error("hz_fb_sample: invalid arguments");
        return HZ_E_INVALID;
    }
    hz_fbi::SampleLock lk(h);   // a setter from another thread goes first (this sample sees it)
    return hz_fbi::sample_locked(h, x, dist_id, param, y);
}

int hz_fb_sample_many(hz_fb* const* handles, int count, const double* x, int dist_id, double param, double* y) {
    if (!handles || !x || !y || count < 1 || count > hz_rt::kMaxMany || dist_id < HZ_DIST_NONE ||
        dist_id > HZ_DIST_LIMITER) {
        hz::set_error("hz_fb_sample_many: invalid arguments (1 <= count <= %d)", hz_rt::kMaxMany);
        return HZ_E_INVALID;
    }
    std::vector<hz_fb*> order(handles, handles + count);
    for (int m = 0; m < count; ++m) {
        if (!handles[m] || handles[m]->device != handles[0]->device || handles[m]->order != handles[0]->order) {
            hz::set_error("hz_fb_sample_many: the handles must share a device and an order");
            return HZ_E_INVALID;
        }
    }
    const int O = handles[0]->order;
    if (hz_rt::kManyHeader + count * (O + 2) > hz_rt::kArgWords) {
        hz::set_error("hz_fb_sample_many: at most %d handles of order %d per request",
                      (hz_rt::kArgWords - hz_rt::kManyHeader) / (O + 2), O);
        return HZ_E_INVALID;
    }
    std::sort(order.begin(), order.end());
    if (std::adjacent_find(order.begin(), order.end()) != order.end()) {
        hz::set_error("hz_fb_sample_many: a handle appears twice");
        return HZ_E_INVALID;
    }
    // every member held (in address order: no lock-order inversion between callers)
    std::vector<std::unique_ptr<hz_fbi::SampleLock>> locks;
    for (hz_fb* h : order) locks.emplace_back(new hz_fbi::SampleLock(h));
    return hz_fbi::sample_many_locked(handles, count, x, dist_id, param, y);
}

int hz_fb_sample_tick(hz_fb* h) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::SampleLock lk(h);
    hz_fbi::tick_locked(h);
    return HZ_OK;
}

int hz_fb_sample_info(hz_fb* h, int* active, long long* served, int* groups) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    if (active) *active = h->rt.active ? 1 : 0;
    if (served) *served = h->rt.seq;
    if (groups) *groups = groups_for(h->N);
    return HZ_OK;
}

}  // extern "C"
