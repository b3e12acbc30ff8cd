// hz_fb_rt.hip -- the per-sample ("real-time") Filterbank<double> engine.
//
// The reference's operator API is per sample: `y = F(x); F.tick();` inside a PortAudio callback
// (src/filterbank.h:125-148, tests/resynthesis.cpp:35-39), and callers may feed y back into the
// next x (tests/spectral.cpp:94-104), so a sample cannot wait for a block.  A kernel launch plus
// two copies per sample costs tens of microseconds; at 48 kHz a sample has 20.8 us.
//
// Instead one kernel stays resident on the handle's stream while per-sample calls continue and
// serves them through a mailbox in fine-grained pinned host memory (hipHostMallocCoherent):
//   host:   x, dist, ticks, op -> request line, then the request number (release store)
//   device: workgroup 0 polls the request number (system-scope acquire loads), forwards it to the
//           other workgroups through device memory, every workgroup runs its bands and writes its
//           partial mix and the request number to its own 64-byte response line (system scope)
//   host:   spins on the response lines, sums the partial mixes in workgroup order.
// Measured round trip of the transport on MI355X: 3.8 us (scripts/probe/mailbox_probe.hip).
//
// Band state lives in registers for the kernel's lifetime: per band the O+1 rows of the
// reference's output ring (filterbank.h:52, duplicated there; here rotated instead of indexed so
// every register index is static), the pre-amp and gain smoothers and the coefficients; the input
// ring is wave-uniform.  In ring order R[0..O-1] = y[t-1 .. t-O] and R[O] = the row at `origin`:
//   compute(x)  (filterbank.h:170-187, the restatement's operation order, no FMA contraction):
//               pre, gain smoothed; y = pre (F0 x + sum_i F_i x[t-i]) - sum_k B_k R[k]; R[O] = y
//   tick()      (filterbank.h:142-148) origin - 1: R rotates right by one (R[0] <- R[O]) -- the
//               same for a tick after a compute (R[O] = y becomes y[t-1]) and a bare tick (the
//               stale row O+1 samples back becomes the newest history row), so bare ticks are exact
//   mixdown     sum_n dist(R[O][n] g[n]) (filterbank.h:130, 138)
// A per-band result is therefore bit-identical to the restatement; the mixdown's summation order
// (per thread, wave tree, workgroups in order) differs from the sequential sum.
//
// Lifetime: the kernel leaves on a STOP request (any block call, get/set_state, setter upload,
// destroy ...: fb_rt_stop), or by itself after kIdle of the 100 MHz real-time counter without a
// request, so every wave always reaches its end.  On the way out it writes the band state back in
// the block engines' layout (ystate / xhist / pg, plus the ring's spare row) and its epoch to
// the mailbox; stream order puts every later launch after it.
#include <chrono>
#include <cstring>

#include "hz_fb_impl.h"

namespace {

constexpr long long kIdle = 10000000;   // 100 ms at 100 MHz without a request: leave
constexpr int kRtThreads = 1024;
constexpr int kMaxGroups = 128;         // every workgroup must be resident (one per CU)
constexpr long long kQuit = -1;

// host-pinned mailbox: request line, then one 64-byte response line per workgroup
struct RtReq {
    double x, param;
    long long ticks;   // bare rotations before the op (taken mod O+1 by the host)
    long long op;      // bit 0: compute; bits 8..15: distortion id; kOpStop: leave
    long long req;     // request number, written last
    double cached;     // (host only) pinned source of a cached sample copied to a device buffer
    long long pad[2];
};
struct RtSlot {
    double y;
    long long done;     // last request served (written after y)
    long long exited;   // epoch of the instance whose workgroup left
    long long pad[5];
};
static_assert(sizeof(RtReq) == 64 && sizeof(RtSlot) == 64, "one cache line each");
constexpr long long kOpStop = 1LL << 20;

// device-memory control word: workgroup 0's idle-exit decision (kQuit), reset per launch
struct RtCtl {
    long long go;
    long long pad[7];
};

struct RtArgs {
    RtReq* req;
    RtSlot* slot;
    RtCtl* ctl;
    const double* coef;   // [N][2O+1]: forward O+1, back O
    const double* pin;
    const double* gin;
    double* ystate;       // [N][O] y[t-1-k] (the block engines' current buffer)
    double* yspare;       // [N][O] the other buffer: [.][O-1] = the ring's spare row
    double* pg;           // [N][2] pre, gain
    double* xhist;        // [O]
    double* xspare;       // [O]: [O-1] = the input ring's spare entry
    long long epoch;
    int N;
    int spare_valid;      // the spare rows are known (else read as 0; the host refuses bare ticks then)
    double sp, sg;
};

__device__ __forceinline__ long long ld_sys(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ldd_sys(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ long long ldr_sys(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(long long* p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <int O, int BPT>
__global__ __launch_bounds__(kRtThreads) void fb_rt_kernel(RtArgs a) {
#pragma clang fp contract(off)
    __shared__ long long s_req, s_ticks, s_op;
    __shared__ double s_x, s_param;
    __shared__ double s_part[kRtThreads / 64];
    __shared__ double s_y[BPT * kRtThreads];   // distortion path: the band outputs x gains
    constexpr int R1 = O + 1;
    const int tid = threadIdx.x;
    const int g = blockIdx.x;
    const int nt = blockDim.x;
    const long base = (long)g * nt * BPT;
    double f[BPT][R1], bk[BPT][O > 0 ? O : 1], R[BPT][R1], pre[BPT], gg[BPT], pi[BPT], gi[BPT];
    bool live[BPT];
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
        const long b = base + tid + (long)j * nt;
        live[j] = b < a.N;
        const long bc = live[j] ? b : 0;
        const double* c = a.coef + bc * (2 * O + 1);
#pragma unroll
        for (int i = 0; i <= O; ++i) f[j][i] = live[j] ? c[i] : 0.0;
#pragma unroll
        for (int k = 0; k < O; ++k) {
            bk[j][k] = live[j] ? c[O + 1 + k] : 0.0;
            R[j][k] = live[j] ? a.ystate[bc * O + k] : 0.0;
        }
        R[j][O] = (live[j] && O > 0 && a.spare_valid) ? a.yspare[bc * O + (O > 0 ? O - 1 : 0)] : 0.0;
        pre[j] = live[j] ? a.pg[2 * bc] : 0.0;
        gg[j] = live[j] ? a.pg[2 * bc + 1] : 0.0;
        pi[j] = live[j] ? a.pin[bc] : 0.0;
        gi[j] = live[j] ? a.gin[bc] : 0.0;
    }
    double XR[R1];   // input ring in the same order (wave-uniform)
#pragma unroll
    for (int k = 0; k < O; ++k) XR[k] = a.xhist[k];
    XR[O] = (O > 0 && a.spare_valid) ? a.xspare[O > 0 ? O - 1 : 0] : 0.0;

    auto rotate = [&]() {
        if constexpr (O > 0) {
#pragma unroll
            for (int j = 0; j < BPT; ++j) {
                const double t = R[j][O];
#pragma unroll
                for (int k = O; k >= 1; --k) R[j][k] = R[j][k - 1];
                R[j][0] = t;
            }
            const double t = XR[O];
#pragma unroll
            for (int k = O; k >= 1; --k) XR[k] = XR[k - 1];
            XR[0] = t;
        }
    };

    // every workgroup polls the host mailbox itself (no forwarding latency); the idle exit is
    // decided by workgroup 0 alone and published through device memory (a.ctl->go = kQuit), which
    // the others poll too -- a workgroup may thus serve one request more than another before
    // leaving; each resumes from its own last served request (its response line) when relaunched
    long long seen = ldr_sys(&a.slot[g].done);   // this workgroup's last served (or consumed STOP) request
    long long last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (tid == 0) {
            long long r = 0;
            for (;;) {
                r = ld_sys(&a.req->req);
                if (r != seen) break;
                if (g == 0) {
                    if (__builtin_amdgcn_s_memrealtime() - last > kIdle) {
                        __hip_atomic_store(&a.ctl->go, kQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        r = kQuit;
                        break;
                    }
                } else if (__hip_atomic_load(&a.ctl->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kQuit) {
                    r = kQuit;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            long long op = 0;
            if (r != kQuit) {
                op = ldr_sys(&a.req->op);
                s_x = ldd_sys(&a.req->x);
                s_param = ldd_sys(&a.req->param);
                s_ticks = ldr_sys(&a.req->ticks);
                if (op & kOpStop) {
                    seen = r;   // consumed: a later instance must not take it for a new request
                    r = kQuit;
                }
            }
            s_op = op;
            s_req = r;
        }
        __syncthreads();
        const long long r = s_req;
        if (r == kQuit) break;
        const long long ticks = s_ticks, op = s_op;
        const double x = s_x, param = s_param;
        for (long long q = 0; q < ticks; ++q) rotate();
        if (op & 1) {   // compute (filterbank.h:170-187)
#pragma unroll
            for (int j = 0; j < BPT; ++j) {
                pre[j] = (1 - a.sp) * pi[j] + a.sp * pre[j];
                gg[j] = (1 - a.sg) * gi[j] + a.sg * gg[j];
                double ff = f[j][0] * x;
#pragma unroll
                for (int i = 1; i <= O; ++i) ff += f[j][i] * XR[i - 1];
                double bsum = 0;
#pragma unroll
                for (int k = 0; k < O; ++k) bsum += bk[j][k] * R[j][k];
                R[j][O] = ff * pre[j] - bsum;
            }
            XR[O] = x;
        }
        // mixdown of the row at origin (filterbank.h:130 / 138)
        const int dist = (int)((op >> 8) & 0xff);
        double v = 0.0;
        if (dist == HZ_DIST_NONE) {
#pragma unroll
            for (int j = 0; j < BPT; ++j) v += live[j] ? R[j][O] * gg[j] : 0.0;
        } else {
            // through LDS, one band at a time: the functors' atan stays out of the band registers
#pragma unroll
            for (int j = 0; j < BPT; ++j) s_y[j * nt + tid] = R[j][O] * gg[j];
#pragma unroll 1
            for (int j = 0; j < BPT; ++j) {
                const double yg = s_y[j * nt + tid];
                double d = yg;
                if (dist == HZ_DIST_SOFTCLIP) d = hz::dist_apply<HZ_DIST_SOFTCLIP>(yg, param);
                else if (dist == HZ_DIST_SATURATE) d = hz::dist_apply<HZ_DIST_SATURATE>(yg, param);
                else d = hz::dist_apply<HZ_DIST_LIMITER>(yg, param);
                v += base + tid + (long)j * nt < a.N ? d : 0.0;
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if ((tid & 63) == 0) s_part[tid >> 6] = v;
        __syncthreads();
        if (tid == 0) {
            double s = 0.0;
            for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += s_part[w];
            __hip_atomic_store(&a.slot[g].y, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            st_sys(&a.slot[g].done, r);
        }
        seen = r;
        last = __builtin_amdgcn_s_memrealtime();
    }
    // leave: the band state back in the block engines' layout
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
        if (!live[j]) continue;
        const long b = base + tid + (long)j * nt;
#pragma unroll
        for (int k = 0; k < O; ++k) a.ystate[b * O + k] = R[j][k];
        if constexpr (O > 0) a.yspare[b * O + O - 1] = R[j][O];
        a.pg[2 * b] = pre[j];
        a.pg[2 * b + 1] = gg[j];
    }
    if (g == 0 && tid == 0) {
#pragma unroll
        for (int k = 0; k < O; ++k) a.xhist[k] = XR[k];
        if constexpr (O > 0) a.xspare[O - 1] = XR[O];
    }
    __syncthreads();
    if (tid == 0) {
        __hip_atomic_store(&a.slot[g].done, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        st_sys(&a.slot[g].exited, a.epoch);
    }
}

typedef void (*RtKernel)(RtArgs);
template <int O>
RtKernel pick_bpt(int bpt) {
    if constexpr (O <= 2) {
        if (bpt >= 2) return fb_rt_kernel<O, 2>;
    }
    return fb_rt_kernel<O, 1>;
}
RtKernel pick_rt(int O, int bpt) {
    switch (O) {
    case 0: return pick_bpt<0>(bpt);
    case 1: return pick_bpt<1>(bpt);
    case 2: return pick_bpt<2>(bpt);
    case 3: return pick_bpt<3>(bpt);
    default: return pick_bpt<4>(bpt);
    }
}

long long host_load(const long long* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

}  // namespace

namespace hz_fbi {

// geometry: threads per workgroup, bands per thread, workgroups
static void rt_geometry(const hz_fb* h, int* threads, int* bpt, int* groups) {
    const int N = h->N;
    const int t = std::min(kRtThreads, (N + 63) / 64 * 64);
    // one band per thread up to 64 workgroups; then two (orders <= 2: registers without spills)
    const int b = (long)N > 64L * t && h->order <= 2 ? 2 : 1;
    *threads = t;
    *bpt = b;
    *groups = (int)((N + (long)t * b - 1) / ((long)t * b));
}

bool fb_rt_supported(const hz_fb* h) {
    int t, b, G;
    rt_geometry(h, &t, &b, &G);
    return G <= kMaxGroups;
}

// has the instance left (on its own, idle)?
static bool rt_left(const hz_fb* h) {
    const RtSlot* slot = (const RtSlot*)((char*)h->rt.mb + sizeof(RtReq));
    return host_load(&slot[0].exited) == h->rt.epoch;
}

// bookkeeping once the instance is gone (or going): the canonical state is (will be) current
static void rt_detach(hz_fb* h) {
    h->rt.active = false;
    h->spare_ok = h->rt.spare_known;
}

int fb_rt_stop(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    if (T.active) {
        if (!rt_left(h)) {
            RtReq* q = (RtReq*)T.mb;
            q->op = kOpStop;
            q->ticks = 0;
            __atomic_store_n(&q->req, ++T.seq, __ATOMIC_RELEASE);
        }
        rt_detach(h);
    }
    // ticks since the last served sample: the block engines' ring rotation
    const int O = h->order;
    const long rot = O > 0 ? T.pending_ticks % (O + 1) : 0;
    T.pending_ticks = 0;
    for (long i = 0; i < rot; ++i) HZ_TRY(fb_tick_rotate(h));
    return HZ_OK;
}

int fb_rt_resolve(hz_fb* h, double* y0) {
    if (!h->rt.computed) return 0;
    HZ_TRY(hz_fb_sample(h, 0.0, h->dist_id, h->dist_param, y0));
    HZ_TRY(hz_fb_sample_tick(h));
    HZ_TRY(fb_rt_stop(h));
    return 1;
}

double* fb_rt_cached_slot(hz_fb* h) { return &((RtReq*)h->rt.mb)->cached; }

void fb_rt_free(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    if (T.mb) (void)hipHostFree(T.mb);
    if (T.d_ctl) (void)hipFree(T.d_ctl);
    if (T.d_coef) (void)hipFree(T.d_coef);
    T.mb = T.dmb = T.d_ctl = nullptr;
    T.d_coef = nullptr;
    T.active = false;
}

static int rt_start(hz_fb* h) {
    hz_fb::Rt& T = h->rt;
    int threads, bpt, G;
    rt_geometry(h, &threads, &bpt, &G);
    const int O = h->order;
    if (!T.mb) {
        const size_t bytes = sizeof(RtReq) + sizeof(RtSlot) * kMaxGroups;
        HZ_TRY_HIP(hipHostMalloc(&T.mb, bytes, hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(T.mb, 0, bytes);
        HZ_TRY_HIP(hipHostGetDevicePointer(&T.dmb, T.mb, 0));
        HZ_TRY_HIP(hipMalloc(&T.d_ctl, sizeof(RtCtl)));
    }
    // coefficients in the kernel's layout (rare: a start follows a setter or a block call)
    const size_t nc = (size_t)h->N * (2 * O + 1);
    if (nc > T.coef_cap) {
        if (T.d_coef) HZ_TRY_HIP(hipFree(T.d_coef));
        T.d_coef = nullptr;
        HZ_TRY_HIP(hipMalloc(&T.d_coef, sizeof(double) * nc));
        T.coef_cap = nc;
    }
    T.h_coef.resize(nc);
    for (int n = 0; n < h->N; ++n) {
        for (int i = 0; i <= O; ++i) T.h_coef[(size_t)n * (2 * O + 1) + i] = h->F[(size_t)n * (O + 1) + i];
        for (int k = 0; k < O; ++k) T.h_coef[(size_t)n * (2 * O + 1) + O + 1 + k] = h->B[(size_t)n * O + k];
    }
    HZ_TRY_HIP(hipMemcpyAsync(T.d_coef, T.h_coef.data(), sizeof(double) * nc, hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipMemsetAsync(T.d_ctl, 0, sizeof(RtCtl), h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // pageable sources; earlier work drained
    RtArgs a;
    a.req = (RtReq*)T.dmb;
    a.slot = (RtSlot*)((char*)T.dmb + sizeof(RtReq));
    a.ctl = (RtCtl*)T.d_ctl;
    a.coef = T.d_coef;
    a.pin = h->d_pin;
    a.gin = h->d_gin;
    a.ystate = h->d_ystate[h->scur];
    a.yspare = h->d_ystate[h->scur ^ 1];
    a.pg = h->d_pg[h->scur];
    a.xhist = h->d_xhist[h->xcur];
    a.xspare = h->d_xhist[h->xcur ^ 1];
    a.epoch = ++T.epoch;
    a.N = h->N;
    a.spare_valid = h->spare_ok ? 1 : 0;
    a.sp = h->sp;
    a.sg = h->sg;
    hipLaunchKernelGGL(pick_rt(O, bpt), dim3(G), dim3(threads), 0, h->stream, a);
    HZ_TRY_HIP(hipGetLastError());
    T.active = true;
    T.groups = G;
    T.spare_known = h->spare_ok;
    // the resident kernel owns the state from here; the stationary history no longer follows it
    h->resp.run = 0;
    return HZ_OK;
}

}  // namespace hz_fbi

extern "C" {

int hz_fb_sample(hz_fb* h, double x, int dist_id, double param, double* y) {
    if (!h || !y || dist_id < HZ_DIST_NONE || dist_id > HZ_DIST_LIMITER) {
        hz::set_error("hz_fb_sample: invalid arguments");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    hz_fb::Rt& T = h->rt;
    const int O = h->order;
    const long ticks = O > 0 ? T.pending_ticks % (O + 1) : 0;
    const bool spare_known = T.active ? T.spare_known : h->spare_ok;   // the ring row a bare tick exposes
    if (!T.computed && ticks > 0 && !spare_known) {
        hz::set_error("hz_fb_sample: tick() without operator() after a block call or set_state: the ring row "
                      "it would reuse (O+1 samples back) is not kept");
        return HZ_E_STATE;
    }
    if (!hz_fbi::fb_rt_supported(h)) {
        hz::set_error("hz_fb_sample: %d bands exceed the per-sample engine (%d workgroups of %d)", h->N, kMaxGroups,
                      kRtThreads);
        return HZ_E_UNSUPPORTED;
    }
    const bool dirty = h->dirty_coef || h->dirty_pin || h->dirty_gin || h->tv_pending || h->resp.implicit;
    if (T.active && (dirty || hz_fbi::rt_left(h))) {
        // a setter since the last sample (or the instance left, idle): restart over fresh uploads;
        // the pending ticks stay with the request
        const long keep = T.pending_ticks;
        T.pending_ticks = 0;
        HZ_TRY(hz_fbi::fb_rt_stop(h));
        T.pending_ticks = keep;
    }
    if (!T.active) {
        HZ_TRY(hz_fbi::fb_upload_staged(h));
        HZ_TRY(hz_fbi::fb_resp_materialize(h));
        HZ_TRY(hz_fbi::rt_start(h));
    }
    RtReq* q = (RtReq*)T.mb;
    RtSlot* slot = (RtSlot*)((char*)T.mb + sizeof(RtReq));
    const bool compute = !T.computed;
    q->x = x;
    q->param = param;
    q->ticks = ticks;
    q->op = (compute ? 1 : 0) | ((long long)dist_id << 8);
    const long long want = ++T.seq;
    __atomic_store_n(&q->req, want, __ATOMIC_RELEASE);
    // wait for every workgroup; an instance that left (idle) before taking the request is
    // relaunched and serves it (stream order: after the old one's state write-back)
    const auto t0 = std::chrono::steady_clock::now();
    int relaunched = 0;
    for (;;) {
        bool all = true;
        for (int g = 0; g < T.groups && all; ++g) all = host_load(&slot[g].done) >= want;
        if (all) break;
        if (hz_fbi::rt_left(h)) {
            // workgroup 0 left (idle) as the request arrived: every workgroup leaves after at most
            // this request; the relaunch (stream-ordered after them) resumes each workgroup from
            // its own response line, so the ones that served it do not serve it twice
            if (relaunched++ > 2) {
                hz::set_error("hz_fb_sample: the per-sample engine left repeatedly without serving");
                return HZ_E_HIP;
            }
            hz_fbi::rt_detach(h);
            HZ_TRY(hz_fbi::rt_start(h));
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
            hz::set_error("hz_fb_sample: the per-sample engine did not answer within 5 s");
            return HZ_E_HIP;
        }
    }
    double s = 0.0;
    for (int g = 0; g < T.groups; ++g) s += slot[g].y;
    *y = s;
    T.pending_ticks = 0;
    if (compute) {
        T.computed = true;
        T.spare_known = true;   // the row at origin now holds this sample's outputs
        T.cached = s;
        hz_fbi::fb_mirror_advance(h, 1);
    }
    T.cached_dist = dist_id;
    return HZ_OK;
}

int hz_fb_sample_tick(hz_fb* h) {
    if (!h) return HZ_E_INVALID;
    ++h->rt.pending_ticks;
    h->rt.computed = false;
    return HZ_OK;
}

int hz_fb_sample_info(hz_fb* h, int* active, long long* served, int* groups) {
    if (!h) return HZ_E_INVALID;
    const bool on = h->rt.active && h->rt.mb && !hz_fbi::rt_left(h);
    if (active) *active = on ? 1 : 0;
    if (served) *served = h->rt.seq;
    int t, b, G;
    hz_fbi::rt_geometry(h, &t, &b, &G);
    if (groups) *groups = G;
    return HZ_OK;
}

}  // extern "C"
