// hz_rt.hip -- the per-sample server (hz_rt.h): one resident kernel per device, serving the
// per-sample operator calls of the input-driven banks through a pinned-host mailbox.
//
//   host:   op arguments -> the request line, then the request number (release store)
//   device: every workgroup polls the request number (system-scope acquire), loads the line's
//           arguments (system scope), runs its share of the op's units (bands, lines, grains)
//           and writes its partial and the request number to its own 64-byte response line
//   host:   waits for every workgroup's response, sums the partials in workgroup order
// State stays in device memory in the block engines' layouts (rings, smoothers, coefficients),
// so per-sample and block calls interleave; every request ends with a system-scope release (the
// response) and starts with an acquire (the poll), and the host orders block work before and
// after requests by stream synchronisation.
//
// Exactly-once service: the host writes a request line only after every participating workgroup
// (named in the request word itself) acknowledged the previous one; a workgroup resumes from its
// own last acknowledged request when the kernel is relaunched after an idle exit (workgroup 0 decides it after kIdleNs without a request and the
// others follow through a device-memory flag), so a request is served once by each workgroup even
// when it arrives while the instance leaves.
#include <immintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hz_rt.h"

namespace hz_rt {

constexpr long long kIdleTicks = 200000;   // 2 ms of the 100 MHz real-time counter without a request
                                           // (env HZ_RT_IDLE_US overrides it at each launch)
constexpr long long kQuit = -1;

struct ServerArgs {
    Req* req;
    Slot* slot;
    long long* ctl;   // device memory: workgroup 0's idle-exit decision
    long long epoch;
    long long idle;   // real-time ticks without a request before leaving
    // (tests) workgroup 0 holds its answer to request stall_req back by stall ticks: an unanswered
    // request as the host sees it (env HZ_RT_DEBUG_STALL = "request:microseconds")
    long long stall_req, stall;
};

namespace {

__device__ __forceinline__ long long ld_acq(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ long long ld_sys(const long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ double ldd_sys(const double* p) {
    return __longlong_as_double(ld_sys((const long long*)p));
}
__device__ __forceinline__ void st_sys(long long* p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void std_sys(double* p, double v) { st_sys((long long*)p, __double_as_longlong(v)); }
__device__ __forceinline__ void st_rel(long long* p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct SrvLds {
    long long w[kArgWords + 1];
    long long req;
    int grp;
    double part[kThreads / 64];
    double mpart[kThreads / 64][kMaxMany];   // OP_FB_MANY: per wave and member
    // OP_GRAN (one workgroup): the handle's grain list and this sample's terms
    long long gkey, gver;
    int gcount;
    Grain gr[kMaxGrains];
    double term[kMaxGrains];
};

// ---------------------------------------------------------------------------------------------
// OP_FB: Filterbank operator() / tick() (src/filterbank.h:125-148, 170-187) for the bands of this
// workgroup, in the restatement's operation order without FMA contraction (every band's output
// and state bit-identical to it; the mixdown's order is thread, wave tree, waves, workgroups)
template <int O>
__device__ double op_fb(const FbArgs& a, int g, int groups) {
#pragma clang fp contract(off)
    constexpr int R1 = O + 1;
    if (a.nsparse > 0) {   // one-band setters since the last sample: the owners write the targets
        for (int j = (int)threadIdx.x; j < a.nsparse; j += kThreads) {
            const int b = (int)ldd_sys(a.sparse + 3 * j);
            if ((b / kThreads) % groups == g) {
                a.pin[b] = ldd_sys(a.sparse + 3 * j + 1);
                a.gin[b] = ldd_sys(a.sparse + 3 * j + 2);
            }
        }
        __syncthreads();   // (the band loop below reads them from another thread of the workgroup)
    }
    double v = 0.0;
    for (int b = g * kThreads + (int)threadIdx.x; b < a.N; b += groups * kThreads) {
        const double* c = a.coef + (long)b * (2 * O + 1);
        double f[R1], bk[O > 0 ? O : 1], R[R1];
#pragma unroll
        for (int i = 0; i <= O; ++i) R[i] = a.R[(long)b * R1 + i];
        if (a.reload_coef) {   // coefficients() since the last sample: from the payload
            const double* rc = a.reload_coef + (long)b * (2 * O + 1);
            double* cw = const_cast<double*>(c);
#pragma unroll
            for (int i = 0; i <= 2 * O; ++i) {
                const double cv = ldd_sys(rc + i);
                cw[i] = cv;
                if (i <= O) f[i] = cv;
                else bk[i - O - 1] = cv;
            }
        } else {
#pragma unroll
            for (int i = 0; i <= O; ++i) f[i] = c[i];
#pragma unroll
            for (int k = 0; k < O; ++k) bk[k] = c[O + 1 + k];
        }
        double pre = a.pg[2 * b], gain = a.pg[2 * b + 1];
        double pi, gi;
        if (a.reload) {   // setters since the last sample: the targets from the payload
            pi = ldd_sys(a.reload + b);
            gi = ldd_sys(a.reload + a.N + b);
            a.pin[b] = pi;
            a.gin[b] = gi;
        } else {
            pi = a.pin[b];
            gi = a.gin[b];
        }
        // bare ticks: the ring rotates right (tick() moves origin back; hz_fb_rt.hip)
        for (int q = 0; q < a.ticks; ++q) {
            const double t0 = R[O];
#pragma unroll
            for (int k = O; k >= 1; --k) R[k] = R[k - 1];
            R[0] = t0;
        }
        if (a.compute) {
            pre = (1 - a.sp) * pi + a.sp * pre;
            gain = (1 - a.sg) * gi + a.sg * gain;
            double ff = f[0] * a.x;
#pragma unroll
            for (int i = 1; i <= O; ++i) ff += f[i] * a.xr[i - 1];
            double bsum = 0;
#pragma unroll
            for (int k = 0; k < O; ++k) bsum += bk[k] * R[k];
            R[O] = ff * pre - bsum;
        }
#pragma unroll
        for (int i = 0; i <= O; ++i) a.R[(long)b * R1 + i] = R[i];
        a.pg[2 * b] = pre;
        a.pg[2 * b + 1] = gain;
        const double yg = R[O] * gain;
        double d = yg;
        if (a.dist == HZ_DIST_SOFTCLIP) d = hz::dist_apply<HZ_DIST_SOFTCLIP>(yg, a.param);
        else if (a.dist == HZ_DIST_SATURATE) d = hz::dist_apply<HZ_DIST_SATURATE>(yg, a.param);
        else if (a.dist == HZ_DIST_LIMITER) d = hz::dist_apply<HZ_DIST_LIMITER>(yg, a.param);
        v += d;
    }
    return v;
}

// ---------------------------------------------------------------------------------------------
// OP_FB_MANY: operator() of several Filterbanks (one order O) for one sample each -- op_fb's band
// arithmetic, op for op -- over the descriptor's 64-band chunks: wave w of workgroup g takes chunks
// (g * waves + w) + k * (groups * waves); each chunk's mixdown is a wave tree, added per member in
// chunk order into the wave's LDS slot, then summed over the waves in order into out[g][member]
template <int O>
__device__ void op_fb_many(const ManyArgs& a, const long long* xvw, int g, int groups, SrvLds& s) {
#pragma clang fp contract(off)
    constexpr int R1 = O + 1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int kWaves = kThreads / 64;
    const int H = a.H;
    if (lane < kMaxMany) s.mpart[wave][lane] = 0.0;
    for (int c = g * kWaves + wave; c < a.nchunks; c += groups * kWaves) {
        const ManyChunk& ck = a.chunks[c];
        const int m = ck.m, b = lane;
        const int sh = 4 * m;
        const int ticks = (int)((a.meta >> sh) & 7), compute = (int)((a.meta >> (sh + 3)) & 1);
        const double* xm = (const double*)xvw + m * (O + 2);   // x, xr[0..O]
        double v = 0.0;
        if (b < ck.n) {
            const double* cf = ck.coef + (long)b * (2 * O + 1);
            double f[R1], bk[O > 0 ? O : 1], R[R1];
#pragma unroll
            for (int i = 0; i <= O; ++i) {
                R[i] = ck.R[(long)b * R1 + i];
                f[i] = cf[i];
            }
#pragma unroll
            for (int k = 0; k < O; ++k) bk[k] = cf[O + 1 + k];
            double pre = ck.pg[2 * b], gain = ck.pg[2 * b + 1];
            const double pi = ck.pin[b], gi = ck.gin[b];
            for (int q = 0; q < ticks; ++q) {   // bare ticks: the ring rotates right
                const double t0 = R[O];
#pragma unroll
                for (int k = O; k >= 1; --k) R[k] = R[k - 1];
                R[0] = t0;
            }
            if (compute) {
                pre = (1 - ck.sp) * pi + ck.sp * pre;
                gain = (1 - ck.sg) * gi + ck.sg * gain;
                double ff = f[0] * xm[0];
#pragma unroll
                for (int i = 1; i <= O; ++i) ff += f[i] * xm[i];   // xr[i - 1]
                double bsum = 0;
#pragma unroll
                for (int k = 0; k < O; ++k) bsum += bk[k] * R[k];
                R[O] = ff * pre - bsum;
            }
#pragma unroll
            for (int i = 0; i <= O; ++i) ck.R[(long)b * R1 + i] = R[i];
            ck.pg[2 * b] = pre;
            ck.pg[2 * b + 1] = gain;
            const double yg = R[O] * gain;
            v = yg;
            if (a.dist == HZ_DIST_SOFTCLIP) v = hz::dist_apply<HZ_DIST_SOFTCLIP>(yg, a.param);
            else if (a.dist == HZ_DIST_SATURATE) v = hz::dist_apply<HZ_DIST_SATURATE>(yg, a.param);
            else if (a.dist == HZ_DIST_LIMITER) v = hz::dist_apply<HZ_DIST_LIMITER>(yg, a.param);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) s.mpart[wave][m] += v;
    }
    __syncthreads();
    if (tid < H) {
        double y = 0.0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) y += s.mpart[w][tid];   // waves in order
        std_sys(a.out + (long)g * H + tid, y);
    }
}

// ---------------------------------------------------------------------------------------------
// OP_DLY: one sample of every line (src/delay.h:71-89 over src/buffer.h:40-47), the block
// kernel's arithmetic (hz_delay.hip dly_line_kernel) for a 1-sample call: a tap of age 0 reads
// this sample's input (forward) or the partial sum (feedback); the rings take x and y at origin
template <typename T>
__device__ void op_dly(const DlyArgs& a, int g, int groups) {
#pragma clang fp contract(off)
    const unsigned size = a.size, o = a.o;
    for (int l = g * kThreads + (int)threadIdx.x; l < a.N; l += groups * kThreads) {
        const int4* tp = a.taps + (long)l * 2 * a.S;
        const T* gn = (const T*)a.gains + (long)l * 2 * a.S;
        T* rx = (T*)a.rx + (long)l * size;
        T* ry = (T*)a.ry + (long)l * size;
        const T x = (T)(a.xin ? ldd_sys(a.xin + l) : a.x);
        T acc = (T)0;
        for (int i = 0; i < a.S; ++i) {
            const int4 qf = tp[i];
            const T f = gn[i];
            const T b = gn[a.S + i];
            const unsigned af = ((int)o < qf.x) ? (unsigned)qf.z : (unsigned)qf.y;
            const T xv = af == 0 ? x : rx[o >= af ? o - af : o + size - af];
            T yv = (T)0;
            if (b != (T)0) {
                const int4 qb = tp[a.S + i];
                const unsigned ab = ((int)o < qb.x) ? (unsigned)qb.z : (unsigned)qb.y;
                yv = ab == 0 ? acc : ry[o >= ab ? o - ab : o + size - ab];
            }
            const T fx = f * xv;
            const T by = b * yv;
            acc = acc + (fx - by);
        }
        rx[o] = x;
        ry[o] = acc;
        std_sys(a.out + l, (double)acc);
    }
}

// OP_DLY with a line's taps across lanes (S <= 64, SP = S rounded up to a power of two, so a line's
// lanes share a wave): every lane loads its tap's records and ring values at once -- instead of
// one thread walking the taps, a tap record then a ring read per tap -- and the line's first lane
// accumulates in tap order through shuffles (a zero-age feedback tap reads the running sum, as
// op_dly does), so every product and sum is op_dly's, bit for bit
template <class T>
__device__ void op_dly_lanes(const DlyArgs& a, int g, int groups) {
#pragma clang fp contract(off)
    const unsigned size = a.size, o = a.o;
    const int S = a.S;
    int SP = 1;
    while (SP < S) SP <<= 1;
    const int per = kThreads / SP;                   // lines per workgroup pass
    const int i = (int)threadIdx.x % SP, base = (int)threadIdx.x - i;
    const int lanebase = base & 63;
    for (int l0 = g * per; l0 < a.N; l0 += groups * per) {   // uniform across the workgroup
        const int l = l0 + (int)threadIdx.x / SP;
        const bool live = l < a.N && i < S;
        const long lc = live ? l : 0;
        T fx = (T)0, by = (T)0, b = (T)0;
        int zero_age = 0;
        T x = (T)0;
        if (l < a.N) x = (T)(a.xin ? ldd_sys(a.xin + l) : a.x);
        if (live) {
            const int4* tp = a.taps + lc * 2 * S;
            const T* gn = (const T*)a.gains + lc * 2 * S;
            const T* rx = (const T*)a.rx + lc * size;
            const T* ry = (const T*)a.ry + lc * size;
            const int4 qf = tp[i];
            const T f = gn[i];
            b = gn[S + i];
            const unsigned af = ((int)o < qf.x) ? (unsigned)qf.z : (unsigned)qf.y;
            const T xv = af == 0 ? x : rx[o >= af ? o - af : o + size - af];
            fx = f * xv;
            if (b != (T)0) {
                const int4 qb = tp[S + i];
                const unsigned ab = ((int)o < qb.x) ? (unsigned)qb.z : (unsigned)qb.y;
                if (ab == 0) zero_age = 1;
                else by = b * ry[o >= ab ? o - ab : o + size - ab];
            }
        }
        T acc = (T)0;
        for (int k = 0; k < S; ++k) {   // every lane shuffles; the line's lane 0 keeps the sum
            const T fk = __shfl(fx, lanebase + k);
            T bk = __shfl(by, lanebase + k);
            const T gk = __shfl(b, lanebase + k);
            const int zk = __shfl(zero_age, lanebase + k);
            if (zk) bk = gk * acc;
            acc = acc + (fk - bk);
        }
        if (i == 0 && l < a.N) {
            T* rx = (T*)a.rx + (long)l * size;
            T* ry = (T*)a.ry + (long)l * size;
            rx[o] = x;
            ry[o] = acc;
            std_sys(a.out + l, (double)acc);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// OP_GRAN (workgroup 0): the sample at time t of src/granulator.h:88-104 over the source ring,
// the block kernel's per-grain arithmetic (hz_granulator.hip gran_kernel), terms summed in voice
// order by one thread (the block kernel's order)
__device__ __forceinline__ unsigned fastmod(unsigned x, unsigned long fm, unsigned size) {
    const unsigned long low = fm * (unsigned long)x;
    return (unsigned)__umul64hi(low, (unsigned long)size);
}

__device__ double op_gran(const GranArgs& a, SrvLds& s) {
#pragma clang fp contract(off)
    const int tid = threadIdx.x;
    if (s.gkey != a.key || s.gver != a.version) {   // the handle's grain list changed: reload
        __syncthreads();
        const long long* src = (const long long*)a.grains;
        long long* dst = (long long*)s.gr;
        for (int i = tid; i < a.count * 8; i += kThreads) dst[i] = ld_sys(src + i);
        __syncthreads();
        if (tid == 0) {
            s.gkey = a.key;
            s.gver = a.version;
            s.gcount = a.count;
        }
        __syncthreads();
    }
    const long t = a.t;
    const unsigned size = a.size, origin = a.origin;
    for (int e = tid; e < a.count; e += kThreads) {
        const Grain& gr = s.gr[e];
        double term = 0.0;
        if (t >= gr.t_first && t < gr.t_end) {
            const unsigned ticks = gr.ticks0 + (unsigned)(t - gr.t_first);
            const double position = gr.offsets + (1 - gr.speeds) * ticks;
            const int center = (int)position;
            const double disp = position - center;
            long tau0, tau1;
            if (center >= 0 && (unsigned)center < size) {
                tau0 = t - center;
                tau1 = (unsigned)center + 1u < size ? tau0 - 1 : t;
            } else {
                const unsigned x0 = origin - (unsigned)center + size;
                const unsigned s0 = fastmod(x0, a.fm, size);
                const unsigned s1 = x0 == 0u ? a.wrap1 : (s0 == 0u ? size - 1u : s0 - 1u);
                tau0 = t - (long)(origin >= s0 ? origin - s0 : origin + size - s0);
                tau1 = t - (long)(origin >= s1 ? origin - s1 : origin + size - s1);
            }
            // this sample's input is the argument (the ring takes it below)
            const double v0 = tau0 == t ? a.x : a.ring[tau0 & a.mask];
            const double v1 = tau1 == t ? a.x : a.ring[tau1 & a.mask];
            const double src = v0 * (1 - disp) + v1 * disp;
            const double tk = (double)ticks;
            double phase;
            if (gr.rsizes != 0.0) {
                const double q0 = tk * gr.rsizes;
                phase = __builtin_fma(__builtin_fma(-q0, gr.sizes, tk), gr.rsizes, q0);
            } else {
                phase = tk / gr.sizes;
            }
            term = gr.gains * src * (0.5 * (1 - hann_cos(2 * hz::kPI * phase, true)));   // wave.h:148
        }
        s.term[e] = term;
    }
    __syncthreads();
    double out = 0.0;
    if (tid == 0) {
        for (int e = 0; e < a.count; ++e) {
            const Grain& gr = s.gr[e];
            if (t >= gr.t_first && t < gr.t_end) out += s.term[e];
        }
        a.ring[t & a.mask] = a.x;
    }
    return out;
}

__global__ __launch_bounds__(kThreads) void rt_server_kernel(ServerArgs a) {
    __shared__ SrvLds s;
    const int tid = threadIdx.x;
    const int g = blockIdx.x;
    if (tid == 0) s.gkey = -1;
    long long seen = ld_sys(&a.slot[g].done);   // resume after this workgroup's last served request
    long long last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (tid == 0) {
            long long r;
            int grp = 0;
            for (;;) {
                // the request word carries the participating workgroups (low 4 bits): a workgroup
                // decides from this one 64-bit load, and only participants -- whom the host waits
                // for before it rewrites the line -- read the arguments
                const long long wd = ld_acq(&a.req->req);
                r = wd >> 4;
                grp = (int)(wd & 15);
                if (r != seen) break;
                if (g == 0) {
                    if (__builtin_amdgcn_s_memrealtime() - last > a.idle) {
                        __hip_atomic_store(a.ctl, kQuit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        r = kQuit;
                        break;
                    }
                } else if (__hip_atomic_load(a.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == kQuit) {
                    r = kQuit;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s.req = r;
            s.grp = grp;
        }
        __syncthreads();
        const long long r = s.req;
        if (r == kQuit) break;
        const int groups = s.grp;
        if (g >= groups) {   // not taking part: no answer (the host waits for the participants only)
            seen = r;
            last = __builtin_amdgcn_s_memrealtime();
            continue;
        }
        if (tid <= kArgWords) s.w[tid] = ld_sys((const long long*)&a.req->op + tid);   // op|groups, args
        __syncthreads();
        const int op = (int)(unsigned)(s.w[0] & 0xffffffffu);
        if (op == OP_STOP) {
            seen = r;
            break;
        }
        double y = 0.0;
        if (g < groups) {
            if (op == OP_FB) {
                FbArgs fa;
                __builtin_memcpy(&fa, &s.w[1], sizeof(fa));
                switch (fa.O) {
                case 0: y = op_fb<0>(fa, g, groups); break;
                case 1: y = op_fb<1>(fa, g, groups); break;
                case 2: y = op_fb<2>(fa, g, groups); break;
                case 3: y = op_fb<3>(fa, g, groups); break;
                default: y = op_fb<4>(fa, g, groups); break;
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) y += __shfl_xor(y, o);
                if ((tid & 63) == 0) s.part[tid >> 6] = y;
                __syncthreads();
                y = 0.0;
#pragma unroll
                for (int w = 0; w < kThreads / 64; ++w) y += s.part[w];   // waves in order
            } else if (op == OP_DLY) {
                DlyArgs da;
                __builtin_memcpy(&da, &s.w[1], sizeof(da));
                if (da.S <= 64) {
                    if (da.is_float) op_dly_lanes<float>(da, g, groups);
                    else op_dly_lanes<double>(da, g, groups);
                } else if (da.is_float) {
                    op_dly<float>(da, g, groups);
                } else {
                    op_dly<double>(da, g, groups);
                }
            } else if (op == OP_FB_MANY) {
                ManyArgs ma;
                __builtin_memcpy(&ma, &s.w[1], sizeof(ManyArgs) - sizeof(double));
                const long long* xvw = &s.w[1 + kManyHeader];
                switch (ma.O) {
                case 0: op_fb_many<0>(ma, xvw, g, groups, s); break;
                case 1: op_fb_many<1>(ma, xvw, g, groups, s); break;
                case 2: op_fb_many<2>(ma, xvw, g, groups, s); break;
                case 3: op_fb_many<3>(ma, xvw, g, groups, s); break;
                default: op_fb_many<4>(ma, xvw, g, groups, s); break;
                }
            } else if (op == OP_GRAN) {
                GranArgs ga;
                __builtin_memcpy(&ga, &s.w[1], sizeof(ga));
                y = op_gran(ga, s);
            }
        }
        // every storing wave drains, then one lane answers with a system-scope release
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            if (a.stall > 0 && g == 0 && r == a.stall_req) {   // (tests) a late answer, bounded
                const long long t0 = __builtin_amdgcn_s_memrealtime();
                while (__builtin_amdgcn_s_memrealtime() - t0 < a.stall) __builtin_amdgcn_s_sleep(100);
            }
            std_sys(&a.slot[g].y, y);
            st_rel(&a.slot[g].done, r);
        }
        seen = r;
        last = __builtin_amdgcn_s_memrealtime();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
        st_sys(&a.slot[g].done, seen);
        st_rel(&a.slot[g].exited, a.epoch);
    }
}

long long host_load(const long long* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

}  // namespace

struct Server {
    int device = 0;
    std::recursive_mutex mu;
    hipStream_t stream = nullptr;
    void* mb = nullptr;          // pinned: Req, then kGroups Slots
    // large-BAR devices: the request line in fine-grained device memory the host stores into
    // (write-combined, fenced), so the workgroups poll and read arguments from their own memory
    // instead of across the host link (scripts/probe/mailbox_probe.hip: round trip 5.2 -> 2.6 us);
    // the answers stay in pinned host memory (env HZ_RT_HOST_MAILBOX=1: the request line there too)
    Req* d_req = nullptr;
    long long* d_ctl = nullptr;
    long long seq = 0, epoch = 0, requests = 0, launches = 0;
    bool active = false;
    bool broken = false;         // a request went unanswered: later calls fail (no double service)
    long long answer_ms = 5000;  // the host's wait for an answer
    double* pay = nullptr;       // pinned payload / result
    size_t pay_cap = 0;
    double* res = nullptr;
    size_t res_cap = 0;
    Req* req() { return d_req ? d_req : (Req*)mb; }
    // the host's stores to a device request line are write-combined: drained in order around the
    // request word (no-op for the pinned line, whose x86 stores are ordered)
    void wc_fence() {
        if (d_req) _mm_sfence();
    }
    Slot* slot() { return (Slot*)((char*)mb + sizeof(Req)); }
};

namespace {

Server* g_servers[64] = {};
std::mutex g_servers_mu;

int srv_init(Server* s) {
    HZ_TRY_HIP(hipSetDevice(s->device));
    int least = 0, greatest = 0;
    HZ_TRY_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
    // the highest priority: a hardware queue of its own (normal streams keep theirs)
    HZ_TRY_HIP(hipStreamCreateWithPriority(&s->stream, hipStreamNonBlocking, greatest));
    const size_t bytes = sizeof(Req) + sizeof(Slot) * kGroups;
    HZ_TRY_HIP(hipHostMalloc(&s->mb, bytes, hipHostMallocCoherent | hipHostMallocMapped));
    std::memset(s->mb, 0, bytes);
    HZ_TRY_HIP(hipMalloc(&s->d_ctl, 64));
    int large_bar = 0;
    if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, s->device) != hipSuccess) large_bar = 0;
    if (large_bar && !std::getenv("HZ_RT_HOST_MAILBOX")) {
        void* d = nullptr;
        if (hipExtMallocWithFlags(&d, sizeof(Req), hipDeviceMallocFinegrained) == hipSuccess) {
            if (hipMemset(d, 0, sizeof(Req)) == hipSuccess) s->d_req = (Req*)d;
            else (void)hipFree(d);
        }
    }
    return HZ_OK;
}

bool srv_left(Server* s) { return host_load(&s->slot()[0].exited) == s->epoch; }

int srv_launch(Server* s) {
    HZ_TRY_HIP(hipMemsetAsync(s->d_ctl, 0, 64, s->stream));
    ServerArgs a;
    void* dmb = nullptr;
    HZ_TRY_HIP(hipHostGetDevicePointer(&dmb, s->mb, 0));
    a.req = s->d_req ? s->d_req : (Req*)dmb;
    a.slot = (Slot*)((char*)dmb + sizeof(Req));
    a.ctl = s->d_ctl;
    a.epoch = ++s->epoch;
    a.idle = kIdleTicks;
    if (const char* e = std::getenv("HZ_RT_IDLE_US")) {
        const long long us = std::atoll(e);
        if (us > 0 && us <= 10000000) a.idle = us * 100;
    }
    a.stall_req = a.stall = 0;
    s->answer_ms = 5000;
    // test hooks, honoured only with HZ_RT_TEST_HOOKS=1 (a stray variable in production must not
    // stall the server or shorten the host's wait): INTEGRATION.md section 4
    const char* hooks = std::getenv("HZ_RT_TEST_HOOKS");
    const bool test_hooks = hooks && hooks[0] == '1' && hooks[1] == 0;
    if (const char* e = test_hooks ? std::getenv("HZ_RT_DEBUG_STALL") : nullptr) {   // (tests) "request:microseconds", <= 2 s
        long long rq = 0, us = 0;
        if (std::sscanf(e, "%lld:%lld", &rq, &us) == 2 && rq > 0 && us > 0 && us <= 2000000) {
            a.stall_req = rq;
            a.stall = us * 100;
        }
    }
    if (const char* e = test_hooks ? std::getenv("HZ_RT_ANSWER_TIMEOUT_MS") : nullptr) {   // (tests) the host's wait
        const long long ms = std::atoll(e);
        if (ms > 0 && ms <= 5000) s->answer_ms = ms;
    }
    hipLaunchKernelGGL(rt_server_kernel, dim3(kGroups), dim3(kThreads), 0, s->stream, a);
    HZ_TRY_HIP(hipGetLastError());
    s->active = true;
    ++s->launches;
    return HZ_OK;
}

// one server's resident instance leaves (a STOP request) and the call waits for it: the next
// request relaunches it with every XCD's L2 written back and invalidated by the kernel boundary
void srv_quiesce(Server* s) {
    if (!s->active || srv_left(s)) {
        s->active = false;
        return;
    }
    Req* q = s->req();
    q->op = OP_STOP;
    q->groups = kGroups;
    s->wc_fence();
    __atomic_store_n(&q->req, (++s->seq << 4) | kGroups, __ATOMIC_RELEASE);
    s->wc_fence();
    const auto t0 = std::chrono::steady_clock::now();
    while (!srv_left(s) && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) {
    }
    (void)hipStreamSynchronize(s->stream);
    s->active = false;
}

void srv_shutdown() {
    // process exit: every resident instance leaves (a STOP request), so no wave outlives the host
    for (Server* s : g_servers) {
        if (!s || !s->active || srv_left(s)) continue;
        std::lock_guard<std::recursive_mutex> lk(s->mu);
        Req* q = s->req();
        q->op = OP_STOP;
        q->groups = kGroups;
        s->wc_fence();
        __atomic_store_n(&q->req, (++s->seq << 4) | kGroups, __ATOMIC_RELEASE);
        s->wc_fence();
        const auto t0 = std::chrono::steady_clock::now();
        while (!srv_left(s) && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) {
        }
        (void)hipStreamSynchronize(s->stream);
        s->active = false;
    }
}

}  // namespace

Server* server(int device) {
    std::lock_guard<std::mutex> lk(g_servers_mu);
    if (device < 0 || device >= 64) return nullptr;
    if (!g_servers[device]) {
        Server* s = new Server();
        s->device = device;
        if (srv_init(s) != HZ_OK) {
            delete s;
            return nullptr;
        }
        static bool registered = false;
        if (!registered) {
            std::atexit(srv_shutdown);
            registered = true;
        }
        g_servers[device] = s;
    }
    return g_servers[device];
}

std::recursive_mutex& lock(Server* s) { return s->mu; }

void quiesce(Server* s) {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    srv_quiesce(s);
}

static double* grow(double** p, size_t* cap, size_t n) {
    if (n <= *cap) return *p;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t c = std::max<size_t>(n, 4096);
    if (hipHostMalloc((void**)p, c * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
        return nullptr;
    *cap = c;
    return *p;
}

double* payload(Server* s, size_t n) { return grow(&s->pay, &s->pay_cap, n); }
double* result(Server* s, size_t n) { return grow(&s->res, &s->res_cap, n); }

const void* dev(Server* s, const void* host_ptr) {
    (void)s;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, const_cast<void*>(host_ptr), 0) != hipSuccess) return nullptr;
    return d;
}

int call(Server* s, int op, const void* args, size_t bytes, int groups, double* y, double* y2) {
    std::lock_guard<std::recursive_mutex> lk(s->mu);
    HZ_TRY_HIP(hipSetDevice(s->device));
    if (bytes > sizeof(long long) * kArgWords || groups < 1 || groups > kGroups) {
        hz::set_error("hz_rt::call: op arguments %zu bytes, %d workgroups", bytes, groups);
        return HZ_E_INVALID;
    }
    if (s->broken) {
        hz::set_error("hz_rt: the per-sample server stopped answering earlier; per-sample calls are off");
        return HZ_E_HIP;
    }
    if (!s->active || srv_left(s)) {
        s->active = false;
        HZ_TRY(srv_launch(s));
    }
    Req* q = s->req();
    Slot* slot = s->slot();
    q->op = op;
    q->groups = groups;
    std::memcpy(q->w, args, bytes);
    const long long want = ++s->seq;
    s->wc_fence();   // the arguments land before the request word
    __atomic_store_n(&q->req, (want << 4) | groups, __ATOMIC_RELEASE);
    s->wc_fence();   // and the request word leaves the write-combining buffer now
    const auto t0 = std::chrono::steady_clock::now();
    int relaunched = 0;
    for (;;) {
        bool all = true;
        for (int g = 0; g < groups && all; ++g) all = host_load(&slot[g].done) >= want;
        if (all) break;
        if (srv_left(s)) {
            // the instance left (idle) as the request arrived: the workgroups that had not served it
            // serve it after the relaunch (each resumes from its own response line)
            if (relaunched++ > 3) {
                s->broken = true;
                hz::set_error("hz_rt: the per-sample server left repeatedly without serving");
                return HZ_E_HIP;
            }
            HZ_TRY(srv_launch(s));
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(s->answer_ms)) {
            // the request stays posted: a late answer would advance a state the caller was told
            // did not move, so no later request may follow it
            s->broken = true;
            hz::set_error("hz_rt: the per-sample server did not answer within %lld ms", s->answer_ms);
            return HZ_E_HIP;
        }
    }
    double a = 0.0, b = 0.0;
    for (int g = 0; g < groups; ++g) {
        a += slot[g].y;
        b += slot[g].y2;
    }
    if (y) *y = a;
    if (y2) *y2 = b;
    ++s->requests;
    return HZ_OK;
}

void info(Server* s, long long* requests, long long* launches, int* active) {
    if (requests) *requests = s->requests;
    if (launches) *launches = s->launches;
    if (active) *active = (s->active && !srv_left(s)) ? 1 : 0;
}

}  // namespace hz_rt

extern "C" {

int hz_rt_info(int device, long long* requests, long long* launches, int* active) {
    hz_rt::Server* s = hz_rt::server(device);
    if (!s) return HZ_E_NODEV;
    hz_rt::info(s, requests, launches, active);
    return HZ_OK;
}

}  // extern "C"
