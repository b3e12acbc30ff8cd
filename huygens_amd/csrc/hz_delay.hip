// hz_delay.hip -- Delaybank<T,N>: N independent Delay<T> lines on MI355X (gfx950).
//
// Replaces src/delay.h:10-108 over src/buffer.h:9-86 (and defines the Delaybank that
// src/delaybank.h:15-54 only stubs).  Per line, per sample (delay.h:71-89):
//     in[o] = x;  out[o] = 0;
//     for i in taps: out[o] += f_i * in(d_i) - b_i * out(e_i);   y = out(0);  o = (o+1) % size
// with the ring read of buffer.h:40-47:  idx = (uint32)(o - c + size) % size, c = (int)(T)d.
//
// Exact indexing without a divide per tap: for o in [0, size) the uint32 expression wraps
// iff o < c - size, so a read at delay c has one of two AGES (o - idx mod size):
//     no wrap: c mod size,     wrap: (c - 2^32) mod size,
// resolved on the host into {thr = c - size, age_nowrap, age_wrap} per tap.  The slot
// idx = o - age then holds the sample of time t - age (or 0 before the first write).
//
// Time parallelism.  A feedback tap with gain != 0 and age a >= 1 makes sample t depend
// on sample t - a, so the call is cut into sub-blocks of Lc = min such age: inside a
// sub-block every sample is independent.  Reads whose source time lies in this call come
// straight from the call's input / output arrays; older ones from the rings, which are
// only written (committed) after the whole call -- so no slot is overwritten while a
// later sample of the call still needs its old value.  Age 0 on the feedback side is the
// reference's partial-sum read of the current slot and is the accumulator itself.
//
// Layout in HBM: rings [N][size] for input and output (T), taps [N][2S] int4 (forward
// then feedback) + gains [N][2S] T; line outputs [N][n] (line-major) and the mixdown [n].
//
// Numerics: the interpolated read's zero-weight neighbour term (data[idx-1] * 0) and the
// `* (1 - 0)` are elided; for finite ring contents they cannot change a result bit
// (tests/test_delay_gpu.py compares bit-for-bit with the restatement).  FP contraction
// is disabled in the kernel so every product and sum rounds as in the reference.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <new>
#include <vector>

#include "hz_chain.h"
#include "hz_common.h"
#include "hz_rt.h"

namespace {

constexpr int kThreads = 1024;

struct DlyArgs {
    const void* in;      // mono [n] or line-major [N][n]
    void* y;             // line outputs [N][n]
    const int4* taps;    // [N][2S] {thr, age_nowrap, age_wrap, 0}
    const void* gains;   // [N][2S] T
    void* ring_x;        // [N][size]
    void* ring_y;        // [N][size]
    long n, Lc;
    long k0, k1;         // sub-block range of this launch
    int S, in_per_line, commit;
    unsigned size, o0;
};

template <typename T>
__device__ __forceinline__ unsigned tap_age(const int4& q, unsigned o) {
    return ((int)o < q.x) ? (unsigned)q.z : (unsigned)q.y;
}

template <typename T, int kBatch>
__global__ __launch_bounds__(kThreads) void dly_line_kernel(DlyArgs a) {
#pragma clang fp contract(off)
    const int line = blockIdx.y;
    const int Gt = gridDim.x, g = blockIdx.x;
    const int S = a.S;
    const unsigned size = a.size;
    const int4* __restrict__ tp = a.taps + (long)line * 2 * S;
    const T* __restrict__ gn = (const T*)a.gains + (long)line * 2 * S;
    const T* __restrict__ xin = (const T*)a.in + (a.in_per_line ? (long)line * a.n : 0);
    T* yout = (T*)a.y + (long)line * a.n;
    T* rx = (T*)a.ring_x + (long)line * size;
    T* ry = (T*)a.ring_y + (long)line * size;

    for (long k = a.k0; k < a.k1; ++k) {
        const long s0 = k * a.Lc, s1 = min(a.n, s0 + a.Lc);
        const long per = (s1 - s0 + Gt - 1) / Gt;
        const long b0 = s0 + g * per, b1 = min(s1, b0 + per);
        // kBatch samples per thread: every read of a tap is issued before any store, so
        // the gathers of a batch overlap (the stores of this sub-block are never read in it)
        for (long base = b0; base < b1; base += (long)blockDim.x * kBatch) {
            long jj[kBatch];
            unsigned oo[kBatch];
            T acc[kBatch];
#pragma unroll
            for (int m = 0; m < kBatch; ++m) {
                jj[m] = min(base + threadIdx.x + (long)m * blockDim.x, b1 - 1);
                oo[m] = (a.o0 + (unsigned)jj[m]) % size;
                acc[m] = (T)0;
            }
            for (int i = 0; i < S; ++i) {
                const int4 qf = tp[i];
                const T f = gn[i];
                const T b = gn[S + i];
                T xv[kBatch], yv[kBatch];
#pragma unroll
                for (int m = 0; m < kBatch; ++m) {
                    const unsigned o = oo[m], af = tap_age<T>(qf, o);
                    const T* src = ((long)af <= jj[m]) ? xin + (jj[m] - af) : rx + (o >= af ? o - af : o + size - af);
                    xv[m] = *src;   // one branch-free gather: the pointer is selected, not the load
                    yv[m] = (T)0;
                }
                if (b != (T)0) {   // uniform over the workgroup (one line)
                    const int4 qb = tp[S + i];
#pragma unroll
                    for (int m = 0; m < kBatch; ++m) {
                        const unsigned o = oo[m], ab = tap_age<T>(qb, o);
                        const T* src = ((long)ab <= jj[m]) ? yout + (jj[m] - (long)(ab ? ab : 0))
                                                           : ry + (o >= ab ? o - ab : o + size - ab);
                        const T v = *src;   // age 0 reads yout[j] (stale); replaced by the partial sum
                        yv[m] = (ab == 0) ? acc[m] : v;
                    }
                }
#pragma unroll
                for (int m = 0; m < kBatch; ++m) {
                    const T fx = f * xv[m];
                    const T by = b * yv[m];
                    acc[m] = acc[m] + (fx - by);
                }
            }
#pragma unroll
            for (int m = 0; m < kBatch; ++m)
                if (base + threadIdx.x + (long)m * blockDim.x < b1) yout[jj[m]] = acc[m];
        }
        if (k + 1 < a.k1) __syncthreads();   // sub-block k visible to k+1 (same CU, same L1)
    }
    if (a.commit) {   // single-launch mode: one workgroup per line, all reads of the call done
        __syncthreads();
        const long j0 = a.n > (long)size ? a.n - (long)size : 0;
        for (long j = j0 + threadIdx.x; j < a.n; j += blockDim.x) {
            const unsigned slot = (unsigned)((a.o0 + (unsigned long)j) % size);
            rx[slot] = xin[j];
            ry[slot] = yout[j];
        }
    }
}

template <typename T>
__global__ __launch_bounds__(256) void dly_commit_kernel(DlyArgs a) {
    const int line = blockIdx.y;
    const unsigned size = a.size;
    const T* xin = (const T*)a.in + (a.in_per_line ? (long)line * a.n : 0);
    const T* yout = (const T*)a.y + (long)line * a.n;
    T* rx = (T*)a.ring_x + (long)line * size;
    T* ry = (T*)a.ring_y + (long)line * size;
    const long j0 = a.n > (long)size ? a.n - (long)size : 0;
    for (long j = j0 + (long)blockIdx.x * blockDim.x + threadIdx.x; j < a.n; j += (long)gridDim.x * blockDim.x) {
        const unsigned slot = (unsigned)((a.o0 + (unsigned long)j) % size);
        rx[slot] = xin[j];
        ry[slot] = yout[j];
    }
}

// mixdown (new in this build): sum of the line outputs in line order, in T, / N
template <typename T>
__global__ __launch_bounds__(256) void dly_mix_kernel(const T* __restrict__ y, long n, int N, T* __restrict__ out) {
#pragma clang fp contract(off)
    const long j = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    T s = (T)0;
    // the adds stay in line order; unrolling lets the loads of 16 lines issue together
    // (a 1024-sample streaming block is only 4 workgroups: latency, not bandwidth)
#pragma unroll 16
    for (int l = 0; l < N; ++l) s = s + y[(long)l * n + j];
    out[j] = s / (T)N;
}

}  // namespace

struct hz_dly {
    int N = 0, S = 0, is_float = 0, device = 0;
    unsigned size = 1, origin = 0;
    std::vector<unsigned> ft, bt;   // [N][S] delay times as given
    std::vector<double> fg, bg;     // [N][S] gains, rounded to T
    bool dirty = true;
    long Lc = 0;                    // sub-block length (<= 0: unbounded)
    int split = 0;                  // 0 auto, 1 one workgroup per line, 2 launch per sub-block
    int target_groups = 256;
    int4* d_taps = nullptr;
    void *d_gains = nullptr, *d_rx = nullptr, *d_ry = nullptr;
    void *d_y = nullptr, *d_in = nullptr, *d_out = nullptr;
    size_t y_cap = 0, in_cap = 0, out_cap = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool prof = false;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    long launches = 0;
    bool pending = false;           // block work queued on the stream since the last synchronisation
    size_t elem() const { return is_float ? sizeof(float) : sizeof(double); }
};

namespace {

int dly_check(hz_dly* h) {
    if (!h) {
        hz::set_error("null hz_dly handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    return HZ_OK;
}

// c = (int)(T)d  (buffer.h:42 with the uint delay converted to T by the call in delay.h:82-83)
long eff_center(const hz_dly* h, unsigned d) {
    return h->is_float ? (long)(int)(float)d : (long)(int)(double)d;
}

// {thr, age_nowrap, age_wrap} of a read at delay d for ring size `size` (see header)
int4 resolve_tap(const hz_dly* h, unsigned d) {
    const long c = eff_center(h, d), size = (long)h->size;
    const long thr = c - size;
    const long anw = ((c % size) + size) % size;
    const long aw = (((c - 4294967296L) % size) + size) % size;
    int4 q;
    q.x = (int)std::max<long>(std::min<long>(thr, 0x7fffffffL), -0x7fffffffL);
    q.y = (int)anw;
    q.z = (int)aw;
    q.w = 0;
    return q;
}

int dly_upload(hz_dly* h) {
    if (!h->dirty) return HZ_OK;
    const int N = h->N, S = h->S;
    std::vector<int4> taps((size_t)N * 2 * S);
    std::vector<double> gd((size_t)N * 2 * S);
    std::vector<float> gf((size_t)N * 2 * S);
    long Lc = -1;
    for (int l = 0; l < N; ++l)
        for (int i = 0; i < S; ++i) {
            const size_t ti = (size_t)l * S + i;
            const size_t o = (size_t)l * 2 * S;
            taps[o + i] = resolve_tap(h, h->ft[ti]);
            taps[o + S + i] = resolve_tap(h, h->bt[ti]);
            gd[o + i] = h->fg[ti];
            gd[o + S + i] = h->bg[ti];
            gf[o + i] = (float)h->fg[ti];
            gf[o + S + i] = (float)h->bg[ti];
            if (h->bg[ti] != 0.0) {   // ages of a live feedback read bound the sub-block
                const int4 q = taps[o + S + i];
                if (q.y > 0) Lc = (Lc < 0) ? q.y : std::min<long>(Lc, q.y);
                if (q.x > 0 && q.z > 0) Lc = (Lc < 0) ? q.z : std::min<long>(Lc, q.z);
            }
        }
    h->Lc = Lc;
    HZ_TRY_HIP(hipMemcpyAsync(h->d_taps, taps.data(), sizeof(int4) * taps.size(), hipMemcpyHostToDevice, h->stream));
    if (h->is_float)
        HZ_TRY_HIP(hipMemcpyAsync(h->d_gains, gf.data(), sizeof(float) * gf.size(), hipMemcpyHostToDevice, h->stream));
    else
        HZ_TRY_HIP(hipMemcpyAsync(h->d_gains, gd.data(), sizeof(double) * gd.size(), hipMemcpyHostToDevice, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));   // host vectors go out of scope
    h->dirty = false;
    return HZ_OK;
}

int ensure(void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return HZ_OK;
    if (*p) HZ_TRY_HIP(hipFree(*p));
    *p = nullptr;
    HZ_TRY_HIP(hipMalloc(p, bytes));
    *cap = bytes;
    return HZ_OK;
}

template <typename T>
int dly_launch_t(hz_dly* h, const void* d_in, void* d_out, long n, int in_per_line, int mix) {
    const int N = h->N;
    void* y = d_out;
    if (mix) {
        HZ_TRY(ensure(&h->d_y, &h->y_cap, sizeof(T) * (size_t)N * n));
        y = h->d_y;
    }
    const long Lc = (h->Lc > 0) ? std::min<long>(h->Lc, n) : n;
    const long nsub = (n + Lc - 1) / Lc;
    // workgroups per line in per-sub-block mode
    const long gt_max = std::max<long>(1, std::min<long>((Lc + kThreads - 1) / kThreads,
                                                         (2L * h->target_groups + N - 1) / N));
    int mode = h->split;
    // auto: several workgroups per line (a launch per sub-block) unless the lines alone fill
    // the chip; measured 2x faster for C5's 64 lines x 480k samples (bench c5 split table)
    if (mode == 0) mode = (gt_max > 1 && (nsub <= 8 || N < h->target_groups)) ? 2 : 1;
    if (mode == 2 && gt_max == 1) mode = 1;

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
    DlyArgs a;
    a.in = d_in;
    a.y = y;
    a.taps = h->d_taps;
    a.gains = h->d_gains;
    a.ring_x = h->d_rx;
    a.ring_y = h->d_ry;
    a.n = n;
    a.Lc = Lc;
    a.S = h->S;
    a.in_per_line = in_per_line;
    a.size = h->size;
    a.o0 = h->origin;
    // samples per thread per pass: 8 when a workgroup's slice of a sub-block is long
    const long slice = (mode == 1) ? Lc : (Lc + gt_max - 1) / gt_max;
    auto kern = slice >= 4L * kThreads ? dly_line_kernel<T, 8> : (slice > kThreads ? dly_line_kernel<T, 2> : dly_line_kernel<T, 1>);
    if (mode == 1) {
        a.k0 = 0;
        a.k1 = nsub;
        a.commit = 1;
        hipLaunchKernelGGL(kern, dim3(1, N), dim3(kThreads), 0, h->stream, a);
        HZ_TRY_HIP(hipGetLastError());
    } else {
        a.commit = 0;
        for (long k = 0; k < nsub; ++k) {
            a.k0 = k;
            a.k1 = k + 1;
            hipLaunchKernelGGL(kern, dim3((unsigned)gt_max, N), dim3(kThreads), 0, h->stream, a);
            HZ_TRY_HIP(hipGetLastError());
        }
        const long span = std::min<long>(n, (long)h->size);
        const unsigned gx = (unsigned)std::max<long>(1, std::min<long>((span + 255) / 256, 64));
        hipLaunchKernelGGL(dly_commit_kernel<T>, dim3(gx, N), dim3(256), 0, h->stream, a);
        HZ_TRY_HIP(hipGetLastError());
    }
    if (e) HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
    if (mix) {
        hipLaunchKernelGGL(dly_mix_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->stream,
                           (const T*)y, n, N, (T*)d_out);
        HZ_TRY_HIP(hipGetLastError());
    }
    h->origin = (unsigned)(((unsigned long)h->origin + (unsigned long)n) % h->size);
    h->launches += h->prof ? 1 : 0;
    h->pending = true;
    return HZ_OK;
}

int dly_launch(hz_dly* h, const void* d_in, void* d_out, long n, int in_per_line, int mix) {
    if (n <= 0) return HZ_OK;
    if (n >= (1L << 31)) {
        hz::set_error("hz_dly_process: n must be < 2^31 per call");
        return HZ_E_INVALID;
    }
    HZ_TRY(dly_upload(h));
    return h->is_float ? dly_launch_t<float>(h, d_in, d_out, n, in_per_line, mix)
                       : dly_launch_t<double>(h, d_in, d_out, n, in_per_line, mix);
}

int set_tap(hz_dly* h, int line, int back, unsigned i, unsigned t, double g) {
    const double lim = h->is_float ? 2147483520.0 : 2147483647.0;   // (int)(T)t defined
    if ((double)t > lim) {
        hz::set_error("delay time %u exceeds the int range of Buffer::operator() (buffer.h:42)", t);
        return HZ_E_INVALID;
    }
    if (back && t == 0) g = 0.0, t = 0;   // zero-time feedback -> {0, 0} (delay.h:48-51, 64-67)
    if (h->is_float) g = (double)(float)g;
    const size_t k = (size_t)line * h->S + i;
    (back ? h->bt : h->ft)[k] = t;
    (back ? h->bg : h->fg)[k] = g;
    h->dirty = true;
    return HZ_OK;
}

}  // namespace

namespace hz_chain {

int dly_block_begin(hz_dly* h, long n, DlyBlock* b, bool* fusable) {
    *fusable = false;
    HZ_TRY(dly_check(h));
    HZ_TRY(dly_upload(h));
    b->taps = h->d_taps;
    b->gains = (const float*)h->d_gains;
    b->rx = (float*)h->d_rx;
    b->ry = (float*)h->d_ry;
    b->size = h->size;
    b->o0 = h->origin;
    b->N = h->N;
    b->S = h->S;
    b->stream = h->stream;
    if (!h->is_float || h->S > kMaxTaps || n <= 0 || 2 * n > (long)h->size) return HZ_OK;
    // every read of the block: the current sample, or a ring slot written before the call that no
    // sample of the call overwrites (a read at age a from sample j hits slot o0 + j - a)
    auto ok = [&](long a) { return a == 0 || (a >= n && a <= (long)h->size - n); };
    for (int l = 0; l < h->N; ++l)
        for (int i = 0; i < h->S; ++i)
            for (int back = 0; back < 2; ++back) {
                const size_t ti = (size_t)l * h->S + i;
                if (back && h->bg[ti] == 0.0) continue;   // the kernel skips zero feedback gains
                const int4 q = resolve_tap(h, back ? h->bt[ti] : h->ft[ti]);
                if (!ok(q.y) || (q.x > 0 && !ok(q.z))) return HZ_OK;
            }
    *fusable = true;
    return HZ_OK;
}

void dly_block_end(hz_dly* h, long n) {
    h->origin = (unsigned)(((unsigned long)h->origin + (unsigned long)n) % h->size);
    h->pending = true;
}

}  // namespace hz_chain

extern "C" {

int hz_dly_create(int lines, unsigned sparsity, unsigned time, int is_float, int device, hz_dly** out) {
    if (!out || lines <= 0 || sparsity == 0 || sparsity > 4096 || time >= 0x7fffffffu) {
        hz::set_error("hz_dly_create: invalid arguments");
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_dly* h = new (std::nothrow) hz_dly();
    if (!h) return HZ_E_ALLOC;
    h->N = lines;
    h->S = (int)sparsity;
    h->is_float = is_float ? 1 : 0;
    h->device = device;
    h->size = time + 1u;   // Delay(sparsity, time) : input(time + 1), output(time + 1)
    h->ft.assign((size_t)lines * sparsity, 0u);
    h->bt.assign((size_t)lines * sparsity, 0u);
    h->fg.assign((size_t)lines * sparsity, 0.0);
    h->bg.assign((size_t)lines * sparsity, 0.0);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        h->target_groups = prop.multiProcessorCount;
    const size_t ring = h->elem() * (size_t)lines * h->size;
    bool ok = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) == hipSuccess;
    ok = ok && hipMalloc(&h->d_taps, sizeof(int4) * (size_t)lines * 2 * sparsity) == hipSuccess;
    ok = ok && hipMalloc(&h->d_gains, h->elem() * (size_t)lines * 2 * sparsity) == hipSuccess;
    ok = ok && hipMalloc(&h->d_rx, ring) == hipSuccess && hipMalloc(&h->d_ry, ring) == hipSuccess;
    ok = ok && hipMemsetAsync(h->d_rx, 0, ring, h->stream) == hipSuccess;   // Buffer: zeroed
    ok = ok && hipMemsetAsync(h->d_ry, 0, ring, h->stream) == hipSuccess;
    ok = ok && hipStreamSynchronize(h->stream) == hipSuccess;
    if (!ok) {
        hz::set_error("hz_dly_create: device allocation failed (%zu bytes of rings)", 2 * ring);
        if (h->stream) (void)hipStreamDestroy(h->stream);
        for (void* p : {(void*)h->d_taps, h->d_gains, h->d_rx, h->d_ry})
            if (p) (void)hipFree(p);
        delete h;
        return HZ_E_ALLOC;
    }
    h->own_stream = true;
    *out = h;
    return HZ_OK;
}

int hz_dly_destroy(hz_dly* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (void* p : {(void*)h->d_taps, h->d_gains, h->d_rx, h->d_ry, h->d_y, h->d_in, h->d_out})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_dly_coefficients(hz_dly* h, int line, const unsigned* ft, const double* fg, int nf, const unsigned* bt,
                        const double* bg, int nb) {   // delay.h:37-56
    if (!h || line < 0 || line >= h->N || nf < 0 || nb < 0 || (nf && (!ft || !fg)) || (nb && (!bt || !bg))) {
        hz::set_error("hz_dly_coefficients: invalid arguments");
        return HZ_E_INVALID;
    }
    for (int i = 0; i < h->S; ++i) {
        HZ_TRY(i < nf ? set_tap(h, line, 0, i, ft[i], fg[i]) : set_tap(h, line, 0, i, 0, 0.0));
        HZ_TRY(i < nb ? set_tap(h, line, 1, i, bt[i], bg[i]) : set_tap(h, line, 1, i, 0, 0.0));
    }
    return HZ_OK;
}

int hz_dly_modulate_forward(hz_dly* h, int line, unsigned n, unsigned t, double g) {   // delay.h:59-60
    if (!h || line < 0 || line >= h->N || n >= (unsigned)h->S) {
        hz::set_error("hz_dly_modulate_forward: invalid arguments");
        return HZ_E_INVALID;
    }
    return set_tap(h, line, 0, n, t, g);
}

int hz_dly_modulate_back(hz_dly* h, int line, unsigned n, unsigned t, double g) {   // delay.h:63-68
    if (!h || line < 0 || line >= h->N || n >= (unsigned)h->S) {
        hz::set_error("hz_dly_modulate_back: invalid arguments");
        return HZ_E_INVALID;
    }
    return set_tap(h, line, 1, n, t, g);
}

int hz_dly_process_device(hz_dly* h, const void* d_in, void* d_out, size_t n, int in_per_line, int mix) {
    HZ_TRY(dly_check(h));
    if (n && (!d_in || !d_out)) return HZ_E_INVALID;
    return dly_launch(h, d_in, d_out, (long)n, in_per_line, mix);
}

int hz_dly_process(hz_dly* h, const void* in, void* out, size_t n, int in_per_line, int mix) {
    HZ_TRY(dly_check(h));
    if (n == 0) return HZ_OK;
    if (!in || !out) return HZ_E_INVALID;
    const size_t in_bytes = h->elem() * n * (in_per_line ? h->N : 1);
    const size_t out_bytes = h->elem() * n * (mix ? 1 : h->N);
    HZ_TRY(ensure(&h->d_in, &h->in_cap, in_bytes));
    HZ_TRY(ensure(&h->d_out, &h->out_cap, out_bytes));
    HZ_TRY_HIP(hipMemcpyAsync(h->d_in, in, in_bytes, hipMemcpyHostToDevice, h->stream));
    HZ_TRY(dly_launch(h, h->d_in, h->d_out, (long)n, in_per_line, mix));
    HZ_TRY_HIP(hipMemcpyAsync(out, h->d_out, out_bytes, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

// one sample of every line through the device's per-sample server (hz_rt.hip OP_DLY): the
// reference's `y = D(x); D.tick();` (tests/delay.cpp:20-28) without a launch per sample; in: one
// T (mono) or N T (per line); out: N T
int hz_dly_sample(hz_dly* h, const void* in, void* out, int in_per_line) {
    HZ_TRY(dly_check(h));
    if (!in || !out) return HZ_E_INVALID;
    HZ_TRY(dly_upload(h));
    if (h->pending) {   // block calls' ring updates land before the server reads the rings
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        h->pending = false;
    }
    hz_rt::Server* srv = hz_rt::server(h->device);
    if (!srv) return HZ_E_NODEV;
    std::lock_guard<std::recursive_mutex> lk(hz_rt::lock(srv));
    const int N = h->N;
    double* res = hz_rt::result(srv, N);
    double* pay = in_per_line ? hz_rt::payload(srv, N) : nullptr;
    if (!res || (in_per_line && !pay)) return HZ_E_ALLOC;
    hz_rt::DlyArgs a{};
    a.rx = h->d_rx;
    a.ry = h->d_ry;
    a.taps = h->d_taps;
    a.gains = h->d_gains;
    if (in_per_line) {
        for (int l = 0; l < N; ++l) pay[l] = h->is_float ? (double)((const float*)in)[l] : ((const double*)in)[l];
        a.xin = (const double*)hz_rt::dev(srv, pay);
    } else {
        a.x = h->is_float ? (double)*(const float*)in : *(const double*)in;
    }
    a.out = (double*)hz_rt::dev(srv, res);
    a.N = N;
    a.S = h->S;
    a.is_float = h->is_float;
    a.size = h->size;
    a.o = h->origin;
    const int groups = std::max(1, std::min(hz_rt::kGroups, (N + hz_rt::kThreads - 1) / hz_rt::kThreads));
    HZ_TRY(hz_rt::call(srv, hz_rt::OP_DLY, &a, sizeof(a), groups, nullptr));
    for (int l = 0; l < N; ++l) {
        if (h->is_float) ((float*)out)[l] = (float)res[l];
        else ((double*)out)[l] = res[l];
    }
    h->origin = (unsigned)(((unsigned long)h->origin + 1ul) % h->size);
    return HZ_OK;
}

// Buffer::tick of both rings without a sample (delay.h:92-97 after no operator()): the origins
// move, nothing is written, so the slots keep the samples of `size` ticks earlier -- later reads
// see exactly those stale values, as in the reference (every read goes through the rings across
// calls; the rings are committed at each call's end)
int hz_dly_tick(hz_dly* h, unsigned long count) {
    HZ_TRY(dly_check(h));
    h->origin = (unsigned)(((unsigned long)h->origin + count % h->size) % h->size);
    return HZ_OK;
}

int hz_dly_origin(hz_dly* h, unsigned* origin) {
    if (!h || !origin) return HZ_E_INVALID;
    *origin = h->origin;
    return HZ_OK;
}

int hz_dly_info(hz_dly* h, long* chunk, unsigned* size) {
    if (!h) return HZ_E_INVALID;
    HZ_TRY(dly_check(h));
    HZ_TRY(dly_upload(h));
    if (chunk) *chunk = h->Lc;
    if (size) *size = h->size;
    return HZ_OK;
}

int hz_dly_set_split(hz_dly* h, int mode) {
    if (!h || mode < 0 || mode > 2) return HZ_E_INVALID;
    h->split = mode;
    return HZ_OK;
}

int hz_dly_set_stream(hz_dly* h, void* stream) {
    HZ_TRY(dly_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) HZ_TRY_HIP(hipStreamDestroy(h->stream));
    h->stream = (hipStream_t)stream;
    h->own_stream = false;
    return HZ_OK;
}

int hz_dly_synchronize(hz_dly* h) {
    HZ_TRY(dly_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_dly_set_target_groups(hz_dly* h, int groups) {
    if (!h || groups <= 0) return HZ_E_INVALID;
    h->target_groups = groups;
    return HZ_OK;
}

int hz_dly_profile(hz_dly* h, int enable) {
    HZ_TRY(dly_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    h->prof = enable != 0;
    h->ev_used = 0;
    h->launches = 0;
    return HZ_OK;
}

int hz_dly_profile_read(hz_dly* h, double* ms, long* launches) {
    HZ_TRY(dly_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    double tot = 0.0;
    for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
        float t = 0.f;
        HZ_TRY_HIP(hipEventElapsedTime(&t, h->ev[i], h->ev[i + 1]));
        tot += t;
    }
    if (ms) *ms = tot;
    if (launches) *launches = h->launches;
    h->ev_used = 0;
    h->launches = 0;
    return HZ_OK;
}

}  // extern "C"
