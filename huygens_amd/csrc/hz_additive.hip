// hz_additive.hip -- Additive<double> and Sinusoids<double> banks for MI355X (gfx950).
//
// Both are banks of Oscillator<T> phase accumulators (src/oscillator.h:27-38) mixed
// through cycle(p) = sin(2 PI p) (src/wave.h:147):
//   Additive  (src/additive.h:38-62):  out = sum_v [amp_v != 0] sum_j amp_v decay^j
//             sin(2 PI phi_vj) / (V norm);  tick: amp_v <- (1-a) active_v + a amp_v, then
//             for voices with active_v || amp_v: freqmod(mtof(position_vj)); Oscillator::tick()
//   Sinusoids (src/sinusoids.h:34-57): out = sum_i decay^i sin(2 PI phi_i) / norm
//
// Oscillator::tick advances phase by f/SR and relaxes f toward its target with stiffness s:
//   phi(t) = phi0 + A t + D (1 - s^t),   A = f_target/SR,  D = (f0 - f_target)/((1-s) SR)
// (phase and target_phase stay equal without phasemod, so the pull term is the identity).
// The engine evaluates that closed form:
//   * lanes are TIME (16-sample chunks of a 1024-sample tile); a wave owns a slice of one
//     voice's overtones, accumulates sum_j c_j sin(...) per sample in registers, then
//     multiplies by the voice envelope amp(t) = act + a^t (amp0 - act) (closed-form seed,
//     one-pole recurrence inside the chunk);
//   * chunks where the frequency transient still moves the phase (|D| s^t > 2^-60) are
//     evaluated per sample (sincospi); all others seed a phasor by w = e^{2 pi i A} per
//     16-sample chunk (seed = z(t0) (w^16)^p (w^256)^r from per-partial tables,
//     z(t0+1024) = z(t0) w^1024) and run the two-term sine recurrence inside the chunk;
//   * time segments need no carry (closed form), so small banks still fill the chip;
//   * a wave takes tpw tasks in turn (the envelope applied per task); the waves' mixes are summed
//     through LDS and written once per workgroup: straight to the output when one group of
//     workgroups covers every task (long calls), else as group rows a second kernel sums.
// PI: the reference's truncated PI enters only through sin(2 PI frac(phi)); using 2 pi
// changes the argument by <= 4.2e-13 rad.
#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "hz_common.h"

namespace {

constexpr int kL = 32;   // samples per lane chunk (16: 1.28 ms per C3 launch; 32 halves the per-chunk
                         // seed / table / transient-check work per sample)
constexpr int kTile = 64 * kL;
constexpr int kWaves = 8;
constexpr int kMaxPerWave = 64;
constexpr int kPad = 66;

// per-partial record (depends only on the target frequency and the output weight):
// A = f_target/SR (cycles/sample), c (output weight), W1 = e^{2 pi i A},
// T1[p] = W1^(kL p) (p < 16), T2[r] = W1^(16 kL r) (r < 4), WT = W1^(64 kL)
struct PRec {
    static constexpr int A = 0, C = 1;
    static constexpr int W1 = 2;
    static constexpr int T1 = 4;
    static constexpr int T2 = T1 + 32;
    static constexpr int WT = T2 + 8;
    static constexpr int SIZE = 48;
};

// one wave task: a slice of one voice's partials
struct Task {
    int first;   // first partial (local index)
    int count;   // partials in the slice
    int voice;   // voice slot (amp arrays)
    int pad;
};

struct AddArgs {
    const Task* tasks;
    const double* phi;     // [P] oscillator phase at call start
    const double* f;       // [P] oscillator frequency at call start
    const double* ft;      // [P] target frequency
    const double* amp0;    // [V] envelope value at call start
    const double* act;     // [V] envelope target (Minimizer::active)
    const double* c0;      // [P] output weights of the call's first sample, or null when
                           // equal to the records' (Sinusoids::operator() runs before tick()
                           // applies a decaymod, sinusoids.h:34-57)
    double* partial;       // [G][n_pad]: one row per group (G > 1), or the output itself (G == 1)
    double scale;          // (G == 1) the output scale, applied here
    long n, n_pad, seg_len;
    int ntasks, nseg;
    int tpw;               // tasks per wave: workgroup g's wave w takes tasks (g tpw + k) kWaves + w
    double a;              // attack smoothing coefficient
    double s;              // oscillator stiffness
};

__device__ __forceinline__ void cmul(double ar, double ai, double br, double bi, double& cr, double& ci) {
    const double r = fma(ar, br, -ai * bi);
    const double i = fma(ar, bi, ai * br);
    cr = r;
    ci = i;
}

// lane q's double (q uniform)
__device__ __forceinline__ double lane_d(double v, int q) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffff), q);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), q);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}

// frac(phi0 + A t + D (1 - s^t)) with the A t product kept exact (fma residual)
__device__ __forceinline__ double phase_at(double phi0, double A, double D, double s, double t, double st) {
    const double p = A * t;
    const double e = fma(A, t, -p);
    double q = p - floor(p);
    q += phi0 + e + D * (1.0 - st);
    return q - floor(q);
}

// kL samples of one partial in its frequency transient, exact closed form per sample, added to
// the LDS column `col` (stride kPad); out of line so sinpi's registers stay out of the main loop
// (scaled by the voice envelope amp(t), advanced per sample as in the mix)
__device__ __attribute__((noinline)) void add_transient(double* col, double phi0, double A, double c, double D,
                                                        double s, long tc, double st, double amp, double ea,
                                                        double act) {
    for (int j = 0; j < kL; ++j) {
        const double ph = phase_at(phi0, A, D, s, (double)(tc + j), st);
        col[j * kPad] = fma(amp, c * sinpi(2.0 * ph), col[j * kPad]);
        st *= s;
        amp = fma(ea, amp, (1.0 - ea) * act);
    }
}

__global__ __launch_bounds__(64 * kWaves) void add_mix_kernel(const double* __restrict__ rec, AddArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* part = lds;                           // [W][kL][kPad] the waves' mix rows
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p16 = lane & 15, r4 = lane >> 4;
    const int seg = blockIdx.y;
    const long seg_t0 = (long)seg * a.seg_len;
    const long seg_end = min(seg_t0 + a.seg_len, a.n);
    const int ntiles = (int)((seg_end - seg_t0 + kTile - 1) / kTile);
    const double a_lane = pow(a.a, (double)(kL * lane));
    double a_t = seg_t0 ? pow(a.a, (double)seg_t0) : 1.0;
    const double inv_trans = 1.0 / ((1.0 - a.s) * hz::kSR);
    double* my = part + wave * (kL * kPad);

    for (int tile = 0; tile < ntiles; ++tile) {
        const long t0 = seg_t0 + (long)tile * kTile;
        const long tc = t0 + (long)kL * lane;
        const double s_tc = pow(a.s, (double)tc);  // transient decay at this chunk
        // the wave's mix of the tile accumulates in its LDS rows (registers hold one task's)
#pragma unroll
        for (int j = 0; j < kL; ++j) my[j * kPad + lane] = 0.0;
        for (int k = 0; k < a.tpw; ++k) {
            const int task = (blockIdx.x * a.tpw + k) * kWaves + wave;
            if (task >= a.ntasks) break;
            const Task tk = a.tasks[task];
            const double amp0 = a.amp0[tk.voice], act = a.act[tk.voice];
            // tile-start phasor of partial `lane` of the task (lanes in parallel; read below with
            // readlane; transient taken as complete -- chunks where it is not are evaluated per sample)
            double zr0 = 0.0, zi0 = 0.0;
            if (lane < tk.count) {
                const int pi = tk.first + lane;
                const double* rr = rec + (long)pi * PRec::SIZE;
                const double D = (a.f[pi] - a.ft[pi]) * inv_trans;
                const double ph = phase_at(a.phi[pi], rr[PRec::A], D, a.s, (double)t0, 0.0);
                sincospi(2.0 * ph, &zi0, &zr0);
            }
            double acc[kL];
#pragma unroll
            for (int j = 0; j < kL; ++j) acc[j] = 0.0;
            bool trans = false;
            // the next partial's record and frequency pair are fetched one iteration ahead (their
            // global latency runs under this partial's recurrence)
            struct Fetch {
                double c, D, t1r, t1i, t2r, t2i, w1r, w1i;
            };
            auto fetch = [&](int q, Fetch& p) {
                const int pi = tk.first + q;
                const double* rr = rec + (long)pi * PRec::SIZE;
                p.c = rr[PRec::C];
                p.D = (a.f[pi] - a.ft[pi]) * inv_trans;
                p.t1r = rr[PRec::T1 + 2 * p16];
                p.t1i = rr[PRec::T1 + 2 * p16 + 1];
                p.t2r = rr[PRec::T2 + 2 * r4];
                p.t2i = rr[PRec::T2 + 2 * r4 + 1];
                p.w1r = rr[PRec::W1];
                p.w1i = rr[PRec::W1 + 1];
            };
            Fetch cur;
            if (tk.count) fetch(0, cur);
            for (int q = 0; q < tk.count; ++q) {
                const int pi = tk.first + q;
                Fetch nxt;
                if (q + 1 < tk.count) fetch(q + 1, nxt);
                const double c = cur.c, D = cur.D;
                const double sr = lane_d(zr0, q), si = lane_d(zi0, q);
                if (a.c0 && tc == 0) acc[0] = fma(a.c0[pi] - c, sinpi(2.0 * a.phi[pi]), acc[0]);
                if (fabs(D) * s_tc > 0x1p-60) {
                    trans = true;   // frequency transient: the second pass below
                } else {
                    // seed z(tc) = z(t0) w^(kL p) w^(16 kL r); inside the chunk the sines follow the
                    // two-term recurrence sin((k+1) th) = 2 cos th sin(k th) - sin((k-1) th): one
                    // FMA per sample instead of a complex multiply (4), re-seeded every kL samples
                    // (error <= kL eps / |sin th| of the partial's amplitude)
                    double ur, ui, zr, zi;
                    cmul(cur.t1r, cur.t1i, cur.t2r, cur.t2i, ur, ui);
                    cmul(sr, si, ur, ui, zr, zi);
                    const double w1r = cur.w1r, w1i = cur.w1i;
                    const double c2 = 2.0 * w1r;
                    double s0 = zi, s1 = fma(zr, w1i, zi * w1r);
                    acc[0] = fma(c, s0, acc[0]);
                    acc[1] = fma(c, s1, acc[1]);
#pragma unroll
                    for (int j = 2; j < kL; ++j) {
                        const double s2 = fma(c2, s1, -s0);
                        acc[j] = fma(c, s2, acc[j]);
                        s0 = s1;
                        s1 = s2;
                    }
                }
                cur = nxt;
            }
            // voice envelope amp(t) = act + a^t (amp0 - act), advanced per sample
            double amp = act + (a_lane * a_t) * (amp0 - act);
            // the settled partials, then (chunks still inside a frequency transient: the first tiles
            // of a retune) the exact closed form per sample, out of line so sinpi's registers do not
            // spill the accumulators
            const double amp_c = amp;
#pragma unroll
            for (int j = 0; j < kL; ++j) {
                my[j * kPad + lane] = fma(amp, acc[j], my[j * kPad + lane]);
                amp = fma(a.a, amp, (1.0 - a.a) * act);
            }
            if (__builtin_amdgcn_ballot_w64(trans) != 0) {
                for (int q = 0; q < tk.count; ++q) {
                    const int pi = tk.first + q;
                    const double* rr = rec + (long)pi * PRec::SIZE;
                    const double D = (a.f[pi] - a.ft[pi]) * inv_trans;
                    if (fabs(D) * s_tc > 0x1p-60)
                        add_transient(my + lane, a.phi[pi], rr[PRec::A], rr[PRec::C], D, a.s, tc, s_tc, amp_c, a.a, act);
                }
            }
        }
        __syncthreads();
        const bool direct = gridDim.x == 1;   // one group: the output itself, scaled
        for (int tl = threadIdx.x; tl < kTile; tl += blockDim.x) {
            const int src = tl / kL, j = tl % kL;
            double s0 = 0.0;
#pragma unroll
            for (int w = 0; w < kWaves; ++w) s0 += part[w * (kL * kPad) + j * kPad + src];
            const long t = t0 + tl;
            if (t < a.n) {
                if (direct) a.partial[t] = s0 * a.scale;
                else a.partial[(long)blockIdx.x * a.n_pad + t] = s0;
            }
        }
        __syncthreads();
        a_t *= pow(a.a, (double)kTile);
    }
}

__global__ __launch_bounds__(256) void add_reduce_kernel(const double* __restrict__ partial, long n_pad, int G,
                                                         long n, double scale, double* __restrict__ out) {
    __shared__ double red[4][64];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const long t = (long)blockIdx.x * 64 + tx;
    double s = 0.0;
    if (t < n)
        for (int g = ty; g < G; g += 4) s += partial[(long)g * n_pad + t];
    red[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && t < n) out[t] = ((red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx])) * scale;
}

// end-of-call oscillator state for the partials of alive voices:
//   phi <- phi(n), f <- ft + s^n (f0 - ft)
__global__ __launch_bounds__(64) void add_advance_kernel(const double* __restrict__ rec, const Task* tasks,
                                                         int ntasks, long n, double s, double s_n,
                                                         const double* __restrict__ ft, double* phi, double* f) {
    const int task = blockIdx.x;
    if (task >= ntasks) return;
    const Task tk = tasks[task];
    const double inv_trans = 1.0 / ((1.0 - s) * hz::kSR);
    for (int q = threadIdx.x; q < tk.count; q += blockDim.x) {
        const int p = tk.first + q;
        const double* rr = rec + (long)p * PRec::SIZE;
        const double D = (f[p] - ft[p]) * inv_trans;
        phi[p] = phase_at(phi[p], rr[PRec::A], D, s, (double)n, s_n);
        f[p] = ft[p] + s_n * (f[p] - ft[p]);
    }
}

void fill_tables(double A, double* rec) {
    using C = std::complex<long double>;
    const long double th = 2.0L * 3.141592653589793238462643383279502884L * (long double)A;
    const C w(std::cos(th), std::sin(th));
    rec[PRec::W1] = (double)w.real();
    rec[PRec::W1 + 1] = (double)w.imag();
    C wl(1, 0);
    for (int k = 0; k < kL; ++k) wl *= w;
    C acc(1, 0);
    for (int p = 0; p < 16; ++p) {
        rec[PRec::T1 + 2 * p] = (double)acc.real();
        rec[PRec::T1 + 2 * p + 1] = (double)acc.imag();
        acc *= wl;
    }
    const C w256 = acc;   // W1^(16 kL)
    acc = C(1, 0);
    for (int r = 0; r < 4; ++r) {
        rec[PRec::T2 + 2 * r] = (double)acc.real();
        rec[PRec::T2 + 2 * r + 1] = (double)acc.imag();
        acc *= w256;
    }
    rec[PRec::WT] = (double)acc.real();
    rec[PRec::WT + 1] = (double)acc.imag();
}

long double mtofl(long double m) { return 440.0L * powl(2.0L, (m - 69) / 12); }

}  // namespace

// ---------------------------------------------------------------------------
// shared engine: V voices x OL local overtones (overtones [o0, o0 + OL) of O)
// ---------------------------------------------------------------------------
struct PhaseBank {
    int V = 1, O = 1, o0 = 0, OL = 1, device = 0;
    double s = 0;      // oscillator stiffness
    double a = 0;      // envelope smoothing (Additive attack); 0 for Sinusoids
    std::vector<double> ft;      // [V*OL] target frequency (Hz)
    std::vector<double> c;       // [V*OL] output weight
    std::vector<double> c_first; // weights of the next call's first sample
    double* d_c0 = nullptr;
    std::vector<double> amp, act;
    std::vector<char> alive;
    double scale = 1.0;
    // device
    double *d_rec = nullptr, *d_phi = nullptr, *d_f = nullptr, *d_ft = nullptr, *d_amp = nullptr,
           *d_act = nullptr, *d_partial = nullptr, *d_out = nullptr;
    Task* d_tasks = nullptr;
    size_t partial_cap = 0, out_cap = 0, task_cap = 0;
    std::vector<double> h_rec;
    std::vector<char> dirty;     // per voice: records need rebuilding
    std::vector<Task> tasks;
    int target_groups = 256;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    bool prof = false;
    std::vector<hipEvent_t> ev;
    size_t ev_used = 0;
    long launches = 0;
    // Per-sample calls (operator() / tick(): fills shorter than kLookMin) are served from a
    // speculative block: the next kLook samples rendered at once from a snapshot of the state
    // (the outputs need no input: src/additive.h:38-62, src/sinusoids.h:34-57), consumed one by
    // one; a setter or a longer fill first rolls the engine back to the consumed position
    // (snapshot restored, exactly that many samples re-rendered), so every sample is the one the
    // per-sample sequence produces.
    static constexpr long kLook = 1024, kLookMin = 64;
    double* la_buf = nullptr;          // pinned [kLook] rendered outputs
    long la_n = 0, la_pos = 0;         // rendered / consumed samples of the speculative block
    double *d_phi_snap = nullptr, *d_f_snap = nullptr;
    std::vector<double> amp_snap, c_first_snap;
    std::vector<char> alive_snap;
    long la_blocks = 0, la_rollbacks = 0;

    int init(int V_, int O_, int o0_, int OL_, double s_, double a_, int dev) {
        V = V_;
        O = O_;
        o0 = o0_;
        OL = OL_;
        s = s_;
        a = a_;
        device = dev;
        const size_t P = (size_t)V * OL;
        ft.assign(P, 0.0);
        c.assign(P, 0.0);
        c_first.assign(P, 0.0);
        amp.assign(V, 0.0);
        act.assign(V, 0.0);
        alive.assign(V, 0);
        dirty.assign(V, 1);
        h_rec.assign(P * PRec::SIZE, 0.0);
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
            target_groups = prop.multiProcessorCount;
        HZ_TRY_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        own_stream = true;
        HZ_TRY_HIP(hipMalloc(&d_rec, sizeof(double) * P * PRec::SIZE));
        HZ_TRY_HIP(hipMalloc(&d_phi, sizeof(double) * P));
        HZ_TRY_HIP(hipMalloc(&d_f, sizeof(double) * P));
        HZ_TRY_HIP(hipMalloc(&d_ft, sizeof(double) * P));
        HZ_TRY_HIP(hipMalloc(&d_amp, sizeof(double) * V));
        HZ_TRY_HIP(hipMalloc(&d_act, sizeof(double) * V));
        HZ_TRY_HIP(hipMalloc(&d_c0, sizeof(double) * P));
        HZ_TRY_HIP(hipMemset(d_phi, 0, sizeof(double) * P));
        HZ_TRY_HIP(hipMemset(d_f, 0, sizeof(double) * P));
        return HZ_OK;
    }

    void release() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        for (void* p : {(void*)d_rec, (void*)d_phi, (void*)d_f, (void*)d_ft, (void*)d_amp, (void*)d_act,
                        (void*)d_partial, (void*)d_out, (void*)d_tasks, (void*)d_c0, (void*)d_phi_snap,
                        (void*)d_f_snap})
            if (p) (void)hipFree(p);
        if (la_buf) (void)hipHostFree(la_buf);
        for (hipEvent_t e : ev) (void)hipEventDestroy(e);
        if (own_stream && stream) (void)hipStreamDestroy(stream);
    }

    // render n samples into d_out (device), then advance all state
    int render(double* d_dst, long n) {
        if (n <= 0) return HZ_OK;
        HZ_TRY_HIP(hipSetDevice(device));
        const size_t P = (size_t)V * OL;
        // records of voices whose targets changed (note events); state stays on the device
        tasks.clear();
        const int per_wave = std::min(kMaxPerWave, std::max(1, OL));
        bool any_dirty = false;
        for (int v = 0; v < V; ++v) {
            if (dirty[v]) {
                for (int j = 0; j < OL; ++j) {
                    const size_t p = (size_t)v * OL + j;
                    double* r = &h_rec[p * PRec::SIZE];
                    r[PRec::A] = ft[p] / hz::kSR;
                    r[PRec::C] = c[p];
                    fill_tables(r[PRec::A], r);
                }
                HZ_TRY_HIP(hipMemcpyAsync(d_rec + (size_t)v * OL * PRec::SIZE, &h_rec[(size_t)v * OL * PRec::SIZE],
                                          sizeof(double) * OL * PRec::SIZE, hipMemcpyHostToDevice, stream));
                dirty[v] = 0;
                any_dirty = true;
            }
            if (!(alive[v] || act[v] != 0.0)) continue;  // never-sounded voices are skipped and frozen
            for (int j0 = 0; j0 < OL; j0 += per_wave)
                tasks.push_back(Task{v * OL + j0, std::min(per_wave, OL - j0), v, 0});
        }
        if (any_dirty)
            HZ_TRY_HIP(hipMemcpyAsync(d_ft, ft.data(), sizeof(double) * P, hipMemcpyHostToDevice, stream));
        HZ_TRY_HIP(hipMemcpyAsync(d_amp, amp.data(), sizeof(double) * V, hipMemcpyHostToDevice, stream));
        HZ_TRY_HIP(hipMemcpyAsync(d_act, act.data(), sizeof(double) * V, hipMemcpyHostToDevice, stream));
        const int ntasks = (int)tasks.size();
        if (ntasks > 0) {
            if ((size_t)ntasks > task_cap) {
                if (d_tasks) HZ_TRY_HIP(hipFree(d_tasks));
                d_tasks = nullptr;
                HZ_TRY_HIP(hipMalloc(&d_tasks, sizeof(Task) * ntasks));
                task_cap = ntasks;
            }
            HZ_TRY_HIP(hipMemcpyAsync(d_tasks, tasks.data(), sizeof(Task) * ntasks, hipMemcpyHostToDevice, stream));
        }
        const bool c0_differs = c_first != c;
        if (c0_differs)
            HZ_TRY_HIP(hipMemcpyAsync(d_c0, c_first.data(), sizeof(double) * P, hipMemcpyHostToDevice, stream));
        HZ_TRY_HIP(hipStreamSynchronize(stream));  // pageable host sources above are reused

        hipEvent_t* e = nullptr;
        if (prof) {
            if (ev_used + 2 > ev.size())
                for (int q = 0; q < 128; ++q) {
                    hipEvent_t ne;
                    HZ_TRY_HIP(hz::prof_event_create(&ne));
                    ev.push_back(ne);
                }
            e = &ev[ev_used];
            ev_used += 2;
            HZ_TRY_HIP(hipEventRecord(e[0], stream));
        }
        if (ntasks == 0) {
            HZ_TRY_HIP(hipMemsetAsync(d_dst, 0, sizeof(double) * n, stream));
        } else {
            // groups: one task per wave by default.  Fewer groups (a wave taking several tasks in turn)
            // cut the partial rows -- one group writes the output directly, 146 -> 67 MB counted per
            // C3 step -- but measured slower (C3: 19 groups 1.19 ms, 4: 1.46, 2: 1.86; one group for the
            // long call 1.47 ms: every workgroup then streams all 3.7 MB of partial records per tile);
            // HZ_ADD_GROUPS sets it (A/B, scripts/r6_c3ab.sh)
            const long ntiles = (n + kTile - 1) / kTile;
            const int gmax = (ntasks + kWaves - 1) / kWaves;
            int G = gmax;
            static const int g_env = getenv("HZ_ADD_GROUPS") ? atoi(getenv("HZ_ADD_GROUPS")) : 0;
            if (g_env > 0) G = std::min(gmax, g_env);
            const int tpw = (ntasks + G * kWaves - 1) / (G * kWaves);
            G = (ntasks + tpw * kWaves - 1) / (tpw * kWaves);
            long nseg = std::max<long>(1, std::min<long>(ntiles, (target_groups + G - 1) / G));
            const long seg_tiles = (ntiles + nseg - 1) / nseg;
            nseg = (ntiles + seg_tiles - 1) / seg_tiles;
            const long n_pad = ntiles * kTile;
            const size_t need = G > 1 ? (size_t)G * n_pad : 1;
            if (need > partial_cap) {
                if (d_partial) HZ_TRY_HIP(hipFree(d_partial));
                d_partial = nullptr;
                HZ_TRY_HIP(hipMalloc(&d_partial, sizeof(double) * need));
                partial_cap = need;
            }
            const size_t lds = sizeof(double) * (kWaves * kL * kPad);
            static bool attr = false;
            if (!attr) {
                HZ_TRY_HIP(hipFuncSetAttribute((const void*)add_mix_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
                attr = true;
            }
            AddArgs args;
            args.tasks = d_tasks;
            args.phi = d_phi;
            args.f = d_f;
            args.ft = d_ft;
            args.amp0 = d_amp;
            args.act = d_act;
            args.c0 = c0_differs ? d_c0 : nullptr;
            args.partial = G > 1 ? d_partial : d_dst;
            args.scale = scale;
            args.tpw = tpw;
            args.n = n;
            args.n_pad = n_pad;
            args.seg_len = seg_tiles * kTile;
            args.ntasks = ntasks;
            args.nseg = (int)nseg;
            args.a = a;
            args.s = s;
            hipLaunchKernelGGL(add_mix_kernel, dim3(G, (unsigned)nseg), dim3(64 * kWaves), lds, stream,
                               (const double*)d_rec, args);
            HZ_TRY_HIP(hipGetLastError());
            if (G > 1) {
                hipLaunchKernelGGL(add_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(256), 0, stream,
                                   (const double*)d_partial, n_pad, G, n, scale, d_dst);
                HZ_TRY_HIP(hipGetLastError());
            }
            const double s_n = (double)powl((long double)s, (long double)n);
            hipLaunchKernelGGL(add_advance_kernel, dim3(ntasks), dim3(64), 0, stream, (const double*)d_rec,
                               (const Task*)d_tasks, ntasks, n, s, s_n, (const double*)d_ft, d_phi, d_f);
            HZ_TRY_HIP(hipGetLastError());
        }
        if (e) HZ_TRY_HIP(hipEventRecord(e[1], stream));
        launches += prof ? 1 : 0;
        c_first = c;
        // envelopes (V scalars): closed form, alive is sticky (a released envelope decays
        // to a denormal fixed point > 0 in the reference and never reaches 0)
        const long double an = powl((long double)a, (long double)n);
        for (int v = 0; v < V; ++v) {
            if (act[v] != 0.0) alive[v] = 1;
            if (!alive[v]) continue;
            amp[v] = (double)((long double)act[v] + an * ((long double)amp[v] - (long double)act[v]));
        }
        return HZ_OK;
    }

    // roll the engine back to the consumed position of the speculative block (before any setter,
    // any longer fill or a device fill)
    int settle() {
        if (la_pos < la_n) {
            const size_t P = (size_t)V * OL;
            HZ_TRY_HIP(hipMemcpyAsync(d_phi, d_phi_snap, sizeof(double) * P, hipMemcpyDeviceToDevice, stream));
            HZ_TRY_HIP(hipMemcpyAsync(d_f, d_f_snap, sizeof(double) * P, hipMemcpyDeviceToDevice, stream));
            amp = amp_snap;
            alive = alive_snap;
            c_first = c_first_snap;
            const long m = la_pos;
            la_n = la_pos = 0;
            ++la_rollbacks;
            if (m > 0) HZ_TRY(render_scratch(m));
        }
        la_n = la_pos = 0;
        return HZ_OK;
    }

    int ensure_out(long n) {
        if ((size_t)n <= out_cap) return HZ_OK;
        if (d_out) HZ_TRY_HIP(hipFree(d_out));
        d_out = nullptr;
        HZ_TRY_HIP(hipMalloc(&d_out, sizeof(double) * n));
        out_cap = n;
        return HZ_OK;
    }

    int render_scratch(long n) {
        HZ_TRY(ensure_out(n));
        return render(d_out, n);
    }

    // a new speculative block: snapshot, render kLook samples, outputs to pinned memory
    int look_ahead() {
        const size_t P = (size_t)V * OL;
        if (!la_buf) {
            HZ_TRY_HIP(hipHostMalloc((void**)&la_buf, sizeof(double) * kLook));
            HZ_TRY_HIP(hipMalloc(&d_phi_snap, sizeof(double) * P));
            HZ_TRY_HIP(hipMalloc(&d_f_snap, sizeof(double) * P));
        }
        HZ_TRY_HIP(hipMemcpyAsync(d_phi_snap, d_phi, sizeof(double) * P, hipMemcpyDeviceToDevice, stream));
        HZ_TRY_HIP(hipMemcpyAsync(d_f_snap, d_f, sizeof(double) * P, hipMemcpyDeviceToDevice, stream));
        amp_snap = amp;
        alive_snap = alive;
        c_first_snap = c_first;
        HZ_TRY(ensure_out(kLook));
        HZ_TRY(render(d_out, kLook));
        HZ_TRY_HIP(hipMemcpyAsync(la_buf, d_out, sizeof(double) * kLook, hipMemcpyDeviceToHost, stream));
        HZ_TRY_HIP(hipStreamSynchronize(stream));
        la_n = kLook;
        la_pos = 0;
        ++la_blocks;
        return HZ_OK;
    }

    int fill_host(double* out, long n) {
        if (n <= 0) return HZ_OK;
        if (n < kLookMin) {   // per-sample calls: from the speculative block
            for (long i = 0; i < n; ++i) {
                if (la_pos == la_n) HZ_TRY(look_ahead());
                out[i] = la_buf[la_pos++];
            }
            return HZ_OK;
        }
        HZ_TRY(settle());
        if ((size_t)n > out_cap) {
            if (d_out) HZ_TRY_HIP(hipFree(d_out));
            d_out = nullptr;
            HZ_TRY_HIP(hipMalloc(&d_out, sizeof(double) * n));
            out_cap = n;
        }
        HZ_TRY(render(d_out, n));
        HZ_TRY_HIP(hipMemcpyAsync(out, d_out, sizeof(double) * n, hipMemcpyDeviceToHost, stream));
        HZ_TRY_HIP(hipStreamSynchronize(stream));
        return HZ_OK;
    }
};

// ---------------------------------------------------------------------------
// Additive<double>  (src/additive.h:11-71 + Minimizer note API, src/minimizer.h:111-181)
// ---------------------------------------------------------------------------
struct hz_add {
    PhaseBank bank;
    int V = 0, O = 0;
    double decay = 0, harmonicity = 1, norm = 1;
    std::vector<double> active;     // Minimizer::active (amplitude targets)
    std::vector<double> pitches;    // Minimizer::pitches
    std::vector<double> guide;      // guides[v].position
    std::vector<double> position;   // particles[v*O+j].position (all overtones)
};

namespace {

int add_check(hz_add* h) {
    if (!h) {
        hz::set_error("null hz_add handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->bank.device));
    return HZ_OK;
}

// Additive::tick's freqmod(mtof(particle position)) for the local overtones of voice v
void add_retarget(hz_add* h, int v) {
    PhaseBank& b = h->bank;
    b.dirty[v] = 1;
    for (int jl = 0; jl < b.OL; ++jl) {
        const int j = b.o0 + jl;
        b.ft[(size_t)v * b.OL + jl] = (double)mtofl((long double)h->position[(size_t)v * h->O + j]);
    }
}

}  // namespace

extern "C" {

int hz_add_create_shard(int voices, int overtones, int o_begin, int o_count, double decay, double harmonicity,
                        double k, int device, hz_add** out) {
    if (!out || voices <= 0 || overtones <= 0 || o_begin < 0 || o_count <= 0 || o_begin + o_count > overtones) {
        hz::set_error("hz_add_create: invalid arguments");
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_add* h = new (std::nothrow) hz_add();
    if (!h) return HZ_E_ALLOC;
    h->V = voices;
    h->O = overtones;
    h->decay = decay;
    h->harmonicity = harmonicity;
    // additive.h:27 normalization; oscillators are Oscillator(0, 0, 0.0001) (35)
    h->norm = decay != 1 ? (1 - std::pow(decay, overtones)) / (1 - decay) : overtones;
    int rc = h->bank.init(voices, overtones, o_begin, o_count, hz::relaxation(0.0001), hz::relaxation(k), device);
    if (rc != HZ_OK) {
        h->bank.release();
        delete h;
        return rc;
    }
    for (int v = 0; v < voices; ++v)
        for (int jl = 0; jl < o_count; ++jl)
            h->bank.c[(size_t)v * o_count + jl] = std::pow(decay, o_begin + jl);
    h->bank.c_first = h->bank.c;
    h->bank.scale = 1.0 / (voices * h->norm);
    h->active.assign(voices, 0.0);
    h->pitches.assign(voices, 0.0);
    h->guide.assign(voices, 0.0);
    h->position.assign((size_t)voices * overtones, 0.0);
    *out = h;
    return HZ_OK;
}

int hz_add_create(int voices, int overtones, double decay, double harmonicity, double k, int device, hz_add** out) {
    return hz_add_create_shard(voices, overtones, 0, overtones, decay, harmonicity, k, device, out);
}

int hz_add_destroy(hz_add* h) {
    if (!h) return HZ_OK;
    h->bank.release();
    delete h;
    return HZ_OK;
}

// request(fundamental, amplitude)  minimizer.h:111-158; physics is out of scope, so the
// particle positions stay where request() puts them.
int hz_add_request(hz_add* h, double fundamental, double amplitude, int* voice_out) {
    if (!h) return HZ_E_INVALID;
    HZ_TRY(add_check(h));
    HZ_TRY(h->bank.settle());   // a speculative block rolls back to the consumed sample first
    int voice = -1;
    for (int i = 0; i < h->V; ++i)
        if (!h->active[i]) {
            voice = i;
            break;
        }
    if (voice < 0) {  // steal the voice whose guide is nearest in pitch
        const double pitch = 69 + std::log2(fundamental / 440.0) * 12;
        double distance = 0;
        int nearest = -1;
        for (int i = 0; i < h->V; ++i) {
            double offset = pitch - h->guide[i];
            offset *= offset;
            if (nearest < 0 || offset < distance) {
                nearest = i;
                distance = offset;
            }
        }
        voice = nearest;
    }
    h->active[voice] = amplitude;
    h->guide[voice] = 69 + std::log2(fundamental / 440.0) * 12;
    for (int j = 0; j < h->O; ++j) {
        const double frequency =
            fundamental * (1 + std::pow((double)j / (h->O - 1), h->harmonicity) * (h->O - 1));
        h->position[(size_t)voice * h->O + j] = 69 + std::log2(frequency / 440.0) * 12;
    }
    h->bank.act[voice] = amplitude;
    add_retarget(h, voice);
    if (voice_out) *voice_out = voice;
    return HZ_OK;
}

// release(voice) minimizer.h:161-172 (voice < 0: all)
int hz_add_release(hz_add* h, int voice) {
    if (!h) return HZ_E_INVALID;
    HZ_TRY(add_check(h));
    HZ_TRY(h->bank.settle());
    for (int i = 0; i < h->V; ++i)
        if (voice < 0 || i == voice) {
            h->active[i] = 0;
            h->bank.act[i] = 0;
        }
    return HZ_OK;
}

int hz_add_makenote(hz_add* h, double pitch, double amplitude, int* voice_out) {   // minimizer.h:174-179
    if (!h) return HZ_E_INVALID;
    int v = -1;
    HZ_TRY(hz_add_request(h, 440.0 * std::pow(2, (pitch - 69) / 12), amplitude, &v));
    if (v >= 0) h->pitches[v] = pitch;
    if (voice_out) *voice_out = v;
    return HZ_OK;
}

int hz_add_endnote(hz_add* h, double pitch) {   // minimizer.h:182-187
    if (!h) return HZ_E_INVALID;
    for (int j = 0; j < h->V; ++j)
        if (h->pitches[j] == pitch) hz_add_release(h, j);
    return HZ_OK;
}

// n x { out[t] = operator()(); tick(); }   additive.h:38-62
int hz_add_fill(hz_add* h, double* out, size_t n) {
    HZ_TRY(add_check(h));
    if (n && !out) return HZ_E_INVALID;
    return h->bank.fill_host(out, (long)n);
}

int hz_add_fill_device(hz_add* h, double* d_out, size_t n) {
    HZ_TRY(add_check(h));
    if (n && !d_out) return HZ_E_INVALID;
    HZ_TRY(h->bank.settle());
    return h->bank.render(d_out, (long)n);
}

// per-sample service statistics: speculative blocks rendered, rollbacks (setters inside a block)
int hz_add_lookahead_info(hz_add* h, long* blocks, long* rollbacks, long* block_len) {
    if (!h) return HZ_E_INVALID;
    if (blocks) *blocks = h->bank.la_blocks;
    if (rollbacks) *rollbacks = h->bank.la_rollbacks;
    if (block_len) *block_len = PhaseBank::kLook;
    return HZ_OK;
}

int hz_add_set_stream(hz_add* h, void* s) {
    HZ_TRY(add_check(h));
    HZ_TRY(h->bank.settle());
    HZ_TRY_HIP(hipStreamSynchronize(h->bank.stream));
    if (h->bank.own_stream) HZ_TRY_HIP(hipStreamDestroy(h->bank.stream));
    if (s) {
        h->bank.stream = (hipStream_t)s;
        h->bank.own_stream = false;
    } else {
        HZ_TRY_HIP(hipStreamCreateWithFlags(&h->bank.stream, hipStreamNonBlocking));
        h->bank.own_stream = true;
    }
    return HZ_OK;
}

int hz_add_set_target_groups(hz_add* h, int groups) {
    if (!h || groups < 1) return HZ_E_INVALID;
    h->bank.target_groups = groups;
    return HZ_OK;
}

int hz_add_profile(hz_add* h, int enable) {
    HZ_TRY(add_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->bank.stream));
    h->bank.prof = enable != 0;
    h->bank.ev_used = 0;
    h->bank.launches = 0;
    return HZ_OK;
}

int hz_add_profile_read(hz_add* h, double* ms, long* launches) {
    HZ_TRY(add_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->bank.stream));
    double m = 0;
    for (size_t i = 0; i + 2 <= h->bank.ev_used; i += 2) {
        float x = 0;
        HZ_TRY_HIP(hipEventElapsedTime(&x, h->bank.ev[i], h->bank.ev[i + 1]));
        m += x;
    }
    if (ms) *ms = m;
    if (launches) *launches = h->bank.launches;
    return HZ_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Sinusoids<double>  (src/sinusoids.h:10-79): one voice, amp = 1, partial i at
// fundamental (i+1)^harmonicity, weight decay^i / normalization.  The smoothing of
// fundamental / decay / harmonicity (stiffness relaxation(k), k = 2/SR by default, i.e.
// 1.5e-8 per sample) is taken to complete at the call boundary.
// ---------------------------------------------------------------------------
struct hz_sin {
    PhaseBank bank;
    int O = 0;
    double fundamental = 0, decay = 0, harmonicity = 1;
};

namespace {
void sin_retarget(hz_sin* h) {
    PhaseBank& b = h->bank;
    b.dirty[0] = 1;
    const double norm = h->decay != 1 ? (1 - std::pow(h->decay, h->O)) / (1 - h->decay) : h->O;
    for (int i = 0; i < h->O; ++i) {
        b.ft[i] = h->fundamental * std::pow(i + 1, h->harmonicity);
        b.c[i] = std::pow(h->decay, i) / norm;
    }
}
}  // namespace

extern "C" {

int hz_sin_create(double fundamental, int overtones, double decay, double harmonicity, double k, int device,
                  hz_sin** out) {
    if (!out || overtones <= 0) {
        hz::set_error("hz_sin_create: invalid arguments");
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_sin* h = new (std::nothrow) hz_sin();
    if (!h) return HZ_E_ALLOC;
    h->O = overtones;
    h->fundamental = fundamental;
    h->decay = decay;
    h->harmonicity = harmonicity;
    // Synth(form, fundamental * pow(i+1, harmonicity)) with the default k = 2/SR (sinusoids.h:23-27)
    int rc = h->bank.init(1, overtones, 0, overtones, hz::relaxation(2.0 / hz::kSR), 0.0, device);
    if (rc != HZ_OK) {
        h->bank.release();
        delete h;
        return rc;
    }
    (void)k;
    h->bank.act[0] = 1.0;
    h->bank.amp[0] = 1.0;
    h->bank.alive[0] = 1;
    h->bank.scale = 1.0;
    sin_retarget(h);
    h->bank.c_first = h->bank.c;
    // oscillators start at their target frequency, phase 0 (oscillator.h:16-24)
    std::vector<double> f0(h->bank.ft);
    HZ_TRY_HIP(hipMemcpy(h->bank.d_f, f0.data(), sizeof(double) * overtones, hipMemcpyHostToDevice));
    *out = h;
    return HZ_OK;
}

int hz_sin_destroy(hz_sin* h) {
    if (!h) return HZ_OK;
    h->bank.release();
    delete h;
    return HZ_OK;
}

int hz_sin_fundmod(hz_sin* h, double target) {   // sinusoids.h:67-68
    if (!h) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->bank.device));
    HZ_TRY(h->bank.settle());
    h->fundamental = target;
    sin_retarget(h);
    return HZ_OK;
}

int hz_sin_decaymod(hz_sin* h, double target) {   // sinusoids.h:61-62
    if (!h) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->bank.device));
    HZ_TRY(h->bank.settle());
    h->decay = target;
    sin_retarget(h);
    return HZ_OK;
}

int hz_sin_harmmod(hz_sin* h, double target) {    // sinusoids.h:64-65
    if (!h) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->bank.device));
    HZ_TRY(h->bank.settle());
    h->harmonicity = target;
    sin_retarget(h);
    return HZ_OK;
}

// n x { out[t] = operator()(); tick(); }   sinusoids.h:34-57
int hz_sin_fill(hz_sin* h, double* out, size_t n) {
    if (!h) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->bank.device));
    if (n && !out) return HZ_E_INVALID;
    return h->bank.fill_host(out, (long)n);
}

int hz_sin_fill_device(hz_sin* h, double* d_out, size_t n) {
    if (!h) return HZ_E_INVALID;
    HZ_TRY_HIP(hipSetDevice(h->bank.device));
    if (n && !d_out) return HZ_E_INVALID;
    HZ_TRY(h->bank.settle());
    return h->bank.render(d_out, (long)n);
}

}  // extern "C"
