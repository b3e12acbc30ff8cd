// hz_rt.h -- the per-sample server (hz_rt.hip): one resident kernel per device that serves the
// per-sample operator calls of every input-driven bank -- Filterbank operator()/tick()
// (src/filterbank.h:125-148), Delay/Delaybank operator()/tick() (src/delay.h:71-97) and
// Granulator operator()/tick() with its source Buffer (src/granulator.h:81-104) -- through a
// mailbox in pinned host memory.  The reference calls these once per sample inside the audio
// callback (tests/resynthesis.cpp:35-39, tests/delay.cpp:20-28, tests/granny.cpp:32-56), and a
// caller may feed an output back into the next input, so a sample cannot wait for a block.
//
// One server for all handles (instead of a resident kernel per handle): with GPU_MAX_HW_QUEUES
// hardware queues per process, a resident kernel per handle occupied one queue each and every
// other stream mapped onto that queue waited for its idle exit.  The server runs on a stream of
// the highest priority (its own hardware queue) and leaves after kIdleNs without a request.
#pragma once

#include <cstddef>
#include <mutex>

#include "hz_common.h"

namespace hz_rt {

constexpr int kGroups = 8;      // workgroups of the resident kernel (each polls the mailbox)
constexpr int kThreads = 512;   // threads per workgroup (units per workgroup per pass)
constexpr int kMaxGrains = 1024;

enum : int { OP_NONE = 0, OP_FB = 1, OP_DLY = 2, OP_GRAN = 3, OP_STOP = 4, OP_FB_MANY = 5 };

// Granulator grain record (hz_granulator.hip: the block engine's layout, one 64-B line)
struct alignas(16) Grain {
    long t_first, t_end;                      // reads at t_first <= t < t_end
    double offsets, sizes, speeds, gains;     // granulator.h:67-70 (samples, samples, ratio, gain)
    unsigned ticks0, pad0;
    double rsizes;                            // RN(1 / sizes) for a normal finite quotient, else 0
};
static_assert(sizeof(Grain) == 64, "grain record is one 64 B line");

// cos(x) for 0 <= x <= 2 PI + 1e-9 (the hann argument 2 PI phase, phase in [0, 1]): k = rint(x 2/pi)
// in 0..4, r = x - k pi/2 in a two-part Cody-Waite split (k pio2_1 exact: 33-bit head), then
// fdlibm's __kernel_sin / __kernel_cos polynomials on |r| <= pi/4 (< 1 ulp each) -- against the
// library cos's general argument reduction
__device__ __forceinline__ double cos_0_2pi(double x) {
    constexpr double kInvPio2 = 6.36619772367581382433e-01;
    constexpr double kPio2_1 = 1.57079632673412561417e+00, kPio2_1t = 6.07710050650619224932e-11;
    const double kf = __builtin_rint(x * kInvPio2);
    const int k = (int)kf;
    const double r = (x - kf * kPio2_1) - kf * kPio2_1t;
    const double z = r * r;
    // __kernel_sin(r): r + r^3 (S1 + z (S2 + ...))
    double ps = 1.58969099521155010221e-10;
    ps = __builtin_fma(ps, z, -2.50507602534068634195e-08);
    ps = __builtin_fma(ps, z, 2.75573137070700676789e-06);
    ps = __builtin_fma(ps, z, -1.98412698298579493134e-04);
    ps = __builtin_fma(ps, z, 8.33333333332248946124e-03);
    ps = __builtin_fma(ps, z, -1.66666666666666324348e-01);
    const double sn = __builtin_fma(r * z, ps, r);
    // __kernel_cos(r): 1 - z/2 + z^2 (C1 + z (C2 + ...)), the 1 - z/2 part compensated
    double pc = -1.13596475577881948265e-11;
    pc = __builtin_fma(pc, z, 2.08757232129817482790e-09);
    pc = __builtin_fma(pc, z, -2.75573143513906633035e-07);
    pc = __builtin_fma(pc, z, 2.48015872894767294178e-05);
    pc = __builtin_fma(pc, z, -1.38888888888741095749e-03);
    pc = __builtin_fma(pc, z, 4.16666666666666019037e-02);
    const double hz_ = 0.5 * z, w = 1.0 - hz_;
    const double cs = w + (((1.0 - w) - hz_) + z * z * pc);
    switch (k & 3) {
    case 0: return cs;
    case 1: return -sn;
    case 2: return -cs;
    default: return sn;
    }
}

// sin and cos of 0 <= x <= 2 PI + 1e-9, the reduction and polynomials of cos_0_2pi (its cosine is
// bit-identical to cos_0_2pi's)
__device__ __forceinline__ void sincos_0_2pi(double x, double* sn_out, double* cs_out) {
    constexpr double kInvPio2 = 6.36619772367581382433e-01;
    constexpr double kPio2_1 = 1.57079632673412561417e+00, kPio2_1t = 6.07710050650619224932e-11;
    const double kf = __builtin_rint(x * kInvPio2);
    const int k = (int)kf;
    const double r = (x - kf * kPio2_1) - kf * kPio2_1t;
    const double z = r * r;
    double ps = 1.58969099521155010221e-10;
    ps = __builtin_fma(ps, z, -2.50507602534068634195e-08);
    ps = __builtin_fma(ps, z, 2.75573137070700676789e-06);
    ps = __builtin_fma(ps, z, -1.98412698298579493134e-04);
    ps = __builtin_fma(ps, z, 8.33333333332248946124e-03);
    ps = __builtin_fma(ps, z, -1.66666666666666324348e-01);
    const double sn = __builtin_fma(r * z, ps, r);
    double pc = -1.13596475577881948265e-11;
    pc = __builtin_fma(pc, z, 2.08757232129817482790e-09);
    pc = __builtin_fma(pc, z, -2.75573143513906633035e-07);
    pc = __builtin_fma(pc, z, 2.48015872894767294178e-05);
    pc = __builtin_fma(pc, z, -1.38888888888741095749e-03);
    pc = __builtin_fma(pc, z, 4.16666666666666019037e-02);
    const double hz_ = 0.5 * z, w = 1.0 - hz_;
    const double cs = w + (((1.0 - w) - hz_) + z * z * pc);
    switch (k & 3) {
    case 0: *sn_out = sn; *cs_out = cs; break;
    case 1: *sn_out = cs; *cs_out = -sn; break;
    case 2: *sn_out = -sn; *cs_out = -cs; break;
    default: *sn_out = -cs; *cs_out = sn; break;
    }
}

// the Granulator's window term's cosine, block kernel and per-sample server alike (bit-identical)
__device__ __forceinline__ double hann_cos(double arg, bool fast) {
    return (fast && arg >= 0.0 && arg <= 6.2831853072) ? cos_0_2pi(arg) : cos(arg);
}

// ---- op arguments (copied into the request line; <= kArgWords 8-byte words) ------------------
// Filterbank sample: ring rows R [N][O+1] in ring order (R[0..O-1] = y[t-1 .. t-O], R[O] = the
// row at origin), smoothers pg [N][2], coefficients [N][2O+1], targets pin / gin [N].
struct FbArgs {
    double* R;
    double* pg;
    const double* coef;
    double* pin;
    double* gin;
    const double* reload;   // (device address of pinned payload) [N] pin then [N] gin, or null
    const double* reload_coef;   // (pinned payload) [N][2O+1] new coefficients, or null
    const double* sparse;   // (pinned payload) [nsparse] (band, pin, gin) triples, or null
    double x, param, sp, sg;
    double xr[5];           // input ring (ring order) after the ticks, before this compute
    int N, O;
    int ticks, compute, dist, nsparse;
};
// Delaybank sample (hz_delay.hip layout): rings [N][size], taps [N][2S] {thr, age_nowrap,
// age_wrap, 0}, gains [N][2S] T; every line reads x (mono) or xin[line]; y[line] -> out
struct DlyArgs {
    void* rx;
    void* ry;
    const int4* taps;
    const void* gains;
    const double* xin;      // (pinned payload) per-line inputs, or null: mono x
    double* out;            // (pinned result) [N] line outputs (in T's precision, widened)
    double x;
    int N, S, is_float, pad;
    unsigned size, o;
};
// Granulator sample at time t: x into the time-indexed ring, then the sum over the active grains
// (voice order); the grain list is cached in the serving workgroup's LDS by (key, version)
struct GranArgs {
    double* ring;
    const Grain* grains;    // (pinned payload) the handle's grains that may still read, voice order
    long mask, t, key, version;
    double x;
    unsigned long fm;
    int count, pad;
    unsigned size, origin, wrap1, pad2;
};

// OP_FB_MANY: one sample of several Filterbanks in one request (the per-channel banks of
// tests/filterbanks.cpp:191-211).  The static part is a device table of 64-band chunks (each with
// its member's arrays offset to the chunk's first band); the request line carries each member's
// input and input ring.
constexpr int kMaxMany = 12;
struct alignas(64) ManyChunk {
    double* R;              // ring rows [n][O+1] from the chunk's first band
    double* pg;             // smoothers [n][2]
    const double* coef;     // [n][2O+1]
    const double* pin;
    const double* gin;
    int n, m;               // bands in the chunk (<= 64), member
    double sp, sg;
};
struct ManyArgs {
    const ManyChunk* chunks;
    double* out;            // (pinned result) [groups][H] partial mixdowns
    double param;
    int H, nchunks;
    int O, dist;
    unsigned long long meta;   // per member 4 bits: ticks (0..O) | compute << 3
    double xv[1];           // per member x, then its input ring xr[0..O] (O + 2 words each)
};
constexpr int kManyHeader = 6;   // words before xv

constexpr int kArgWords = 62;
struct alignas(64) Req {
    long long req;          // request number << 4 | participating workgroups, written last (release)
    int op, groups;         // op; workgroups that take part (the others skip the request)
    long long w[kArgWords]; // op arguments
};
static_assert(sizeof(FbArgs) <= sizeof(long long) * kArgWords && sizeof(DlyArgs) <= sizeof(long long) * kArgWords &&
                  sizeof(GranArgs) <= sizeof(long long) * kArgWords,
              "op arguments fit the request line");
static_assert(offsetof(ManyArgs, xv) == 8 * kManyHeader, "OP_FB_MANY header");
struct alignas(64) Slot {   // per workgroup
    double y, y2;           // partial mix
    long long done;         // last request served (written after y)
    long long exited;       // epoch of the instance whose workgroup left
    long long pad[4];
};

// ---- host side ------------------------------------------------------------------------------
struct Server;
// the device's server (created on first use; lives for the process)
Server* server(int device);
// pinned staging shared by the server's requests (host pointer; device address via dev())
double* payload(Server* s, size_t doubles);   // grows (only between requests)
double* result(Server* s, size_t doubles);
const void* dev(Server* s, const void* host_ptr);
// one request: args copied into the line, the participating workgroups answer; -> sum of the taking-part
// workgroups' partials (y, y2) in workgroup order.  Serialised per device (the caller holds
// lock(s) across a multi-request sequence when the order matters).
int call(Server* s, int op, const void* args, size_t bytes, int groups, double* y, double* y2 = nullptr);
std::recursive_mutex& lock(Server* s);
// the resident instance leaves now (the next request relaunches it): a handle whose bands change
// workgroups (OP_FB <-> OP_FB_MANY) must not read rows another XCD's L2 wrote
void quiesce(Server* s);
// statistics: requests served, launches of the resident kernel
void info(Server* s, long long* requests, long long* launches, int* active);

}  // namespace hz_rt
