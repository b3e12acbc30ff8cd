// hz_fb_state.h -- the band-state pass of the stationary engine as a workgroup-level device
// function: every band's zero-start state after a window of len samples (len a multiple of 8192),
//     S_n = sum_c M_n^(C-1-c) pin_n E_n x_c        (c < C = len / 128 chunks of 128 samples)
// with E_n the chunk's zero-state end-state map over its L + O input taps and M_n the chunk
// transition (the chunk-128 LTI records, hz_fb_rec.h; the band recurrence of
// src/filterbank.h:178-179 restated chunk-wise).  That is N O len multiply-adds, ~0.8 GFLOP at
// C2 (4096 bands, O = 2, len = 49152): the pass is bound by the FP64 matrix cores (78.6 TFLOP/s).
//
// Work split: one workgroup = 32 band-state columns (16 bands of O = 2; OP = O padded to a power
// of two columns per band) x one run of tiles; 4 waves (one per SIMD), wave m owns chunk rows
// 16m..16m+15 of every 8192-sample tile (64 chunks) and runs two independent chains of 33
// v_mfma_f64_16x16x4f64 per tile, one per 16-column block, whose accumulators start from M^64
// applied to the previous tiles' sum, so after the last tile accumulator row c holds
//     A_c = sum_tiles M^(64 (T-1-t)) z_{t,c},   z_{t,c} = pin E x_{t,c}
// and S = sum_c M^(63-c) A_c (one weighted reduction at the end, across lanes and waves).
//   * A operands (the chunk windows) go straight from the L2-resident x window into registers
//     with no LDS and no barrier: the MFMA's k index is free up to a permutation shared by A and
//     B, and lane group g (k within the step) of k-step q takes tap
//         tap(q, g) = 8 (q >> 1) + 2 g + (q & 1)   (q < 32),   128 + g   (q = 32)
//     so each lane reads its chunk's taps as 16 aligned pairs (buffer_load_dwordx4: 16 chunks x
//     64 contiguous bytes per instruction) plus one double; each pair is reloaded with the next
//     tile's taps as soon as its two k-steps have issued (one register set, a tile of latency);
//   * B operands (pin E in that tap order, fb_state_ops_kernel) live in registers, loaded with
//     tile 0's A operands in the order the first tile's k-steps use them;
//   * the O taps before the window are the zero-start history: the window is addressed through
//     a buffer resource whose range check returns 0 for them (tap pairs never straddle the window
//     start: odd orders shift the taps by one, s = O & 1, with a zero E row) and for taps past
//     the window's end (E entries 0 there).
// At O <= 2 a wave fits 256 registers, so a CU holds a state workgroup beside a transform
// workgroup: hz_fb_resp.hip runs the pass as extra workgroups of its transform kernels.
//
// Banks with fewer band groups than CUs split the window into equal runs of tiles ("pieces", one
// workgroup each); they store their partials, combined by Horner steps, S = P (... (P S_0 + S_1)
// ...) + S_last, P = (M^64)^(tiles per piece): standalone, by the last workgroup of a band group to
// arrive (device-scope counter, re-armed); inside the inverse kernel, by a small kernel after it.
#pragma once

#include "hz_dd.h"
#include "hz_fb_impl.h"
#include "hz_fb_rec.h"

namespace hz_state {

constexpr int kL = 128;             // chunk (samples)
constexpr int kTile = 64 * kL;      // 8192 samples per tile
constexpr int kCols = 32;           // band-state columns per workgroup (two 16-wide MFMA blocks)
constexpr int kKE = 33;             // MFMA k-steps per chunk (132 tap slots)
constexpr int kThreads = 256;       // 4 waves
// A band group's operand block (fb_state_ops_kernel): per band kEs doubles -- pin E_0[i] for
// i < XW (the end-state map's first row: its row k is E_0 shifted by k taps past the O history
// taps), zeros up to kEh, then the history taps pin E_H[k O + i] -- followed by the M^e weights of
// every column: W[sb][col][p][j] = row k of M^e(p) at column k ^ j (j < 4), e(p) = 64 (the tile
// carry), 4, 0..3, 16, 32, 48 (the end's Horner steps), then the low word of M^64 (p = 9: the
// tile carry applies hi + lo, hz_dd.h).  A lane gathers its 66 B operands from
// its band's row (the two state columns of a band share it: 31 KB per group at O = 2 instead of
// the 48 KB of operands laid out per lane)
constexpr int kEh = 136, kEs = 152;
constexpr int kPows = 10;
constexpr int kW = 2 * 16 * kPows * 4;
template <int O>
constexpr int grp_e() { return (kCols / (O == 3 ? 4 : O)) * kEs; }
template <int O>
constexpr int grp_doubles() { return grp_e<O>() + kW; }
inline int grp_doubles(int O) {
    return O == 1 ? grp_doubles<1>() : O == 2 ? grp_doubles<2>() : O == 3 ? grp_doubles<3>() : grp_doubles<4>();
}
__host__ __device__ constexpr int pow_of(int p) { return p == 0 ? 64 : p == 1 ? 4 : p < 6 ? p - 2 : 16 * (p - 5); }

template <int O>
struct StateGeom {
    static constexpr int OP = O == 3 ? 4 : O;       // columns per band
    static constexpr int BANDS = kCols / OP;        // bands per workgroup
    static constexpr int XW = kL + O;               // chunk input taps
    static constexpr int S = O & 1;                 // tap shift: tap pairs 16-B aligned in x
    static_assert(XW + S <= 4 * kKE, "taps fit the k-steps");
    static_assert(4 * kKE - 1 - S + (O - 1) < kEh && kEh + O * O <= kEs, "band row layout");
};

inline int bands_per_group(int O) { return kCols / (O == 3 ? 4 : O); }

// tap slot of k-step q for lane group g (the MFMA's k index within the step)
__host__ __device__ constexpr int tap_slot(int q, int g) { return q < 32 ? 8 * (q >> 1) + 2 * g + (q & 1) : 128 + g; }

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// lane l <- lane (l ^ j) within its quad (DPP quad_perm), j = 1, 2, 3
template <int J>
__device__ __forceinline__ double quad_xor(double v) {
    constexpr int ctrl = J == 1 ? 0xB1 : J == 2 ? 0x4E : 0x1B;
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(b & 0xffffffff), ctrl, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), ctrl, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// sum_j w[j] v_(lane ^ j): a band's O x O matrix row k applied to its state columns
template <int OP>
__device__ __forceinline__ double mix_cols(const double* w, double v) {
    double r = w[0] * v;
    if constexpr (OP >= 2) r = fma(w[1], quad_xor<1>(v), r);
    if constexpr (OP >= 4) {
        r = fma(w[2], quad_xor<2>(v), r);
        r = fma(w[3], quad_xor<3>(v), r);
    }
    return r;
}

// the same with a double-double row (w + wl): the tile carry, applied once per tile
template <int OP>
__device__ __forceinline__ double mix_cols2(const double* w, const double* wl, double v) {
    double x[OP];
    x[0] = v;
    if constexpr (OP >= 2) x[1] = quad_xor<1>(v);
    if constexpr (OP >= 4) {
        x[2] = quad_xor<2>(v);
        x[3] = quad_xor<3>(v);
    }
    double r = wl[0] * x[0];
#pragma unroll
    for (int j = 1; j < OP; ++j) r = fma(wl[j], x[j], r);
#pragma unroll
    for (int j = 0; j < OP; ++j) r = fma(w[j], x[j], r);
    return r;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t state_rsrc(const double* p, long count) {
    const unsigned long long b = (unsigned long long)p;
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane((int)(count * (long)sizeof(double)));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, bytes, 0x00020000);
}

// a lane's 33 A operands of one tile: x[v / 8 + tap_slot(q, g)], v = the byte offset of its chunk's
// first slot (16-B aligned; negative = before the window: out of range, 0)
__device__ __forceinline__ void load_a(__amdgpu_buffer_rsrc_t xr, int v, int g, double (&a)[kKE]) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const u32x4 p = __builtin_amdgcn_raw_buffer_load_b128(xr, v + (int)sizeof(double) * (8 * j + 2 * g), 0, 0);
        a[2 * j] = __builtin_bit_cast(double, ((unsigned long long)p.y << 32) | p.x);
        a[2 * j + 1] = __builtin_bit_cast(double, ((unsigned long long)p.w << 32) | p.z);
    }
    a[32] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, v + (int)sizeof(double) * (128 + g), 0, 0));
}

// one tile of both chains: acc_sb <- (M^64 acc_sb if carry) + sum_q A_q B_{sb,q}; each A pair is
// reloaded with the next tile's taps (byte offset vn) as soon as its two k-steps are issued
template <int OP>
__device__ __forceinline__ void state_tile(double (&a)[kKE], const double (&b)[2][kKE], const double (&m64)[2][OP],
                                           const double (&m64l)[2][OP], bool carry, __amdgpu_buffer_rsrc_t xr, int vn, int g, f64x4& acc0,
                                           f64x4& acc1) {
    if (carry) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            acc0[rr] = mix_cols2<OP>(m64[0], m64l[0], acc0[rr]);
            acc1[rr] = mix_cols2<OP>(m64[1], m64l[1], acc1[rr]);
        }
    }
#pragma unroll
    for (int q = 0; q < kKE; ++q) {
        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[0][q], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[q], b[1][q], acc1, 0, 0, 0);
        if (q & 1) {
            const u32x4 p = __builtin_amdgcn_raw_buffer_load_b128(xr, vn + (int)sizeof(double) * (8 * (q >> 1) + 2 * g), 0, 0);
            a[q - 1] = __builtin_bit_cast(double, ((unsigned long long)p.y << 32) | p.x);
            a[q] = __builtin_bit_cast(double, ((unsigned long long)p.w << 32) | p.z);
        } else if (q == 32) {
            a[32] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, vn + (int)sizeof(double) * (128 + g), 0, 0));
        }
        __builtin_amdgcn_sched_barrier(0);   // keep each reload beside its k-steps (the scheduler
                                             // bunched them at the tile's end: a wait per tile)
    }
}

struct StateArgs {
    const double* rec;     // chunk-128 records [N][rs]
    int rs;                // record size (doubles)
    const double* eop;     // [G][grp_doubles<O>] band rows of pin E, M^e weights (fb_state_ops_kernel)
    const double* x;       // [len] the window
    long len;
    int nbands;
    int G;                 // band groups (workgroups per piece)
    int tps;               // tiles per piece
    int nseg;              // pieces of the window (equal runs of tps tiles)
    double* part;          // [G][nseg][kCols] piece partials (nseg > 1)
    unsigned* count;       // [G] arrival counters (nseg > 1; 0 between launches)
    int deferred;          // nseg > 1 inside another kernel: partials only, combined by a kernel of
                           // its own after it (fb_state_combine_kernel: the agent-scope fences of
                           // the last-arrival combine cost 8 us beside the inverse transforms)
    double* out;           // [N][O]
    long long* stamps;     // (diagnostic builds, -DHZ_DIAG_STAMPS) [pieces][G][4] per-workgroup stamps
};

struct StateLds {
    double red[4][kCols];
    int is_last;
};

// (M^64)^e by squaring in double-double (O x O, row-major; hz_dd.h): the Horner over the pieces
// applies it nseg - 1 times
template <int O>
__device__ __forceinline__ void m64_pow(const double* M64, const double* M64l, int e, double (&P)[O][O],
                                        double (&Pl)[O][O]) {
    hz_dd::dd B[O][O], Cp[O][O];
    hz_dd::load<O>(M64, M64l, B);
    hz_dd::mat_pow<O>(B, e, Cp);
    for (int i = 0; i < O; ++i)
        for (int j = 0; j < O; ++j) {
            P[i][j] = Cp[i][j].hi;
            Pl[i][j] = Cp[i][j].lo;
        }
}

// band b's state from its piece partials p0[s kCols + i]: Horner over the pieces of `tiles` tiles
template <int O>
__device__ __forceinline__ void combine_pieces(const StateArgs& a, int b, const double* p0, int tiles) {
    using R = hz_fbi::RecL<O, kL>;
    const double* rb = a.rec + (long)b * a.rs;
    double S[O], P[O][O], Pl[O][O];
    m64_pow<O>(rb + R::QC + 64 * O * O, rb + R::PSL, tiles, P, Pl);
    for (int i = 0; i < O; ++i) S[i] = p0[i];
    for (int s = 1; s < a.nseg; ++s) {
        const double* ps = p0 + (long)s * kCols;
        double nS[O];
        for (int i = 0; i < O; ++i) {
            double acc2 = ps[i];
            for (int q = 0; q < O; ++q) acc2 = fma(Pl[i][q], S[q], acc2);
            for (int q = 0; q < O; ++q) acc2 = fma(P[i][q], S[q], acc2);
            nS[i] = acc2;
        }
        for (int i = 0; i < O; ++i) S[i] = nS[i];
    }
    for (int i = 0; i < O; ++i) a.out[(long)b * O + i] = S[i];
}

// the workgroup of band group g over piece seg (tiles [seg tps, (seg + 1) tps)); 256 threads
template <int O>
__device__ __forceinline__ void state_group(const StateArgs& a, int g, int seg, StateLds& L) {
    using Gm = StateGeom<O>;
    constexpr int OP = Gm::OP;
    const int lane = threadIdx.x & 63;
    const int m = threadIdx.x >> 6;             // chunk rows 16m .. 16m + 15 of every tile
    const int col = lane & 15;                  // column within a 16-column block
    const int lg = lane >> 4;                   // lane group: the MFMA's k index
    const int pc = seg, ntl = a.tps;
    const __amdgpu_buffer_rsrc_t xr = state_rsrc(a.x, a.len);
#ifdef HZ_DIAG_STAMPS
    long long* stp = a.stamps ? a.stamps + ((long)seg * a.G + g) * 4 : nullptr;
    if (stp && threadIdx.x == 0) {
        stp[0] = __builtin_amdgcn_s_memrealtime();
        stp[3] = ((long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) | __builtin_amdgcn_s_getreg((31 << 11) | 4);
    }
#endif
    // tile it's A offset (bytes) of this lane's chunk 64 it + 16 m + col of the piece
    const long t0 = (long)seg * a.tps * kTile;
    auto voff = [&](int it) {
        return (int)((t0 + (long)it * kTile + (long)(16 * m + col) * kL - O - Gm::S) * (long)sizeof(double));
    };
    // rows k of the band's M^e as weights of the columns k ^ j, from the group's weight block
    // (p: pow_of); buffer loads off the block's resource (32-bit offsets, no address registers)
    constexpr int kGrpO = grp_doubles<O>(), kEO = grp_e<O>();
    const __amdgpu_buffer_rsrc_t er = state_rsrc(a.eop + (long)g * kGrpO, kGrpO);
    auto ld = [&](int i) { return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(er, 8 * i, 0, 0)); };
    auto wrow = [&](int sb, int p, double (&wt)[OP]) {
        const int w = kEO + ((sb * 16 + col) * kPows + p) * 4;
#pragma unroll
        for (int j = 0; j < OP; ++j) wt[j] = ld(w + j);
    };
    // the carry weights first, then tile 0's A operands and every B operand straight into
    // registers in the order the first tile's k-steps use them: its MFMAs start as their operands
    // arrive (a staged LDS copy waited for the whole block behind a barrier: 3.4 us before the
    // first MFMA)
    double m64[2][OP], m64l[2][OP];
    wrow(0, 0, m64[0]);
    wrow(1, 0, m64[1]);
    wrow(0, 9, m64l[0]);
    wrow(1, 9, m64l[1]);
    // B operand (sb, q) of this lane: pin E[k][tap], tap = tap_slot(q, lg) - S, from its band's row
    // (tap >= O: E_0[tap + k]; tap < O: E_H[k O + tap]; columns k >= O and taps < 0: 0)
    const int k = col % OP;
    const double kmask = k < O ? 1.0 : 0.0;
    auto b_idx = [&](int sb, int q) {
        const int row = ((16 * sb + col) / OP) * kEs;
        const int tap = tap_slot(q, lg) - Gm::S;
        if (q >= 2) return row + tap + k;   // tap >= 7 >= O
        return tap < 0 ? row + kEh - 1 : tap < O ? row + kEh + (k < O ? k : 0) * O + tap : row + tap + k;
    };
    double xa[kKE], bq[2][kKE];
    {
        const int v = voff(0);
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const u32x4 pr = __builtin_amdgcn_raw_buffer_load_b128(xr, v + (int)sizeof(double) * (8 * j + 2 * lg), 0, 0);
            xa[2 * j] = __builtin_bit_cast(double, ((unsigned long long)pr.y << 32) | pr.x);
            xa[2 * j + 1] = __builtin_bit_cast(double, ((unsigned long long)pr.w << 32) | pr.z);
            if (j == 0) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    bq[0][u] = ld(b_idx(0, u)) * kmask;
                    bq[1][u] = ld(b_idx(1, u)) * kmask;
                }
            } else {
                // k-steps 2j, 2j + 1 read adjacent row entries: one 16-B load (8-B aligned) per
                // pair keeps the prologue's loads under the 63 a wave can have in flight
#pragma unroll
                for (int sb = 0; sb < 2; ++sb) {
                    const u32x4 pb = __builtin_amdgcn_raw_buffer_load_b128(er, 8 * b_idx(sb, 2 * j), 0, 0);
                    bq[sb][2 * j] = __builtin_bit_cast(double, ((unsigned long long)pb.y << 32) | pb.x) * kmask;
                    bq[sb][2 * j + 1] = __builtin_bit_cast(double, ((unsigned long long)pb.w << 32) | pb.z) * kmask;
                }
            }
        }
        xa[32] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, v + (int)sizeof(double) * (128 + lg), 0, 0));
        bq[0][32] = ld(b_idx(0, 32)) * kmask;
        bq[1][32] = ld(b_idx(1, 32)) * kmask;
    }
    // the carry weights complete here (the oldest loads): redefined by an empty asm, so the loop's
    // waits track only the x loads (the compiler otherwise waited for every load in flight before
    // each carry)
#pragma unroll
    for (int j = 0; j < OP; ++j)
        asm volatile("" : "+v"(m64[0][j]), "+v"(m64[1][j]), "+v"(m64l[0][j]), "+v"(m64l[1][j]));
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
    // tile it from xa, reloaded with tile it + 1 as it goes (past the last tile: unused loads)
#ifdef HZ_DIAG_STAMPS
    if (stp && threadIdx.x == 0) stp[1] = __builtin_amdgcn_s_memrealtime();
#endif
    for (int it = 0; it < ntl; ++it) state_tile<OP>(xa, bq, m64, m64l, it > 0, xr, voff(it + 1), lg, acc0, acc1);
#ifdef HZ_DIAG_STAMPS
    if (stp && threadIdx.x == 0) stp[2] = __builtin_amdgcn_s_memrealtime();
#endif
    // S = sum_c M^(63-c) A_c, lane rows c = 16m + lg + 4 rr, by Horner steps: over rr with M^4
    // (anchored at row 16m + lg + 12), M^(3-lg) (row 16m + 15), the sum over lg, M^(16(3-m))
    // (row 63), then the sum over the row blocks (waves)
    auto finish = [&](int sb, const f64x4& acc) {
        double m4[OP], mg[OP], mw[OP];
        wrow(sb, 1, m4);
        wrow(sb, 2 + (3 - lg), mg);
        wrow(sb, m == 3 ? 2 : 5 + (3 - m), mw);
        double T = acc[0];
#pragma unroll
        for (int rr = 1; rr < 4; ++rr) T = mix_cols<OP>(m4, T) + acc[rr];
        T = mix_cols<OP>(mg, T);
        T += __shfl_xor(T, 16);
        T += __shfl_xor(T, 32);
        const double v = mix_cols<OP>(mw, T);
        if (lane < 16) L.red[m][16 * sb + lane] = v;
    };
    finish(0, acc0);
    finish(1, acc1);
    __syncthreads();
    const int t = threadIdx.x;
    double* prow = a.part + (long)g * a.nseg * kCols;   // this group's piece partials
    if (t < kCols) {
        const double S = ((L.red[0][t] + L.red[1][t]) + L.red[2][t]) + L.red[3][t];
        const int b = g * Gm::BANDS + t / OP, kk = t % OP;
        if (a.nseg == 1) {
            if (b < a.nbands && kk < O) a.out[(long)b * O + kk] = S;
        } else {
            prow[(long)pc * kCols + t] = S;
            if (!a.deferred) __threadfence();   // visible at agent scope before the arrival below
        }
    }
    if (a.nseg == 1 || a.deferred) return;
    // the last workgroup of this band group to arrive combines the partials
    __syncthreads();
    if (t == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.count + g, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        L.is_last = prev == (unsigned)(a.nseg - 1);
    }
    __syncthreads();
    if (!L.is_last) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (t < Gm::BANDS) {
        const int b = g * Gm::BANDS + t;
        if (b < a.nbands) combine_pieces<O>(a, b, prow + t * OP, a.tps);
    }
    if (t == 0) __hip_atomic_store(a.count + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace hz_state

namespace hz_fbi {
// the band-state pass's arguments for a launch inside another kernel (orders <= 2): G nseg extra
// workgroups, workgroup i running state_group<O>(a, i % G, i / G, lds)
int fb_state_chained(hz_fb* h, const double* x, long len, double* out, hz_state::StateArgs* a);
int fb_state_combine(hz_fb* h, const hz_state::StateArgs& a, hipStream_t st);   // after it, when a.nseg > 1
#ifdef HZ_DIAG_STAMPS
void fb_state_stamps_dump(const hz_state::StateArgs& a, int nfft, long call);
#endif
}  // namespace hz_fbi
