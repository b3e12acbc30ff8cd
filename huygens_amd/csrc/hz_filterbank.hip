// hz_filterbank.hip -- Filterbank<double> block engine for MI355X (gfx950).
//
// Replaces src/filterbank.h:16-188 (Filterbank<T>::compute/operator()/tick):
//   pre_n[t] = (1-sp) pin_n + sp pre_n[t-1]                       (172)
//   g_n[t]   = (1-sg) gin_n + sg g_n[t-1]                         (173)
//   y_n[t]   = pre_n[t] * sum_i F[n][i] x[t-i] - sum_k B[n][k] y_n[t-1-k]   (178-179)
//   out[t]   = sum_n dist(y_n[t] g_n[t])                          (130, 138)
//
// Kernel design (DESIGN.md "Filterbank"):
//   * lanes are TIME: lane c of a wave owns samples [16c, 16c+16) of a 1024-sample
//     tile, so the mixdown over bands needs no cross-lane reduction -- each lane
//     accumulates its 16 outputs over the bands the wave visits.
//   * the IIR time recurrence is split into a per-lane zero-state pass (registers),
//     a 64-lane Hillis-Steele scan of the O x O companion-matrix carry (matrix powers
//     M16^(2^s) precomputed per band on the host), and a per-lane fix-up with the
//     per-band homogeneous responses h_k[j] (wave-uniform, scalar loads).
//   * pre/gain smoothing is seeded per lane in closed form pin + sp^t (P0 - pin) and
//     advanced by the reference's own one-pole recurrence inside the chunk.
//   * waves of a workgroup visit different bands of the same tile; their 1024-sample
//     partial mixes are summed through LDS, and one row per band group is written to
//     a partial slab that a second kernel sums (deterministic, no atomics).
//   * a wave walks the tiles of the call sequentially, carrying the band state in
//     registers (readlane of lane 63's scanned end state).
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <chrono>
#include <cstring>
#include <new>
#include <vector>

#include "hz_dd.h"
#include "hz_fb_impl.h"

namespace {

using namespace hz_fbi;

constexpr int kL = 16;            // samples per lane chunk
constexpr int kTile = 64 * kL;    // samples per wave tile (= reference BSIZE 1024)

// Per-band record (doubles), O-dependent layout.
template <int O>
struct Rec {
    static constexpr int B = 0;                  // b[0..O]           feed-forward
    static constexpr int A = O + 1;              // a[0..O-1]         feedback
    static constexpr int H = 2 * O + 1;          // h[k][j] k<O j<16  homogeneous responses
    static constexpr int P = H + kL * O;         // P[s][r][c] s<6    (M16)^(2^s)
    static constexpr int Q = P + 6 * O * O;      // Q[p][r][c] p<16   (M16)^p
    static constexpr int PL = Q + kL * O * O;    // PL[s-4][r][c]     low words of P[4], P[5] (hz_dd.h)
    static constexpr int RAW = PL + 2 * O * O;
    static constexpr int SIZE = (RAW + 7) & ~7;  // 64-B aligned records
};

static int rec_size(int O) {
    switch (O) {
    case 0: return Rec<0>::SIZE;
    case 1: return Rec<1>::SIZE;
    case 2: return Rec<2>::SIZE;
    case 3: return Rec<3>::SIZE;
    default: return Rec<4>::SIZE;
    }
}

struct MixArgs {
    const double* rec;     // [N][REC]
    const double* pin;     // [N]
    const double* gin;     // [N]
    const double* ystate;  // [N][O]  y[-1-k] at call start
    const double* pgstate; // [N][2]  pre, gain at call start
    double* ystate_next;   // end-of-call state: separate buffers (ping-pong), because
    double* pgstate_next;  // other workgroups of the same launch still read the start state
    const double* x;       // [n] device input
    const double* xhist;   // [O] x[-1-k]
    double* xhist_next;    // [O]
    double* partial;       // [G][n_pad]
    double* segstate;      // [N][nseg][O] start state of each time segment (nseg > 1)
    long n;
    long n_pad;
    long seg_len;          // samples per time segment (multiple of kTile)
    int nseg;
    int nbands;
    double sp, sg;         // smoothing coefficients
    double sp_tile, sg_tile;  // sp^1024, sg^1024
    double sp_n, sg_n;     // sp^n, sg^n (final state)
    double dist_param;
};

// LDS layout of one workgroup:
//   xs   : the tile's input x[t0-16 .. t0+1023], padded one slot per 16 samples so
//          lane c's reads (17c + k) hit 64 distinct banks (ds_read_b64)
//   part : [W][16][66] per-wave partial mixes (pad 66: conflict-free ds_write_b64 rows
//          and ds_read_b64 transposed reads)
constexpr int kXsLen = 1040;                     // 16 halo + 1024
constexpr int kXsPad = ((kXsLen + kXsLen / 16) + 1) & ~1;  // 1106 doubles (16-B multiple)

constexpr int kPartPad = 66;
constexpr int kPartWave = kL * kPartPad;
__host__ __device__ constexpr size_t lds_bytes(int waves, bool mix) {
    return sizeof(double) * (2 * kXsPad + (mix ? (size_t)waves * kPartWave : 0));
}
__device__ __forceinline__ int xs_pos(int li) { return li + (li >> 4); }

// MODE_MIX: full pass (zero-state pass, carry scan, fix-up, mixdown) over one
//   time segment (blockIdx.y) of one band group (blockIdx.x).
// MODE_SEGEND: zero-state end state of each segment but the last (no mixdown),
//   feeding fb_seg_carry_kernel when the bank is too small to fill the chip
//   with bands alone (e.g. 512-band shards on 8 GPUs).

// PF (x values prefetched per thread) fixes the workgroup size: 2 -> 16 waves, 3 -> 8, 5 -> 4;
// the launch bound follows it, so 4-wave groups get the whole VGPR file (NB > 1 bands per
// wave interleaved for ILP instead of occupancy).
constexpr int wg_threads(int PF) { return PF == 2 ? 1024 : (PF == 3 ? 512 : 256); }

template <int O, int DIST, int NB, int MODE, int PF>
__global__ __launch_bounds__(wg_threads(PF)) void fb_mix_kernel(const double* __restrict__ rec, MixArgs a) {
    // rec is passed as its own __restrict__ argument so the compiler can prove the
    // kernel's stores never clobber it: wave-uniform record reads become s_load.
    using R = Rec<O>;
    constexpr bool kDistRow = NB == 1 && (DIST == HZ_DIST_SATURATE || DIST == HZ_DIST_LIMITER);
    // (softclip: dist_apply's identity branch inline, its atan tail out of line -- inline, the tail
    // spilled the recurrence registers of every sample: 244 B of scratch per lane, 23.8 GB of
    // scratch traffic per C2 call, 5.9 ms; out of line 80 B, 4.57 ms.  A per-wave max with the tail
    // on the LDS row measured 5.1 ms (its call site, or inlined atan, raised the scratch to 128 /
    // 224 B): profiles/r6/general)
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* part = lds + 2 * kXsPad;  // xs double buffer: lds[0..kXsPad), lds[kXsPad..2 kXsPad)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int W = blockDim.x >> 6;
    const int band0 = (blockIdx.x * W + wave) * NB;
    const long n = a.n;
    const int seg = blockIdx.y;
    const long seg_t0 = (long)seg * a.seg_len;
    const long seg_end = min(seg_t0 + a.seg_len, n);
    const int ntiles = (int)((seg_end - seg_t0 + kTile - 1) / kTile);
    const bool last_seg = seg == a.nseg - 1;
    double* my = part + (long)wave * kPartWave;

    // per-lane smoothing powers sp^(16 lane); the tile factor is wave-uniform
    const double sp_lane = pow(a.sp, (double)(kL * lane));
    const double sg_lane = pow(a.sg, (double)(kL * lane));
    double sp_t = seg_t0 ? uniform(pow(a.sp, (double)seg_t0)) : 1.0;
    double sg_t = seg_t0 ? uniform(pow(a.sg, (double)seg_t0)) : 1.0;

    // carried band state (wave-uniform)
    bool live[NB];
    double S[NB][O > 0 ? O : 1];
    double P0[NB], G0[NB], pin[NB], gin[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const int band = band0 + b;
        live[b] = band < a.nbands;
        const int bb = live[b] ? band : 0;
        const double* s0 = (MODE == MODE_SEGEND) ? nullptr
                         : (seg == 0) ? a.ystate + (long)bb * O
                                      : a.segstate + ((long)bb * a.nseg + seg) * O;
#pragma unroll
        for (int k = 0; k < O; ++k) S[b][k] = (live[b] && s0) ? s0[k] : 0.0;
        P0[b] = live[b] ? a.pgstate[2 * (long)bb] : 0.0;
        G0[b] = live[b] ? a.pgstate[2 * (long)bb + 1] : 0.0;
        pin[b] = live[b] ? a.pin[bb] : 0.0;
        gin[b] = live[b] ? a.gin[bb] : 0.0;
    }

    // input tiles are double-buffered in LDS; tile k+1 is loaded into registers while
    // tile k computes and written to the other buffer before the tile's barrier
    // PF = x values per thread = ceil(1040 / blockDim)
    auto load_x = [&](long t0x, double (&pf)[PF]) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int li = threadIdx.x + q * blockDim.x;
            const long idx = t0x - 16 + li;
            double v = 0.0;
            if (li < kXsLen) {
                if (idx < 0) v = (idx >= -O) ? a.xhist[-idx - 1] : 0.0;
                else if (idx < seg_end) v = a.x[idx];
            }
            pf[q] = v;
        }
    };
    auto store_x = [&](double* xbuf, const double (&pf)[PF]) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int li = threadIdx.x + q * blockDim.x;
            if (li < kXsLen) xbuf[xs_pos(li)] = pf[q];
        }
    };
    {
        double pf0[PF];
        load_x(seg_t0, pf0);
        store_x(lds, pf0);
        __syncthreads();
    }

    for (int tile = 0; tile < ntiles; ++tile) {
        const long t0 = seg_t0 + (long)tile * kTile;  // global sample index of the tile
        const long tc = t0 + (long)kL * lane;
        const bool last_tile = last_seg && tile == ntiles - 1;
        const double* xs = lds + (tile & 1) * kXsPad;
        double pf[PF];
        const bool more = tile + 1 < ntiles;
        if (more) load_x(t0 + kTile, pf);  // in flight during this tile's compute

        // ---- zero-state pass over the lane's 16 samples, all NB bands ----------
        // Fast path once the pre-amp smoother has converged for this tile
        // (sp^t |P0 - pin| <= 2^-60 |pin|: pre == pin to ~1e-18): pin folds into b.
        bool pfast = true, gfast = true;
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            pfast = pfast && (sp_t * fabs(P0[b] - pin[b]) <= 0x1p-60 * fabs(pin[b]));
            gfast = gfast && (sg_t * fabs(G0[b] - gin[b]) <= 0x1p-60 * fabs(gin[b]));
        }
        double zsr[NB][kL];
        auto zsr_pass = [&](auto fast_tag) {
            constexpr bool FAST = decltype(fast_tag)::value;
            double xw[O + 1];  // x[t], x[t-1], ... sliding window
#pragma unroll
            for (int k = 1; k <= O; ++k) xw[k] = xs[17 * lane + 16 - k];
            double pre[NB], bp[NB][O + 1];
            double yh[NB][O > 0 ? O : 1];
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const double* r = rec + (long)(live[b] ? band0 + b : 0) * R::SIZE;
                pre[b] = pin[b] + (sp_lane * sp_t) * (P0[b] - pin[b]);
#pragma unroll
                for (int i = 0; i <= O; ++i) bp[b][i] = FAST ? pin[b] * r[R::B + i] : r[R::B + i];
#pragma unroll
                for (int k = 0; k < O; ++k) yh[b][k] = 0.0;
            }
#pragma unroll
            for (int j = 0; j < kL; ++j) {
                xw[0] = xs[17 * lane + 17 + j];
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    const double* r = rec + (long)(live[b] ? band0 + b : 0) * R::SIZE;
                    double ff = bp[b][0] * xw[0];
#pragma unroll
                    for (int i = 1; i <= O; ++i) ff = fma(bp[b][i], xw[i], ff);
                    double y = ff;
                    if constexpr (!FAST) {
                        pre[b] = fma(a.sp, pre[b], (1.0 - a.sp) * pin[b]);
                        y = ff * pre[b];
                    }
#pragma unroll
                    for (int k = 0; k < O; ++k) y = fma(-r[R::A + k], yh[b][k], y);
#pragma unroll
                    for (int k = O - 1; k > 0; --k) yh[b][k] = yh[b][k - 1];
                    if constexpr (O > 0) yh[b][0] = y;
                    zsr[b][j] = y;
                }
#pragma unroll
                for (int k = O; k > 0; --k) xw[k] = xw[k - 1];
            }
        };
        if (pfast) zsr_pass(std::true_type{});
        else zsr_pass(std::false_type{});

        // ---- carry scan across the 64 chunks of the tile -----------------------
        //   1. intra-row (16 lanes) inclusive scan of the chunk end states with DPP
        //      row_shr 1,2,4,8 (zero fill, no select), matrices M16^(2^s);
        //   2. row totals by v_readlane; the row carries C_0 = S, C_{r+1} =
        //      M16^16 C_r + total_r are wave-uniform (C_4 = the tile end state);
        //   3. chunk start state st(r,p) = Z(r,p-1) + M16^p C_r (row_shr:1 + the
        //      per-band table Q[p] = M16^p).
        double st[NB][O > 0 ? O : 1];
        if constexpr (O > 0) {
            const int row = lane >> 4, p = lane & 15;
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const double* r = rec + (long)(live[b] ? band0 + b : 0) * R::SIZE;
                double qm[O * O];  // this lane's M16^p (issued early, used last)
#pragma unroll
                for (int e = 0; e < O * O; ++e) qm[e] = r[R::Q + p * O * O + e];
                double z[O];
#pragma unroll
                for (int k = 0; k < O; ++k) z[k] = zsr[b][kL - 1 - k];
#define HZ_ROW_STEP(SIDX, D)                                                                 \
    {                                                                                        \
        double nb_[O];                                                                       \
        _Pragma("unroll") for (int k = 0; k < O; ++k) nb_[k] = dpp_d<kDppRowShr + (D)>(z[k]); \
        _Pragma("unroll") for (int rr = 0; rr < O; ++rr)                                     \
            _Pragma("unroll") for (int c = 0; c < O; ++c)                                    \
                z[rr] = fma(r[R::P + (SIDX) * O * O + rr * O + c], nb_[c], z[rr]);           \
    }
                HZ_ROW_STEP(0, 1)
                HZ_ROW_STEP(1, 2)
                HZ_ROW_STEP(2, 4)
                HZ_ROW_STEP(3, 8)
#undef HZ_ROW_STEP
                // row carries (wave-uniform)
                double C[5][O];
#pragma unroll
                for (int k = 0; k < O; ++k) C[0][k] = S[b][k];
#pragma unroll
                for (int rw = 0; rw < 4; ++rw) {
#pragma unroll
                    for (int i = 0; i < O; ++i) {
                        double acc = readlane_d(z[i], 16 * rw + 15);
#pragma unroll
                        for (int q = 0; q < O; ++q) acc = fma(r[R::PL + i * O + q], C[rw][q], acc);
#pragma unroll
                        for (int q = 0; q < O; ++q) acc = fma(r[R::P + 4 * O * O + i * O + q], C[rw][q], acc);
                        C[rw + 1][i] = acc;
                    }
                }
                double Cr[O];
#pragma unroll
                for (int k = 0; k < O; ++k)
                    Cr[k] = row == 0 ? C[0][k] : row == 1 ? C[1][k] : row == 2 ? C[2][k] : C[3][k];
#pragma unroll
                for (int k = 0; k < O; ++k) {
                    double v = dpp_d<kDppRowShr + 1>(z[k]);  // Z(r, p-1), 0 at p == 0
#pragma unroll
                    for (int c = 0; c < O; ++c) v = fma(qm[k * O + c], Cr[c], v);
                    st[b][k] = v;
                }
                // tile end state (the padded tail of a ragged last tile only matters
                // after the final sample, where it is unused)
#pragma unroll
                for (int k = 0; k < O; ++k) S[b][k] = C[4][k];
            }
        }

        if constexpr (MODE == MODE_MIX) {
            // ---- fix-up, gain smoothing and mixdown (bands summed in registers) ---
            // correction c = y - zsr obeys the homogeneous recurrence seeded with the
            // chunk start state: c_j = -sum_k a_k c_{j-1-k}, c_{-1-k} = st[k].
            // Gain fast path once the gain smoother has converged (as for pre).
            auto fix_pass = [&](auto fast_tag) {
                constexpr bool FAST = decltype(fast_tag)::value;
                double g[NB], cr[NB][O > 0 ? O : 1];
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    g[b] = FAST ? gin[b] : gin[b] + (sg_lane * sg_t) * (G0[b] - gin[b]);
#pragma unroll
                    for (int k = 0; k < O; ++k) cr[b][k] = st[b][k];
                }
#pragma unroll
                for (int j = 0; j < kL; ++j) {
                    double v = 0.0;
#pragma unroll
                    for (int b = 0; b < NB; ++b) {
                        const double* r = rec + (long)(live[b] ? band0 + b : 0) * R::SIZE;
                        double y = zsr[b][j];
                        if constexpr (O > 0) {
                            double c = -r[R::A] * cr[b][0];
#pragma unroll
                            for (int k = 1; k < O; ++k) c = fma(-r[R::A + k], cr[b][k], c);
#pragma unroll
                            for (int k = O - 1; k > 0; --k) cr[b][k] = cr[b][k - 1];
                            cr[b][0] = c;
                            y += c;
                        }
                        if constexpr (!FAST) g[b] = fma(a.sg, g[b], (1.0 - a.sg) * gin[b]);
                        double gy = g[b] * y;
                        // (saturate / limiter with one band per wave: on the LDS row below, after the
                        // recurrence registers are dead -- inline here they spilled them: C2 bank
                        // 7.7 -> 4.9 ms per 10 s; softclip's branch runs better inline, 5.4 vs 11.9)
                        if constexpr (DIST != HZ_DIST_NONE && !kDistRow) gy = hz::dist_apply<DIST>(gy, a.dist_param);
                        if constexpr (NB == 1) v = gy;  // a dead wave's row is zeroed below
                        else v += live[b] ? gy : 0.0;
                        zsr[b][j] = y;  // keep y for the end-of-signal state capture
                    }
                    my[j * kPartPad + lane] = v;
                }
            };
            if (gfast) fix_pass(std::true_type{});
            else fix_pass(std::false_type{});
            if (NB == 1 && !live[0]) {  // wave-uniform: padding wave past the last band
#pragma unroll
                for (int j = 0; j < kL; ++j) my[j * kPartPad + lane] = 0.0;
            }
            if constexpr (O > 0) {
                if (last_tile) {  // wave-uniform: y history at the last O samples
                    for (int k = 0; k < O; ++k) {
                        const long t = n - 1 - k;
                        if (t < tc || t >= tc + kL) continue;
                        const int jj = (int)(t - tc);
#pragma unroll
                        for (int b = 0; b < NB; ++b) {
                            if (!live[b]) continue;
                            double y = 0.0;
#pragma unroll
                            for (int j = 0; j < kL; ++j) y = (j == jj) ? zsr[b][j] : y;
                            a.ystate_next[(long)(band0 + b) * O + k] = y;
                        }
                    }
                }
            }
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (!last_tile || lane != 0 || !live[b]) continue;
                const long band = band0 + b;
                if constexpr (O > 0) {
                    // n < O (e.g. per-sample calls): older history entries shift along;
                    // n < O implies one tile, so lane 0's chunk start = call start state
                    if (n < O) {
#pragma unroll
                        for (int k = 0; k < O; ++k)
                            if (k >= n) a.ystate_next[band * O + k] = st[b][k - n];
                    }
                }
                // closed-form end state of the one-pole smoothers after n samples
                a.pgstate_next[2 * band] = pin[b] + a.sp_n * (P0[b] - pin[b]);
                a.pgstate_next[2 * band + 1] = gin[b] + a.sg_n * (G0[b] - gin[b]);
            }

            if constexpr (kDistRow) {   // the same T(*)(T) per sample, from LDS
                for (int j = 0; j < kL; ++j) my[j * kPartPad + lane] = hz::dist_apply<DIST>(my[j * kPartPad + lane], a.dist_param);
            }

            // ---- workgroup reduction of the partial mixes over waves ---------------
            if (more) store_x(lds + ((tile + 1) & 1) * kXsPad, pf);
            __syncthreads();
            for (int tl = threadIdx.x; tl < kTile; tl += blockDim.x) {
                const int src_lane = tl >> 4, j = tl & 15;
                const double* q = part + j * kPartPad + src_lane;
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int w = 0; w < 16; w += 2) {
                    if (w < W) s0 += q[w * kPartWave];
                    if (w + 1 < W) s1 += q[(w + 1) * kPartWave];
                }
                const long t = t0 + tl;
                if (t < n) a.partial[(long)blockIdx.x * a.n_pad + t] = s0 + s1;
            }
        }
        if constexpr (MODE == MODE_SEGEND) {
            if (more) store_x(lds + ((tile + 1) & 1) * kXsPad, pf);
        }
        __syncthreads();  // part is rewritten / the next xs buffer becomes readable
        sp_t *= a.sp_tile;
        sg_t *= a.sg_tile;
    }

    if constexpr (MODE == MODE_SEGEND) {
        // zero-state end state of this segment -> segstate[band][seg + 1] (temporarily;
        // fb_seg_carry_kernel turns it into the true start state of segment seg + 1)
        if (lane == 0 && !last_seg) {
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (!live[b]) continue;
#pragma unroll
                for (int k = 0; k < O; ++k)
                    a.segstate[((long)(band0 + b) * a.nseg + seg + 1) * O + k] = S[b][k];
            }
        }
    } else if constexpr (O > 0) {
        // ---- x history for the next call (ping-pong buffer) ----------------------
        if (last_seg && blockIdx.x == 0 && threadIdx.x < O) {
            const int k = threadIdx.x;
            const long idx = n - 1 - k;
            a.xhist_next[k] = idx >= 0 ? a.x[idx] : a.xhist[-idx - 1];
        }
    }
}

// Sequential carry over time segments, one thread per band:
//   start(s+1) = C^seg_len start(s) + zsr_end(s),  start(0) = ystate.
// C^seg_len = (M16^64)^(seg_len/1024) by binary powering of the record's P[5]^2, in double-double
// and applied as hi S + lo S (hz_dd.h: the same rounded power is applied nseg - 1 times).
template <int O>
__global__ __launch_bounds__(256) void fb_seg_carry_kernel(const double* __restrict__ rec,
                                                           const double* __restrict__ ystate,
                                                           double* __restrict__ segstate, int nbands,
                                                           int nseg, long seg_tiles) {
    using R = Rec<O>;
    using hz_dd::dd;
    const int band = blockIdx.x * blockDim.x + threadIdx.x;
    if (band >= nbands) return;
    const double* r = rec + (long)band * R::SIZE;
    double M[O][O], Ml[O][O];
    {
        dd P5[O][O], M1024[O][O], Cp[O][O];
        hz_dd::load<O>(r + R::P + 5 * O * O, r + R::PL + O * O, P5);
        hz_dd::mat_mul<O>(P5, P5, M1024);
        hz_dd::mat_pow<O>(M1024, seg_tiles, Cp);
        for (int i = 0; i < O; ++i)
            for (int j = 0; j < O; ++j) {
                M[i][j] = Cp[i][j].hi;
                Ml[i][j] = Cp[i][j].lo;
            }
    }
    double S[O];
#pragma unroll
    for (int k = 0; k < O; ++k) S[k] = ystate[(long)band * O + k];
    for (int s = 1; s < nseg; ++s) {
        double* slot = segstate + ((long)band * nseg + s) * O;
        double nS[O];
#pragma unroll
        for (int i = 0; i < O; ++i) {
            double acc = slot[i];
#pragma unroll
            for (int q = 0; q < O; ++q) acc = fma(Ml[i][q], S[q], acc);
#pragma unroll
            for (int q = 0; q < O; ++q) acc = fma(M[i][q], S[q], acc);
            nS[i] = acc;
        }
#pragma unroll
        for (int i = 0; i < O; ++i) {
            S[i] = nS[i];
            slot[i] = nS[i];
        }
    }
}

// out[t] = sum_g partial[g][t]
__global__ __launch_bounds__(256) void fb_reduce_kernel(const double* __restrict__ partial, long n_pad,
                                                        int G, long n, double* __restrict__ out) {
    __shared__ double red[4][64];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const long t = (long)blockIdx.x * 64 + tx;
    double s = 0.0;
    if (t < n)
        for (int g = ty; g < G; g += 4) s += partial[(long)g * n_pad + t];
    red[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && t < n) out[t] = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}

// ---------------------------------------------------------------------------
// host-side precompute of a band record, in double-double (hz_dd.h): the homogeneous responses
// h[k][j], M16, its powers; P[4] and P[5] keep their low words (the carries apply them many times)
// ---------------------------------------------------------------------------
template <int O>
void build_record(const double* b, const double* av, double* rec) {
    using R = Rec<O>;
    using hz_dd::dd;
    std::memset(rec, 0, sizeof(double) * R::SIZE);
    for (int i = 0; i <= O; ++i) rec[R::B + i] = b[i];
    if constexpr (O > 0) {
        for (int k = 0; k < O; ++k) rec[R::A + k] = av[k];
        dd h[O][kL];
        for (int k = 0; k < O; ++k) {
            dd yh[O];
            for (int q = 0; q < O; ++q) yh[q] = {q == k ? 1.0 : 0.0, 0.0};
            for (int j = 0; j < kL; ++j) {
                dd y{0.0, 0.0};
                for (int q = 0; q < O; ++q) y = hz_dd::add(y, hz_dd::mul(yh[q], -av[q]));
                for (int q = O - 1; q > 0; --q) yh[q] = yh[q - 1];
                yh[0] = y;
                h[k][j] = y;
                rec[R::H + k * kL + j] = y.hi;
            }
        }
        dd M[O][O], T[O][O], Qp[O][O];
        for (int rr = 0; rr < O; ++rr)
            for (int c = 0; c < O; ++c) {
                M[rr][c] = h[c][kL - 1 - rr];
                Qp[rr][c] = {rr == c ? 1.0 : 0.0, 0.0};
            }
        for (int p = 0; p < kL; ++p) {
            for (int rr = 0; rr < O; ++rr)
                for (int c = 0; c < O; ++c) rec[R::Q + p * O * O + rr * O + c] = Qp[rr][c].hi;
            hz_dd::mat_mul<O>(Qp, M, T);
            std::memcpy(Qp, T, sizeof(Qp));
        }
        for (int s = 0; s < 6; ++s) {
            for (int rr = 0; rr < O; ++rr)
                for (int c = 0; c < O; ++c) {
                    rec[R::P + s * O * O + rr * O + c] = M[rr][c].hi;
                    if (s >= 4) rec[R::PL + (s - 4) * O * O + rr * O + c] = M[rr][c].lo;
                }
            hz_dd::mat_mul<O>(M, M, T);
            std::memcpy(M, T, sizeof(M));
        }
    }
}

static void build_record_any(int O, const double* b, const double* a, double* rec) {
    switch (O) {
    case 0: build_record<0>(b, a, rec); break;
    case 1: build_record<1>(b, a, rec); break;
    case 2: build_record<2>(b, a, rec); break;
    case 3: build_record<3>(b, a, rec); break;
    default: build_record<4>(b, a, rec); break;
    }
}

typedef void (*MixKernel)(const double*, MixArgs);
typedef void (*CarryKernel)(const double*, const double*, double*, int, int, long);

template <int O, int PF, int NB>
MixKernel pick_dist(int dist, int mode) {
    if (mode == MODE_SEGEND) return fb_mix_kernel<O, HZ_DIST_NONE, NB, MODE_SEGEND, PF>;
    switch (dist) {
    case HZ_DIST_SOFTCLIP: return fb_mix_kernel<O, HZ_DIST_SOFTCLIP, NB, MODE_MIX, PF>;
    case HZ_DIST_SATURATE: return fb_mix_kernel<O, HZ_DIST_SATURATE, NB, MODE_MIX, PF>;
    case HZ_DIST_LIMITER: return fb_mix_kernel<O, HZ_DIST_LIMITER, NB, MODE_MIX, PF>;
    default: return fb_mix_kernel<O, HZ_DIST_NONE, NB, MODE_MIX, PF>;
    }
}

template <int PF, int NB>
MixKernel pick_order(int O, int dist, int mode) {
    switch (O) {
    case 0: return pick_dist<0, PF, NB>(dist, mode);
    case 1: return pick_dist<1, PF, NB>(dist, mode);
    case 2: return pick_dist<2, PF, NB>(dist, mode);
    case 3: return pick_dist<3, PF, NB>(dist, mode);
    default: return pick_dist<4, PF, NB>(dist, mode);
    }
}

// waves per workgroup in {4, 8, 16}: x prefetch depth ceil(1040 / (64 waves)); several
// bands per wave only with 4- or 8-wave groups (register file)
static MixKernel pick_kernel(int O, int dist, int waves, int nb, int mode) {
    switch (waves) {
    case 16: return pick_order<2, 1>(O, dist, mode);
    case 8: return nb == 2 ? pick_order<3, 2>(O, dist, mode) : pick_order<3, 1>(O, dist, mode);
    default:
        if (nb == 4) return pick_order<5, 4>(O, dist, mode);
        if (nb == 2) return pick_order<5, 2>(O, dist, mode);
        return pick_order<5, 1>(O, dist, mode);
    }
}

static CarryKernel pick_carry(int O) {
    switch (O) {
    case 1: return fb_seg_carry_kernel<1>;
    case 2: return fb_seg_carry_kernel<2>;
    case 3: return fb_seg_carry_kernel<3>;
    default: return fb_seg_carry_kernel<4>;
    }
}

}  // namespace

namespace {

int fb_groups(const hz_fb* h) {
    const int per = h->waves * h->bands_per_wave;
    return (h->N + per - 1) / per;
}

int fb_upload(hz_fb* h) {
    bool uploaded = false;
    // LAZY band states of a stationary call follow from the coefficients and pre-amps it ran
    // with: materialise them before new ones reach the device
    if (h->resp.implicit && (h->dirty_coef || h->dirty_pin || h->tv_pending)) HZ_TRY(hz_fbi::fb_resp_materialize(h));
    // gains only, while the bank streams stationary: a transient of the streaming engine instead of
    // a new response and K samples of history (hz_fb_stream.hip fb_stream_gain_setter; its launch
    // also brings the smoothers up to date and writes d_gin)
    const int transient = (h->dirty_gin && !h->dirty_pin && !h->dirty_coef && !h->tv_pending)
                              ? hz_fbi::fb_stream_gain_setter(h) : 0;
    // streamed samples bring the smoothers up to date lazily, toward the targets they ran with:
    // apply them before new targets (mix / boost) reach the device
    if (!transient && (h->dirty_pin || h->dirty_gin)) HZ_TRY(hz_fbi::fb_stream_upkeep(h));
    HZ_TRY(hz_fbi::fb_tv_materialize(h));
    if (h->dirty_coef) {
        const int O = h->order;
        h->h_rec.assign((size_t)h->N * h->rec, 0.0);
        for (int n = 0; n < h->N; ++n)
            build_record_any(O, &h->F[(size_t)n * (O + 1)], O > 0 ? &h->B[(size_t)n * O] : nullptr,
                             &h->h_rec[(size_t)n * h->rec]);
        HZ_TRY_HIP(hipMemcpyAsync(h->d_rec, h->h_rec.data(), sizeof(double) * h->h_rec.size(),
                                  hipMemcpyHostToDevice, h->stream));
        h->dirty_coef = false;
        for (auto& st : h->lti_set) {
            st.dirty = true;
            st.fmix_valid = false;
        }
        hz_fbi::fb_resp_invalidate(h, true);
        uploaded = true;
    }
    if (h->dirty_pin) h->resp.st.rband_valid = false;   // r_n are at pre = pin
    if (h->dirty_pin || h->dirty_gin) {
        for (auto& st : h->lti_set) st.fmix_valid = false;
        if (!transient) hz_fbi::fb_resp_invalidate(h, false);
    }
    if (transient == 1) h->dirty_gin = false;   // the update kernel wrote d_gin: no upload, no synchronisation
    if (h->dirty_pin) {
        HZ_TRY_HIP(hipMemcpyAsync(h->d_pin, h->pin.data(), sizeof(double) * h->N, hipMemcpyHostToDevice,
                                  h->stream));
        h->dirty_pin = false;
        uploaded = true;
    }
    if (h->dirty_gin) {
        HZ_TRY_HIP(hipMemcpyAsync(h->d_gin, h->gin.data(), sizeof(double) * h->N, hipMemcpyHostToDevice,
                                  h->stream));
        h->dirty_gin = false;
        uploaded = true;
    }
    // the uploads read pageable host vectors that setters may change next: make them
    // complete (only when something was uploaded: streaming calls stay asynchronous)
    if (uploaded) HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

// chunk bound so the partial slab stays <= ~1 GiB
long fb_max_chunk(const hz_fb* h) {
    const long G = fb_groups(h);
    long c = (1L << 27) / std::max(1L, G);  // doubles per row
    c = std::max<long>(kTile, (c / kTile) * kTile);
    return c;
}

}  // namespace

namespace hz_fbi {

// five timing events per launch (start, mix start, mix end, reduce start, reduce end)
int fb_prof_events(hz_fb* h, hipEvent_t** e) {
    if (h->ev_used + 5 > h->ev.size()) {
        for (int q = 0; q < 5 * 64; ++q) {
            hipEvent_t ne;
            HZ_TRY_HIP(hz::prof_event_create(&ne));
            h->ev.push_back(ne);
        }
    }
    *e = &h->ev[h->ev_used];
    h->ev_skip.resize(h->ev.size() / 5);
    h->ev_skip[h->ev_used / 5] = 0;
    h->ev_rep.resize(h->ev.size() / 5);
    h->ev_rep[h->ev_used / 5] = 1;
    h->ev_used += 5;
    return HZ_OK;
}

int fb_set_lds_attr(const void* k) {
    static thread_local std::vector<const void*> done;
    if (std::find(done.begin(), done.end(), k) != done.end()) return HZ_OK;
    HZ_TRY_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    done.push_back(k);
    return HZ_OK;
}

// staged setters -> device (the per-sample coefficient path, hz_fb_tv.hip, reads pin / gin)
int fb_upload_staged(hz_fb* h) { return fb_upload(h); }

// host mirror of the closed-form smoother end state written by every launch
// (pgstate_next = pin + sp^n (pre - pin), likewise for the gains)
void fb_mirror_advance(hz_fb* h, long len) { h->mirror_clock += len; }

// pg_host[b] after the d samples since band b was last brought current (its targets unchanged since)
static inline void mirror_apply(hz_fb* h, int b, double spn, double sgn) {
    double& P = h->pg_host[2 * (size_t)b];
    double& G = h->pg_host[2 * (size_t)b + 1];
    P = h->pin[b] + spn * (P - h->pin[b]);
    G = h->gin[b] + sgn * (G - h->gin[b]);
    h->mirror_at[b] = h->mirror_clock;
}

void fb_mirror_sync(hz_fb* h) {
    long last = 0;   // bands synced by one-band setters lag by other counts: powers per distinct lag
    double spn = 1, sgn = 1;
    for (int b = 0; b < h->N; ++b) {
        const long d = h->mirror_clock - h->mirror_at[b];
        if (d == 0) continue;
        if (d != last) {
            spn = (double)powl((long double)h->sp, (long double)d);
            sgn = (double)powl((long double)h->sg, (long double)d);
            last = d;
        }
        mirror_apply(h, b, spn, sgn);
    }
}

void fb_mirror_sync_band(hz_fb* h, int l) {
    if (l < 0) return;
    const long d = h->mirror_clock - h->mirror_at[l];
    if (d == 0) return;
    mirror_apply(h, l, (double)powl((long double)h->sp, (long double)d), (double)powl((long double)h->sg, (long double)d));
}

int fb_launch_general(hz_fb* h, const double* d_in, double* d_out, long n) {
    if (n <= 0) return HZ_OK;
    const int G = fb_groups(h);
    const int O = h->order;
    const long chunk = fb_max_chunk(h);
    const long n_pad_max = std::min<long>(((n + kTile - 1) / kTile) * kTile, chunk);
    const size_t need = (size_t)G * n_pad_max;
    if (need > h->partial_cap) {
        if (h->d_partial) HZ_TRY_HIP(hipFree(h->d_partial));
        h->d_partial = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_partial, sizeof(double) * need));
        h->partial_cap = need;
    }
    MixKernel kmix = pick_kernel(O, h->dist_id, h->waves, h->bands_per_wave, MODE_MIX);
    MixKernel kend = pick_kernel(O, h->dist_id, h->waves, h->bands_per_wave, MODE_SEGEND);
    HZ_TRY(fb_set_lds_attr((const void*)kmix));
    const size_t lds = lds_bytes(h->waves, true);
    const size_t lds_end = lds_bytes(h->waves, false);
    for (long off = 0; off < n; off += chunk) {
        const long len = std::min(chunk, n - off);
        const long ntiles = (len + kTile - 1) / kTile;
        // time segments: enough workgroups to cover every CU at least once
        long nseg = std::max<long>(1, std::min<long>(ntiles, (h->target_groups + G - 1) / G));
        const long seg_tiles = (ntiles + nseg - 1) / nseg;
        nseg = (ntiles + seg_tiles - 1) / seg_tiles;
        if (nseg > 1 && O > 0) {
            const size_t sneed = (size_t)h->N * nseg * O;
            if (sneed > h->seg_cap) {
                if (h->d_seg) HZ_TRY_HIP(hipFree(h->d_seg));
                h->d_seg = nullptr;
                HZ_TRY_HIP(hipMalloc(&h->d_seg, sizeof(double) * sneed));
                h->seg_cap = sneed;
            }
        }
        MixArgs a;
        a.rec = h->d_rec;
        a.pin = h->d_pin;
        a.gin = h->d_gin;
        a.ystate = h->d_ystate[h->scur];
        a.pgstate = h->d_pg[h->scur];
        a.ystate_next = h->d_ystate[h->scur ^ 1];
        a.pgstate_next = h->d_pg[h->scur ^ 1];
        a.x = d_in + off;
        a.xhist = h->d_xhist[h->xcur];
        a.xhist_next = h->d_xhist[h->xcur ^ 1];
        a.partial = h->d_partial;
        a.segstate = h->d_seg;
        a.n = len;
        a.n_pad = ntiles * kTile;
        a.seg_len = seg_tiles * kTile;
        a.nseg = (int)nseg;
        a.nbands = h->N;
        a.sp = h->sp;
        a.sg = h->sg;
        a.sp_tile = (double)powl((long double)h->sp, (long double)kTile);
        a.sg_tile = (double)powl((long double)h->sg, (long double)kTile);
        a.sp_n = (double)powl((long double)h->sp, (long double)len);
        a.sg_n = (double)powl((long double)h->sg, (long double)len);
        a.dist_param = h->dist_param;
        hipEvent_t* e = nullptr;
        if (h->prof) {
            HZ_TRY(fb_prof_events(h, &e));
            HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        }
        if (nseg > 1 && O > 0) {
            // segment end states (zero-state), then the per-band carry over segments
            hipLaunchKernelGGL(kend, dim3(G, (unsigned)(nseg - 1)), dim3(64 * h->waves), lds_end, h->stream,
                               (const double*)h->d_rec, a);
            HZ_TRY_HIP(hipGetLastError());
            hipLaunchKernelGGL(pick_carry(O), dim3((unsigned)((h->N + 255) / 256)), dim3(256), 0, h->stream,
                               (const double*)h->d_rec, (const double*)h->d_ystate[h->scur], h->d_seg, h->N, (int)nseg,
                               seg_tiles);
            HZ_TRY_HIP(hipGetLastError());
        }
        if (e) HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
        hipLaunchKernelGGL(kmix, dim3(G, (unsigned)nseg), dim3(64 * h->waves), lds, h->stream,
                           (const double*)h->d_rec, a);
        HZ_TRY_HIP(hipGetLastError());
        if (e) HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
        if (e) HZ_TRY_HIP(hipEventRecord(e[3], h->stream));
        hipLaunchKernelGGL(fb_reduce_kernel, dim3((unsigned)((len + 63) / 64)), dim3(256), 0, h->stream,
                           (const double*)h->d_partial, a.n_pad, G, len, d_out + off);
        HZ_TRY_HIP(hipGetLastError());
        if (e) HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
        h->xcur ^= 1;
        h->scur ^= 1;
        h->prof_launches += h->prof ? 1 : 0;
        fb_mirror_advance(h, len);
    }
    return HZ_OK;
}

}  // namespace hz_fbi

namespace {

// hz_fb_tick: the ring rotation of a tick() without compute (filterbank.h:142-148).  New
// history = (spare row, cur[0 .. O-2]) into the other buffer; the smoothers are copied
// unchanged.  The other buffer's oldest row is the spare and is read before it is overwritten.
__global__ __launch_bounds__(256) void fb_tick_kernel(const double* __restrict__ ycur, double* __restrict__ yoth,
                                                      const double* __restrict__ pgcur, double* __restrict__ pgoth,
                                                      const double* __restrict__ xcur, double* __restrict__ xoth,
                                                      int N, int O) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < N) {
        const double spare = yoth[(long)b * O + O - 1];
        for (int k = O - 1; k >= 1; --k) yoth[(long)b * O + k] = ycur[(long)b * O + k - 1];
        yoth[(long)b * O] = spare;
        pgoth[2 * (long)b] = pgcur[2 * (long)b];
        pgoth[2 * (long)b + 1] = pgcur[2 * (long)b + 1];
    }
    if (b == 0) {
        const double spare = xoth[O - 1];
        for (int k = O - 1; k >= 1; --k) xoth[k] = xcur[k - 1];
        xoth[0] = spare;
    }
}

int fb_launch(hz_fb* h, const double* d_in, double* d_out, long n) {
    if (n <= 0) return HZ_OK;
    h->spare_ok = n == 1;   // one launch, one state flip: the pre-call state is the spare row
    h->last_path = HZ_FB_PATH_GENERAL;
    const int geom = fb_lti_geom(h, n);
    const int L = fb_lti_chunk(geom);
    const long n_lti = n - n % L;
    // converged for the whole call (the smoothers only get closer): the LTI engine may run, and
    // the stationary engine's history keeps counting
    const bool conv = h->order > 0 && n >= 16 && fb_converged(h);
    // a gain transient streams with the gains still moving (hz_fb_stream.hip)
    const bool sconv = conv || (h->order > 0 && fb_stream_dmode(h));
    // a time-sharded handle (multi-GPU) runs stationary exactly when the caller armed it on
    // every rank; an armed handle that cannot (its history is short, or a setter or short call
    // intervened) fails loudly instead of leaving its peers on another engine
    const bool tshard = fb_resp_time_sharded(h);
    // 1024-sample blocks of a stationary bank: one launch each (hz_fb_stream.hip)
    if (!tshard && fb_stream_eligible(h, n, sconv)) {
        HZ_TRY(fb_launch_stream(h, d_in, d_out, n));
        h->last_path = HZ_FB_PATH_STREAM;
        return HZ_OK;
    }
    const bool elig = fb_resp_eligible(h, n, conv);
    if (tshard && h->resp.armed && !elig) {
        hz::set_error("hz_fb_process: time-sharded handle armed for the stationary engine, but this call "
                      "of %ld samples is not stationary here (re-arm after hz_fb_stationary_ready)", n);
        return HZ_E_STATE;
    }
    if (elig && (!tshard || h->resp.armed)) {
        HZ_TRY(fb_launch_resp(h, d_in, d_out, n));
        h->last_path = HZ_FB_PATH_RESPONSE;
        return HZ_OK;
    }
    HZ_TRY(fb_resp_materialize(h));   // LAZY band states of an earlier stationary call
    if (h->path_mode == HZ_FB_PATH_AUTO && h->dist_id == HZ_DIST_NONE && n_lti > 0 && conv) {
        HZ_TRY(fb_launch_lti(h, geom, d_in, d_out, n_lti));
        h->last_path = HZ_FB_PATH_LTI;
        HZ_TRY(fb_launch_general(h, d_in + n_lti, d_out + n_lti, n - n_lti));
    } else {
        HZ_TRY(fb_launch_general(h, d_in, d_out, n));
    }
    return fb_resp_track(h, d_in, n, conv);
}

int fb_check(hz_fb* h) {
    if (!h) {
        hz::set_error("null hz_fb handle");
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipSetDevice(h->device));
    // every device-side use of the state needs it back from the per-sample engine
    return hz_fbi::fb_rt_stop(h);
}


// global band index -> local, or -1 when outside this shard
int fb_local(const hz_fb* h, int n) {
    if (n < h->band_begin || n >= h->band_begin + h->N) return -1;
    return n - h->band_begin;
}

}  // namespace

namespace hz_fbi {
int fb_tick_rotate(hz_fb* h) {
    const int O = h->order;
    if (O == 0) return HZ_OK;   // one-row rings: origin stays 0, nothing moves
    if (!h->spare_ok) {
        hz::set_error("hz_fb_tick: tick() without operator() after a block call or set_state: the ring row "
                      "it would reuse (O+1 samples back) is not kept");
        return HZ_E_STATE;
    }
    HZ_TRY(hz_fbi::fb_resp_materialize(h));
    h->resp.run = 0;   // the rotation reuses a stale row: no longer the response of the inputs
    hz_fbi::fb_stream_reset(h);
    const int N = h->N;
    hipLaunchKernelGGL(fb_tick_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, h->stream,
                       (const double*)h->d_ystate[h->scur], h->d_ystate[h->scur ^ 1], (const double*)h->d_pg[h->scur],
                       h->d_pg[h->scur ^ 1], (const double*)h->d_xhist[h->xcur], h->d_xhist[h->xcur ^ 1], N, O);
    HZ_TRY_HIP(hipGetLastError());
    h->scur ^= 1;
    h->xcur ^= 1;
    return HZ_OK;
}
}  // namespace hz_fbi

extern "C" {

int hz_fb_create_shard(int order, int N_total, int band_begin, int band_count, double k_p, double k_g,
                       int device, hz_fb** out) {
    if (!out || order < 0 || order > kMaxOrder || N_total <= 0 || band_begin < 0 || band_count <= 0 ||
        band_begin + band_count > N_total) {
        hz::set_error("hz_fb_create: invalid arguments (order %d, N %d, shard [%d,+%d))", order, N_total,
                      band_begin, band_count);
        return HZ_E_INVALID;
    }
    *out = nullptr;
    HZ_TRY(hz::select_device(device));
    hz_fb* h = new (std::nothrow) hz_fb();
    if (!h) return HZ_E_ALLOC;
    h->order = order;
    h->N = band_count;
    h->N_total = N_total;
    h->band_begin = band_begin;
    h->device = device;
    h->sp = hz::relaxation(k_p);
    h->sg = hz::relaxation(k_g);
    h->rec = rec_size(order);
    const size_t N = band_count;
    h->F.assign(N * (order + 1), 0.0);
    h->B.assign(N * std::max(order, 1), 0.0);
    h->pin.assign(N, 0.0);
    h->gin.assign(N, 0.0);
    h->pg_host.assign(2 * N, 0.0);
    h->mirror_at.assign(N, 0);
    h->rt.mark.assign(N, 0);
    hz_fbi::fb_resp_init(h);
    // default geometry: 16 waves x 1 band; fewer waves when the bank is small
    h->waves = 16;
    h->bands_per_wave = 1;
    while (h->waves > 4 && (long)fb_groups(h) * h->waves < 1024 && h->waves * 2 > band_count) h->waves /= 2;
    auto fail = [&](int code) {
        hz_fb_destroy(h);
        return code;
    };
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        hz::set_error("hipStreamCreate failed");
        return fail(HZ_E_HIP);
    }
    h->own_stream = true;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            h->target_groups = prop.multiProcessorCount;
    }
    const int O = std::max(order, 1);
    if (hipMalloc(&h->d_rec, sizeof(double) * N * h->rec) != hipSuccess ||
        hipMalloc(&h->d_pin, sizeof(double) * N) != hipSuccess ||
        hipMalloc(&h->d_gin, sizeof(double) * N) != hipSuccess ||
        hipMalloc(&h->d_ystate[0], sizeof(double) * N * O) != hipSuccess ||
        hipMalloc(&h->d_ystate[1], sizeof(double) * N * O) != hipSuccess ||
        hipMalloc(&h->d_pg[0], sizeof(double) * N * 2) != hipSuccess ||
        hipMalloc(&h->d_pg[1], sizeof(double) * N * 2) != hipSuccess ||
        hipMalloc(&h->d_xhist[0], sizeof(double) * O) != hipSuccess ||
        hipMalloc(&h->d_xhist[1], sizeof(double) * O) != hipSuccess) {
        hz::set_error("hipMalloc failed for filterbank state (%zu bands)", N);
        return fail(HZ_E_ALLOC);
    }
    if (hipMemsetAsync(h->d_ystate[0], 0, sizeof(double) * N * O, h->stream) != hipSuccess ||
        hipMemsetAsync(h->d_ystate[1], 0, sizeof(double) * N * O, h->stream) != hipSuccess ||
        hipMemsetAsync(h->d_pg[0], 0, sizeof(double) * N * 2, h->stream) != hipSuccess ||
        hipMemsetAsync(h->d_pg[1], 0, sizeof(double) * N * 2, h->stream) != hipSuccess ||
        hipMemsetAsync(h->d_xhist[0], 0, sizeof(double) * O, h->stream) != hipSuccess ||
        hipMemsetAsync(h->d_xhist[1], 0, sizeof(double) * O, h->stream) != hipSuccess ||
        hipStreamSynchronize(h->stream) != hipSuccess) {
        hz::set_error("hipMemset failed for filterbank state");
        return fail(HZ_E_HIP);
    }
    *out = h;
    return HZ_OK;
}

int hz_fb_create(int order, int N, double k_p, double k_g, int device, hz_fb** out) {
    return hz_fb_create_shard(order, N, 0, N, k_p, k_g, device, out);
}

int hz_fb_destroy(hz_fb* h) {
    if (!h) return HZ_OK;
    (void)hipSetDevice(h->device);
    h->rt.pending_ticks = 0;
    (void)hz_fbi::fb_rt_stop(h);   // the resident per-sample kernel leaves before the buffers go
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    hz_fbi::fb_rt_free(h);
    for (double* p : {h->d_rec, h->d_pin, h->d_gin, h->d_ystate[0], h->d_ystate[1], h->d_pg[0], h->d_pg[1],
                      h->d_xhist[0], h->d_xhist[1],
                      h->d_partial, h->d_seg, h->d_in, h->d_out})
        if (p) (void)hipFree(p);
    for (auto& st : h->lti_set)
        for (double* p : {st.d_rec, st.d_fmix, st.d_kt})
            if (p) (void)hipFree(p);
    if (h->stream_red) (void)hipStreamSynchronize(h->stream_red);
    for (hipEvent_t e : h->ev) (void)hipEventDestroy(e);
    for (hipEvent_t e : h->sync_ev) (void)hipEventDestroy(e);
    if (h->stream_red) (void)hipStreamDestroy(h->stream_red);
    if (h->d_xhist_red) (void)hipFree(h->d_xhist_red);
    if (h->tv_row) (void)hipHostFree(h->tv_row);
    if (h->pin_io) (void)hipHostFree(h->pin_io);
    if (h->tv_ev) (void)hipEventDestroy(h->tv_ev);
    hz_fbi::fb_resp_free(h);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return HZ_OK;
}

int hz_fb_coefficients(hz_fb* h, int n, const double* fwd, int nf, const double* back, int nb) {
    if (!h || (nf > 0 && !fwd) || (nb > 0 && !back) || nf < 0 || nb < 0) {
        hz::set_error("hz_fb_coefficients: invalid arguments");
        return HZ_E_INVALID;
    }
    hz_fbi::HandleLock lk(h);
    ++h->coef_gen;
    h->setter_seq = h->rt.seq;
    hz_fbi::fb_resp_setter(h);
    if (n < 0 || n >= h->N_total) {
        hz::set_error("hz_fb_coefficients: band %d out of range [0,%d)", n, h->N_total);
        return HZ_E_RANGE;
    }
    const int l = fb_local(h, n);
    if (l < 0) return HZ_OK;
    HZ_TRY(hz_fbi::fb_tv_materialize(h));
    const int O = h->order;
    for (int i = 0; i < std::min(O + 1, nf); ++i) h->F[(size_t)l * (O + 1) + i] = fwd[i];
    for (int i = 0; i < std::min(O, nb); ++i) h->B[(size_t)l * O + i] = back[i];
    h->dirty_coef = true;
    return HZ_OK;
}

int hz_fb_boost(hz_fb* h, int n, double v) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    h->setter_seq = h->rt.seq;
    hz_fbi::fb_resp_setter(h);
    h->converged = false;
    if (n < 0 || n >= h->N_total) {
        hz::set_error("hz_fb_boost: band %d out of range [0,%d)", n, h->N_total);
        return HZ_E_RANGE;
    }
    const int l = fb_local(h, n);
    hz_fbi::fb_mirror_sync_band(h, l);   // band l's device smoothers ran on its old targets until now
    hz_fbi::fb_rt_target_setter(h, l);
    if (l >= 0) {
        h->pin[l] = v;
        h->dirty_pin = true;
    }
    return HZ_OK;
}

int hz_fb_boost_all(hz_fb* h, const double* v, int count) {
    if (!h || (count > 0 && !v) || count < 0) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    hz_fbi::fb_rt_target_setter(h, hz_fbi::kAllBands);
    h->setter_seq = h->rt.seq;
    hz_fbi::fb_resp_setter(h);
    fb_mirror_sync(h);  // the device smoothers ran on the old targets until now
    h->converged = false;
    for (int i = 0; i < std::min(h->N_total, count); ++i) {
        const int l = fb_local(h, i);
        if (l >= 0) h->pin[l] = v[i];
    }
    h->dirty_pin = true;
    return HZ_OK;
}

int hz_fb_mix(hz_fb* h, int n, double v) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    h->setter_seq = h->rt.seq;
    hz_fbi::fb_resp_setter(h);
    h->converged = false;
    if (n < 0 || n >= h->N_total) {
        hz::set_error("hz_fb_mix: band %d out of range [0,%d)", n, h->N_total);
        return HZ_E_RANGE;
    }
    const int l = fb_local(h, n);
    hz_fbi::fb_mirror_sync_band(h, l);   // band l's device smoothers ran on its old targets until now
    hz_fbi::fb_rt_target_setter(h, l);
    if (l >= 0) {
        h->gin[l] = v;
        h->dirty_gin = true;
    }
    return HZ_OK;
}

int hz_fb_mix_all(hz_fb* h, const double* v, int count) {
    if (!h || (count > 0 && !v) || count < 0) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    hz_fbi::fb_rt_target_setter(h, hz_fbi::kAllBands);
    h->setter_seq = h->rt.seq;
    hz_fbi::fb_resp_setter(h);
    fb_mirror_sync(h);  // the device smoothers ran on the old targets until now
    h->converged = false;
    for (int i = 0; i < std::min(h->N_total, count); ++i) {
        const int l = fb_local(h, i);
        if (l >= 0) h->gin[l] = v[i];
    }
    h->dirty_gin = true;
    return HZ_OK;
}

int hz_fb_open(hz_fb* h) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    hz_fbi::fb_rt_target_setter(h, hz_fbi::kAllBands);
    h->setter_seq = h->rt.seq;
    hz_fbi::fb_resp_setter(h);
    fb_mirror_sync(h);  // the device smoothers ran on the old targets until now
    h->converged = false;
    std::fill(h->gin.begin(), h->gin.end(), 1.0);
    h->dirty_gin = true;
    return HZ_OK;
}

int hz_fb_set_distortion(hz_fb* h, int dist_id, double param) {
    if (!h || dist_id < HZ_DIST_NONE || dist_id > HZ_DIST_LIMITER) {
        hz::set_error("hz_fb_set_distortion: unknown functor %d", dist_id);
        return HZ_E_INVALID;
    }
    hz_fbi::HandleLock lk(h);
    h->dist_id = dist_id;
    h->dist_param = param;
    return HZ_OK;
}

int hz_fb_process_device(hz_fb* h, const double* d_in, double* d_out, size_t n) {
    if (n == 0) return HZ_OK;
    if (!h || !d_in || !d_out) {
        hz::set_error("hz_fb_process_device: null handle or buffer");
        return HZ_E_INVALID;
    }
    hz_fbi::HandleLock lk(h);
    if (h->rt.computed) {   // the cached sample first (fb_rt_resolve), copied from pinned memory
        HZ_TRY_HIP(hipSetDevice(h->device));
        double y0 = 0;
        const int k = hz_fbi::fb_rt_resolve(h, &y0);
        if (k < 0) return k;
        double* pin0 = hz_fbi::fb_rt_cached_slot(h);
        *pin0 = y0;
        HZ_TRY_HIP(hipMemcpyAsync(d_out, pin0, sizeof(double), hipMemcpyHostToDevice, h->stream));
        ++d_in;
        ++d_out;
        if (--n == 0) return HZ_OK;
    }
    HZ_TRY(fb_check(h));
    HZ_TRY(fb_upload(h));
    return fb_launch(h, d_in, d_out, (long)n);
}

int hz_fb_process(hz_fb* h, const double* in, double* out, size_t n) {
    if (n == 0) return HZ_OK;
    if (!h || !in || !out) {
        hz::set_error("hz_fb_process: null handle or buffer");
        return HZ_E_INVALID;
    }
    hz_fbi::HandleLock lk(h);
    if (h->rt.computed) {   // the cached sample first (fb_rt_resolve)
        HZ_TRY_HIP(hipSetDevice(h->device));
        const int k = hz_fbi::fb_rt_resolve(h, out);
        if (k < 0) return k;
        ++in;
        ++out;
        if (--n == 0) return HZ_OK;
    }
    HZ_TRY(fb_check(h));
    if (n > h->io_cap) {
        if (h->d_in) HZ_TRY_HIP(hipFree(h->d_in));
        if (h->d_out) HZ_TRY_HIP(hipFree(h->d_out));
        h->d_in = h->d_out = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_in, sizeof(double) * n));
        HZ_TRY_HIP(hipMalloc(&h->d_out, sizeof(double) * n));
        h->io_cap = n;
    }
    HZ_TRY(fb_upload(h));
    // a block the streaming engine takes (the reference's 1024-sample callback): its one kernel is
    // the only reader of the input and writer of the output, so it reads and writes pinned,
    // device-mapped staging directly -- two host copies of 8 KB instead of two DMA transfers
    if ((long)n == kStreamBlock && !fb_resp_time_sharded(h) &&
        fb_stream_eligible(h, (long)n, h->order > 0 && fb_converged(h))) {
        const int nwg = hz_fbi::fb_stream_workgroups();
        if (!h->pin_io) {
            HZ_TRY_HIP(hipHostMalloc((void**)&h->pin_io, sizeof(double) * (2 * kStreamBlock + 256),
                                     hipHostMallocCoherent | hipHostMallocMapped));
            std::memset(h->pin_io + 2 * kStreamBlock, 0, sizeof(double) * 256);
        }
        void* dio = nullptr;
        HZ_TRY_HIP(hipHostGetDevicePointer(&dio, h->pin_io, 0));
        long long* hflags = (long long*)(h->pin_io + 2 * kStreamBlock);
        std::memcpy(h->pin_io, in, sizeof(double) * n);
        hz_fb::Resp::Stream& S = h->resp.st;
        S.flags_dev = (long long*)((double*)dio + 2 * kStreamBlock);
        S.flags_seq = ++h->pin_seq;
        const int rc = fb_launch(h, (const double*)dio, (double*)dio + kStreamBlock, (long)n);
        S.flags_dev = nullptr;
        HZ_TRY(rc);
        if (h->last_path == HZ_FB_PATH_STREAM && nwg <= 256) {   // (256 flag slots)
            // every workgroup has read the input and written the output: no stream synchronisation
            // (a fault or a lost flag falls back to it after 1 s and reports the stream's error)
            const auto t0 = std::chrono::steady_clock::now();
            bool done = false;
            while (!done) {
                done = true;
                for (int g = 0; g < nwg && done; ++g) done = __atomic_load_n(hflags + g, __ATOMIC_ACQUIRE) >= S.flags_seq;
                if (!done && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
                    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
                    break;
                }
            }
        } else {
            HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        }
        std::memcpy(out, h->pin_io + kStreamBlock, sizeof(double) * n);
        return HZ_OK;
    }
    HZ_TRY_HIP(hipMemcpyAsync(h->d_in, in, sizeof(double) * n, hipMemcpyHostToDevice, h->stream));
    HZ_TRY(fb_launch(h, h->d_in, h->d_out, (long)n));
    HZ_TRY_HIP(hipMemcpyAsync(out, h->d_out, sizeof(double) * n, hipMemcpyDeviceToHost, h->stream));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_fb_set_stream(hz_fb* h, void* s) {
    HZ_TRY(fb_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->own_stream) HZ_TRY_HIP(hipStreamDestroy(h->stream));
    if (s) {
        h->stream = (hipStream_t)s;
        h->own_stream = false;
    } else {
        HZ_TRY_HIP(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->own_stream = true;
    }
    return HZ_OK;
}

int hz_fb_get_stream(hz_fb* h, void** s) {
    if (!h || !s) return HZ_E_INVALID;
    *s = (void*)h->stream;
    return HZ_OK;
}

int hz_fb_synchronize(hz_fb* h) {
    HZ_TRY(fb_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    return HZ_OK;
}

int hz_fb_state_size(hz_fb* h, size_t* count) {
    if (!h || !count) return HZ_E_INVALID;
    *count = (size_t)h->order + (size_t)h->N * h->order + (size_t)h->N * 2;
    return HZ_OK;
}

int hz_fb_get_state(hz_fb* h, double* buf, size_t count) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    HZ_TRY(fb_check(h));
    size_t need;
    hz_fb_state_size(h, &need);
    if (!buf || count < need) return HZ_E_INVALID;
    const size_t O = h->order, N = h->N;
    HZ_TRY(hz_fbi::fb_resp_materialize(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (O) {
        HZ_TRY_HIP(hipMemcpy(buf, h->d_xhist[h->xcur], sizeof(double) * O, hipMemcpyDeviceToHost));
        HZ_TRY_HIP(hipMemcpy(buf + O, h->d_ystate[h->scur], sizeof(double) * N * O, hipMemcpyDeviceToHost));
    }
    HZ_TRY_HIP(hipMemcpy(buf + O + N * O, h->d_pg[h->scur], sizeof(double) * N * 2, hipMemcpyDeviceToHost));
    return HZ_OK;
}

int hz_fb_set_state(hz_fb* h, const double* buf, size_t count) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    HZ_TRY(fb_check(h));
    size_t need;
    hz_fb_state_size(h, &need);
    if (!buf || count < need) return HZ_E_INVALID;
    const size_t O = h->order, N = h->N;
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (O) {
        HZ_TRY_HIP(hipMemcpy(h->d_xhist[h->xcur], buf, sizeof(double) * O, hipMemcpyHostToDevice));
        HZ_TRY_HIP(hipMemcpy(h->d_ystate[h->scur], buf + O, sizeof(double) * N * O, hipMemcpyHostToDevice));
    }
    HZ_TRY_HIP(hipMemcpy(h->d_pg[h->scur], buf + O + N * O, sizeof(double) * N * 2, hipMemcpyHostToDevice));
    std::memcpy(h->pg_host.data(), buf + O + N * O, sizeof(double) * N * 2);
    std::fill(h->mirror_at.begin(), h->mirror_at.end(), h->mirror_clock);
    h->converged = false;
    h->spare_ok = false;
    h->resp.implicit = false;   // overwritten
    h->resp.run = 0;
    hz_fbi::fb_stream_reset(h);
    return HZ_OK;
}

int hz_fb_tick(hz_fb* h) {
    if (!h) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    HZ_TRY(fb_check(h));
    return hz_fbi::fb_tick_rotate(h);
}


int hz_fb_setter_seq(hz_fb* h, long long* seq) {
    if (!h || !seq) return HZ_E_INVALID;
    hz_fbi::HandleLock lk(h);
    *seq = h->setter_seq;
    return HZ_OK;
}

int hz_fb_info(hz_fb* h, int* order, int* N_local, int* band_begin, int* N_total) {
    if (!h) return HZ_E_INVALID;
    if (order) *order = h->order;
    if (N_local) *N_local = h->N;
    if (band_begin) *band_begin = h->band_begin;
    if (N_total) *N_total = h->N_total;
    return HZ_OK;
}

int hz_fb_tune(hz_fb* h, int waves_per_group, int bands_per_wave) {
    if (!h) return HZ_E_INVALID;
    const int w = waves_per_group ? waves_per_group : h->waves;
    const int nb = bands_per_wave ? bands_per_wave : (waves_per_group ? 1 : h->bands_per_wave);
    if (!(w == 4 || w == 8 || w == 16) || !(nb == 1 || (w == 4 && (nb == 2 || nb == 4)) || (w == 8 && nb == 2))) {
        hz::set_error("hz_fb_tune: waves in {4,8,16}; bands per wave 1, 2 (4 or 8 waves) or 4 (4 waves)");
        return HZ_E_INVALID;
    }
    h->waves = w;
    h->bands_per_wave = nb;
    return HZ_OK;
}

int hz_fb_set_target_groups(hz_fb* h, int groups) {
    if (!h || groups < 1) return HZ_E_INVALID;
    h->target_groups = groups;
    return HZ_OK;
}

int hz_fb_set_path(hz_fb* h, int path) {
    if (!h || (path != HZ_FB_PATH_AUTO && path != HZ_FB_PATH_GENERAL)) {
        hz::set_error("hz_fb_set_path: path must be HZ_FB_PATH_AUTO or HZ_FB_PATH_GENERAL");
        return HZ_E_INVALID;
    }
    h->path_mode = path;
    return HZ_OK;
}

int hz_fb_last_path(hz_fb* h, int* path) {
    if (!h || !path) return HZ_E_INVALID;
    *path = h->last_path;
    return HZ_OK;
}

int hz_fb_profile(hz_fb* h, int enable) {
    HZ_TRY(fb_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    h->prof = enable != 0;
    h->prof_rep = enable > 1 ? std::min(enable, 64) : 1;
    h->ev_used = 0;
    h->prof_launches = 0;
    return HZ_OK;
}

int hz_fb_profile_read(hz_fb* h, double* segment_ms, double* mix_ms, double* reduce_ms, long* launches) {
    HZ_TRY(fb_check(h));
    HZ_TRY_HIP(hipStreamSynchronize(h->stream));
    if (h->stream_red) HZ_TRY_HIP(hipStreamSynchronize(h->stream_red));
    double sg = 0, m = 0, r = 0;
    for (size_t i = 0; i + 5 <= h->ev_used; i += 5) {
        float a = 0, b = 0, c = 0;
        const unsigned char skip = h->ev_skip[i / 5];
        const hipEvent_t e1 = (skip & 2) ? h->ev[i] : h->ev[i + 1];
        const hipEvent_t e3 = (skip & 8) ? h->ev[i + 2] : h->ev[i + 3];
        if (!(skip & 2)) HZ_TRY_HIP(hipEventElapsedTime(&a, h->ev[i], e1));
        HZ_TRY_HIP(hipEventElapsedTime(&b, e1, h->ev[i + 2]));
        HZ_TRY_HIP(hipEventElapsedTime(&c, e3, h->ev[i + 4]));
        const double rep = h->ev_rep.size() > i / 5 ? (double)h->ev_rep[i / 5] : 1.0;
        sg += a / rep;
        m += b / rep;
        r += c / rep;
    }
    if (segment_ms) *segment_ms = sg;
    if (mix_ms) *mix_ms = m;
    if (reduce_ms) *reduce_ms = r;
    if (launches) *launches = h->prof_launches;
    return HZ_OK;
}

}  // extern "C"
