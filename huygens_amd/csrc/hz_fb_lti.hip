// hz_fb_lti.hip -- the converged ("LTI") path of the Filterbank<double> engine.
//
// When every band's pre-amp and gain smoother has converged to its target
// (src/filterbank.h:172-173 one-pole recurrences; |pre - pin| <= 2^-60 max|pin|,
// likewise for the gains) and no distortion functor is selected, the bank is a
// sum of N linear time-invariant biquads driven by ONE shared input:
//
//   y_n[t] = pin_n sum_i b_n[i] x[t-i] - sum_k a_n[k] y_n[t-1-k]      (178-179)
//   out[t] = sum_n gin_n y_n[t]                                       (130)
//
// Split every 64-lane tile into lane chunks of L samples.  For the chunk
// starting at tc with start state s_n = (y_n[tc-1], ..., y_n[tc-O]):
//
//   y_n[tc+j] = pin_n sum_i F_n[j][i] x[tc-O+i]  +  sum_k K_n[j][k] s_n[k]
//
// (F_n: zero-state response of the chunk to its L+O input taps, K_n: homogeneous
// response).  Summing over bands,
//
//   out[tc+j] = sum_i Fmix[j][i] x[tc-O+i]  +  sum_n sum_k K_n[j][k] (gin_n s_n[k])
//
// with Fmix = sum_n gin_n pin_n F_n -- ONE L x (L+O) matrix for the whole bank,
// applied in the reduce kernel.  Per band the mix kernel only needs
//   * the chunk's zero-state end state e_n = pin_n E_n x (E_n = last O rows of F_n),
//   * the chunk start states (the same DPP carry scan as the general kernel),
//   * the correction sum_k K_n[j][k] gin_n s_n[k] accumulated over the wave's bands,
// i.e. O(L+O) + O L FMAs per chunk instead of running the recurrence twice per
// sample (hz_filterbank.hip's general kernel).  The result is the same linear map
// evaluated in another association order (parity: tests/test_filterbank_lti_gpu.py).
#include "hz_fb_impl.h"

namespace {

using namespace hz_fbi;

// LTI band record (doubles), built on the host in long double.
template <int O, int L>
struct RecL {
    static constexpr int XW = L + O;            // chunk input window x[tc-O .. tc+L-1]
    static constexpr int E = 0;                 // E[k][i]  k<O, i<XW : F[L-1-k][i]
    static constexpr int K = E + O * XW;        // K[j][k]  j<L, k<O  : homogeneous response
    static constexpr int P = K + L * O;         // P[s] = M^(2^s), s<6 (M: chunk transition)
    static constexpr int Q = P + 6 * O * O;     // Q[p] = M^p, p<16
    static constexpr int H = Q + 16 * O * O;    // H[d], d<XW : FIR*IIR impulse response
    static constexpr int GE = H + XW;           // GE[i][j], i<O, j<L : F[j][i] (history taps)
    static constexpr int RAW = GE + O * L;
    static constexpr int SIZE = (RAW + 7) & ~7;
};

static int lti_rec_size(int O, int L) {
    if (L == 16) {
        switch (O) {
        case 0: return RecL<0, 16>::SIZE;
        case 1: return RecL<1, 16>::SIZE;
        case 2: return RecL<2, 16>::SIZE;
        case 3: return RecL<3, 16>::SIZE;
        default: return RecL<4, 16>::SIZE;
        }
    }
    switch (O) {
    case 0: return RecL<0, 32>::SIZE;
    case 1: return RecL<1, 32>::SIZE;
    case 2: return RecL<2, 32>::SIZE;
    case 3: return RecL<3, 32>::SIZE;
    default: return RecL<4, 32>::SIZE;
    }
}

template <int O, int L>
void build_record_lti(const double* b, const double* av, double* rec) {
    using R = RecL<O, L>;
    constexpr int XW = R::XW;
    std::memset(rec, 0, sizeof(double) * R::SIZE);
    // impulse response of 1 / A(z): h[0] = 1, h[m] = -sum_k a_k h[m-1-k]
    long double h[XW];
    for (int m = 0; m < XW; ++m) {
        long double v = (m == 0) ? 1.0L : 0.0L;
        for (int k = 0; k < O && k < m; ++k) v -= (long double)av[k] * h[m - 1 - k];
        h[m] = v;
    }
    // F[j][i]: response at chunk sample j to x[tc - O + i]; s = i - O
    auto F = [&](int j, int i) -> long double {
        const int s = i - O;
        long double acc = 0;
        // u[m] = sum_q b_q x[m - q]: x[s] enters u[m] with q = m - s, 0 <= m <= j, m >= 0
        for (int m = std::max(0, s); m <= j && m - s <= O; ++m) acc += h[j - m] * (long double)b[m - s];
        return acc;
    };
    for (int d = 0; d < XW; ++d) {
        long double acc = 0;
        for (int q = 0; q <= O && q <= d; ++q) acc += (long double)b[q] * h[d - q];
        rec[R::H + d] = (double)acc;
    }
    for (int i = 0; i < O; ++i)
        for (int j = 0; j < L; ++j) rec[R::GE + i * L + j] = (double)F(j, i);
    if constexpr (O > 0) {
        for (int k = 0; k < O; ++k)
            for (int i = 0; i < XW; ++i) rec[R::E + k * XW + i] = (double)F(L - 1 - k, i);
        // homogeneous responses: y[-1-k] = 1, zero input
        long double Kh[L][O];
        for (int k = 0; k < O; ++k) {
            long double yh[O];
            for (int q = 0; q < O; ++q) yh[q] = (q == k) ? 1.0L : 0.0L;
            for (int j = 0; j < L; ++j) {
                long double y = 0;
                for (int q = 0; q < O; ++q) y -= (long double)av[q] * yh[q];
                for (int q = O - 1; q > 0; --q) yh[q] = yh[q - 1];
                yh[0] = y;
                Kh[j][k] = y;
                rec[R::K + j * O + k] = (double)y;
            }
        }
        long double M[O][O], T[O][O], Qp[O][O];
        for (int r = 0; r < O; ++r)
            for (int c = 0; c < O; ++c) {
                M[r][c] = Kh[L - 1 - r][c];
                Qp[r][c] = (r == c) ? 1.0L : 0.0L;
            }
        for (int p = 0; p < 16; ++p) {
            for (int r = 0; r < O; ++r)
                for (int c = 0; c < O; ++c) rec[R::Q + p * O * O + r * O + c] = (double)Qp[r][c];
            for (int r = 0; r < O; ++r)
                for (int c = 0; c < O; ++c) {
                    long double acc = 0;
                    for (int q = 0; q < O; ++q) acc += Qp[r][q] * M[q][c];
                    T[r][c] = acc;
                }
            std::memcpy(Qp, T, sizeof(Qp));
        }
        for (int s = 0; s < 6; ++s) {
            for (int r = 0; r < O; ++r)
                for (int c = 0; c < O; ++c) rec[R::P + s * O * O + r * O + c] = (double)M[r][c];
            for (int r = 0; r < O; ++r)
                for (int c = 0; c < O; ++c) {
                    long double acc = 0;
                    for (int q = 0; q < O; ++q) acc += M[r][q] * M[q][c];
                    T[r][c] = acc;
                }
            std::memcpy(M, T, sizeof(M));
        }
    }
}

static void build_record_lti_any(int O, int L, const double* b, const double* a, double* rec) {
#define HZ_LTI_REC(OO)                                                          \
    case OO:                                                                    \
        if (L == 16) build_record_lti<OO, 16>(b, a, rec);                       \
        else build_record_lti<OO, 32>(b, a, rec);                               \
        break;
    switch (O) {
        HZ_LTI_REC(0)
        HZ_LTI_REC(1)
        HZ_LTI_REC(2)
        HZ_LTI_REC(3)
        HZ_LTI_REC(4)
    }
#undef HZ_LTI_REC
}

struct LtiArgs {
    const double* pin;      // [N] converged pre-amps
    const double* gin;      // [N] converged gains
    const double* ystate;   // [N][O] y[-1-k] at call start
    double* ystate_next;    // [N][O] at call end (ping-pong)
    const double* pgstate;  // [N][2]
    double* pgstate_next;   // [N][2]
    const double* x;        // [n]
    const double* xhist;    // [O]
    double* xhist_next;     // [O]
    double* partial;        // [G][n_pad]
    double* segstate;       // [N][nseg][O]
    long n;                 // samples in this launch (multiple of L)
    long n_pad;
    long seg_len;           // multiple of the tile (64 L)
    int nseg;
    int nbands;
    double sp_n, sg_n;      // sp^n, sg^n (closed-form smoother end state)
};

// LDS: x tile x[t0-O .. t0+64L-1] stored at pos(li) = li + li / L (one pad slot per
// chunk) so lane c's window reads start on distinct banks; double-buffered.
template <int O, int L>
__host__ __device__ constexpr int lti_xs_len() { return 64 * L + O; }
template <int O, int L>
__host__ __device__ constexpr int lti_xs_pad() {
    return ((lti_xs_len<O, L>() + lti_xs_len<O, L>() / L + 1) + 1) & ~1;
}
// gs rows [KD = W NB O][64 chunks + 16 pad]: the MFMA A-operand reads (16 chunks of
// two rows per 32-lane group) land on disjoint bank halves; double-buffered.
constexpr int kGsRow = 80;
template <int O, int L>
__host__ __device__ constexpr size_t lti_lds_bytes(int waves, int nb, bool mix) {
    return sizeof(double) * (2 * (size_t)lti_xs_pad<O, L>() + (mix ? 2 * (size_t)waves * nb * O * kGsRow : 0));
}

typedef double hz_f64x4 __attribute__((ext_vector_type(4)));

// One workgroup = W waves x NB bands (band group g = blockIdx.x) over one time
// segment (blockIdx.y); a wave walks the segment's tiles carrying its bands' state.
// Per tile: each wave computes, for its bands, the chunk zero-state end states (E, VALU
// with wave-uniform coefficients), the carry scan and the chunk start states st; it
// stores gs = gin st to LDS.  After the barrier the bank group's correction mix
//   D[chunk][j] = sum_{(band,k)} gs[(band,k)][chunk] K_band[j][k]
// is a (64 x KD) x (KD x L) product on the FP64 matrix cores (v_mfma_f64_16x16x4f64):
// the reduction over the group's bands happens inside the MFMA, no per-band LDS rows.
template <int O, int L, int NB, int W, int MODE>
__global__ __launch_bounds__(64 * W) void fb_lti_kernel(const double* __restrict__ rec, LtiArgs a) {
    using R = RecL<O, L>;
    constexpr int XW = R::XW;
    constexpr int T = 64 * L;
    constexpr int XS = lti_xs_len<O, L>();
    constexpr int XSP = lti_xs_pad<O, L>();
    constexpr int PF = (XS + 64 * W - 1) / (64 * W);  // x values staged per thread
    constexpr int KD = W * NB * O;                     // MFMA reduction length
    constexpr int KSTEPS = KD / 4;
    constexpr int NBLK = 4 * (L / 16);                 // 16x16 output blocks per tile
    constexpr int BPW = (NBLK + W - 1) / W;            // blocks per mixing wave
    static_assert(KD % 4 == 0, "KD multiple of 4");
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* gsb = lds + 2 * XSP;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp_band0 = blockIdx.x * W * NB;
    const int band0 = grp_band0 + wave * NB;
    const long n = a.n;
    const int seg = blockIdx.y;
    const long seg_t0 = (long)seg * a.seg_len;
    const long seg_end = min(seg_t0 + a.seg_len, n);
    const int ntiles = (int)((seg_end - seg_t0 + T - 1) / T);
    const bool last_seg = seg == a.nseg - 1;

    bool live[NB];
    double S[NB][O], pb[NB], gb[NB];
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
        pb[b] = live[b] ? a.pin[bb] : 0.0;
        gb[b] = live[b] ? a.gin[bb] : 0.0;
    }

    // MFMA B operands (constant over the launch): lane l of k-step q holds
    // K_band[j][k] for kd = 4q + (l >> 4) = band_local O + k, j = 16 nblk + (l & 15)
    double bk[MODE == MODE_MIX ? BPW : 1][MODE == MODE_MIX ? KSTEPS : 1];
    if constexpr (MODE == MODE_MIX) {
#pragma unroll
        for (int u = 0; u < BPW; ++u) {
            const int blk = wave + u * W;
            const int j = 16 * (blk >> 2) + (lane & 15);
#pragma unroll
            for (int q = 0; q < KSTEPS; ++q) {
                const int kd = 4 * q + (lane >> 4);
                const int band = grp_band0 + kd / O;
                bk[u][q] = (blk < NBLK && band < a.nbands) ? rec[(long)band * R::SIZE + R::K + j * O + kd % O] : 0.0;
            }
        }
    }

    auto load_x = [&](long t0x, double (&pf)[PF]) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int li = threadIdx.x + q * 64 * W;
            const long idx = t0x - O + li;
            double v = 0.0;
            if (li < XS) {
                if (idx < 0) v = a.xhist[-idx - 1];
                else if (idx < seg_end) v = a.x[idx];
            }
            pf[q] = v;
        }
    };
    auto store_x = [&](double* xbuf, const double (&pf)[PF]) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int li = threadIdx.x + q * 64 * W;
            if (li < XS) xbuf[li + li / L] = pf[q];
        }
    };
    {
        double pf0[PF];
        load_x(seg_t0, pf0);
        store_x(lds, pf0);
        __syncthreads();
    }

    for (int tile = 0; tile < ntiles; ++tile) {
        const long t0 = seg_t0 + (long)tile * T;
        const bool last_tile = last_seg && tile == ntiles - 1;
        const double* xs = lds + (tile & 1) * XSP;
        double* gs_tile = gsb + (tile & 1) * KD * kGsRow;
        double pf[PF];
        const bool more = tile + 1 < ntiles;
        if (more) load_x(t0 + T, pf);

        // the lane's chunk window x[tc-O .. tc+L-1] (li = L lane + i -> lane (L+1) + i + i/L)
        double xw[XW];
#pragma unroll
        for (int i = 0; i < XW; ++i) xw[i] = xs[lane * (L + 1) + i + i / L];

#pragma unroll
        for (int b = 0; b < NB; ++b) {
            double st[O];
            if (live[b]) {  // wave-uniform
                const double* r = rec + (long)(band0 + b) * R::SIZE;
                // zero-state end state of the lane's chunk: z[k] = y_zs[tc + L-1-k]
                // (two interleaved partial sums per k: half the FMA dependency chain)
                double z[O];
#pragma unroll
                for (int k = 0; k < O; ++k) {
                    double acc0 = r[R::E + k * XW] * xw[0];
                    double acc1 = r[R::E + k * XW + 1] * xw[1];
#pragma unroll
                    for (int i = 2; i + 1 < XW; i += 2) {
                        acc0 = fma(r[R::E + k * XW + i], xw[i], acc0);
                        acc1 = fma(r[R::E + k * XW + i + 1], xw[i + 1], acc1);
                    }
                    if constexpr (XW % 2) acc0 = fma(r[R::E + k * XW + XW - 1], xw[XW - 1], acc0);
                    z[k] = pb[b] * (acc0 + acc1);
                }
                // carry scan over the 64 chunks (as fb_mix_kernel): intra-row DPP scan with
                // M^(2^s), wave-uniform row carries, chunk start st = Z(p-1) + M^p C_row
                const int row = lane >> 4, p = lane & 15;
                double qm[O * O];
#pragma unroll
                for (int e = 0; e < O * O; ++e) qm[e] = r[R::Q + p * O * O + e];
#define HZ_LTI_ROW_STEP(SIDX, D)                                                              \
    {                                                                                         \
        double nb_[O];                                                                        \
        _Pragma("unroll") for (int k = 0; k < O; ++k) nb_[k] = dpp_d<kDppRowShr + (D)>(z[k]); \
        _Pragma("unroll") for (int rr = 0; rr < O; ++rr)                                      \
            _Pragma("unroll") for (int c = 0; c < O; ++c)                                     \
                z[rr] = fma(r[R::P + (SIDX) * O * O + rr * O + c], nb_[c], z[rr]);            \
    }
                HZ_LTI_ROW_STEP(0, 1)
                HZ_LTI_ROW_STEP(1, 2)
                HZ_LTI_ROW_STEP(2, 4)
                HZ_LTI_ROW_STEP(3, 8)
#undef HZ_LTI_ROW_STEP
                double C[5][O];
#pragma unroll
                for (int k = 0; k < O; ++k) C[0][k] = S[b][k];
#pragma unroll
                for (int rw = 0; rw < 4; ++rw) {
#pragma unroll
                    for (int i = 0; i < O; ++i) {
                        double acc = readlane_d(z[i], 16 * rw + 15);
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
                    double vv = dpp_d<kDppRowShr + 1>(z[k]);  // Z(r, p-1), 0 at p == 0
#pragma unroll
                    for (int c = 0; c < O; ++c) vv = fma(qm[k * O + c], Cr[c], vv);
                    st[k] = vv;
                }
#pragma unroll
                for (int k = 0; k < O; ++k) S[b][k] = C[4][k];
                if constexpr (MODE == MODE_MIX) {
                    if (last_tile) {
                        // end-of-call y history = the start state of the chunk beginning at n
                        // (n is a multiple of L; chunks past n see zero input)
                        const int cn = (int)((n - t0) / L);  // in [1, 64]
                        const long band = band0 + b;
                        if (cn < 64) {
                            if (lane == cn)
#pragma unroll
                                for (int k = 0; k < O; ++k) a.ystate_next[band * O + k] = st[k];
                        } else if (lane == 0) {
#pragma unroll
                            for (int k = 0; k < O; ++k) a.ystate_next[band * O + k] = C[4][k];
                        }
                    }
                }
            } else {
#pragma unroll
                for (int k = 0; k < O; ++k) st[k] = 0.0;
            }
            if constexpr (MODE == MODE_MIX) {
#pragma unroll
                for (int k = 0; k < O; ++k) gs_tile[((wave * NB + b) * O + k) * kGsRow + lane] = gb[b] * st[k];
            }
        }

        if constexpr (MODE == MODE_MIX) {
            if (last_tile && lane == 0) {
#pragma unroll
                for (int b = 0; b < NB; ++b) {
                    if (!live[b]) continue;
                    const long band = band0 + b;
                    const double P0 = a.pgstate[2 * band], G0 = a.pgstate[2 * band + 1];
                    a.pgstate_next[2 * band] = pb[b] + a.sp_n * (P0 - pb[b]);
                    a.pgstate_next[2 * band + 1] = gb[b] + a.sg_n * (G0 - gb[b]);
                }
            }
        }
        if (more) store_x(lds + ((tile + 1) & 1) * XSP, pf);
        __syncthreads();
        if constexpr (MODE == MODE_MIX) {
            // ---- group mix on the matrix cores: D[16 chunks][16 samples] per block --------
#pragma unroll
            for (int u = 0; u < BPW; ++u) {
                const int blk = wave + u * W;  // wave-uniform
                if (blk < NBLK) {
                    const int m = blk & 3, nblk = blk >> 2;
                    hz_f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
                    const double* ga = gs_tile + (lane >> 4) * kGsRow + 16 * m + (lane & 15);
#pragma unroll
                    for (int q = 0; q < KSTEPS; q += 2) {
                        acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[4 * q * kGsRow], bk[u][q], acc0, 0, 0, 0);
                        if (q + 1 < KSTEPS)
                            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[4 * (q + 1) * kGsRow], bk[u][q + 1], acc1,
                                                                       0, 0, 0);
                    }
                    // D row = chunk 16 m + (lane >> 4) + 4 r, column = sample j of the chunk
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        const int chunk = 16 * m + (lane >> 4) + 4 * rr;
                        const long t = t0 + (long)chunk * L + 16 * nblk + (lane & 15);
                        if (t < n) a.partial[(long)blockIdx.x * a.n_pad + t] = acc0[rr] + acc1[rr];
                    }
                }
            }
        }
    }

    if constexpr (MODE == MODE_SEGEND) {
        if (lane == 0 && !last_seg) {
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (!live[b]) continue;
#pragma unroll
                for (int k = 0; k < O; ++k) a.segstate[((long)(band0 + b) * a.nseg + seg + 1) * O + k] = S[b][k];
            }
        }
    } else {
        if (last_seg && blockIdx.x == 0 && threadIdx.x < O) {
            const int k = threadIdx.x;
            const long idx = n - 1 - k;
            a.xhist_next[k] = idx >= 0 ? a.x[idx] : a.xhist[-idx - 1];
        }
    }
}

// Sequential carry over time segments (one thread per band), LTI records:
//   start(s+1) = M_tile^seg_tiles start(s) + zsr_end(s), M_tile = P[5]^2 = M^64.
template <int O, int L>
__global__ __launch_bounds__(256) void fb_lti_seg_carry_kernel(const double* __restrict__ rec,
                                                               const double* __restrict__ ystate,
                                                               double* __restrict__ segstate, int nbands,
                                                               int nseg, long seg_tiles) {
    using R = RecL<O, L>;
    const int band = blockIdx.x * blockDim.x + threadIdx.x;
    if (band >= nbands) return;
    const double* r = rec + (long)band * R::SIZE;
    double M[O][O], Pw[O][O], Tm[O][O];
#pragma unroll
    for (int i = 0; i < O; ++i)
#pragma unroll
        for (int j = 0; j < O; ++j) {
            double acc = 0;
#pragma unroll
            for (int q = 0; q < O; ++q) acc = fma(r[R::P + 5 * O * O + i * O + q], r[R::P + 5 * O * O + q * O + j], acc);
            Pw[i][j] = acc;
            M[i][j] = (i == j) ? 1.0 : 0.0;
        }
    for (long e = seg_tiles; e > 0; e >>= 1) {
        if (e & 1) {
            for (int i = 0; i < O; ++i)
                for (int j = 0; j < O; ++j) {
                    double acc = 0;
                    for (int q = 0; q < O; ++q) acc = fma(M[i][q], Pw[q][j], acc);
                    Tm[i][j] = acc;
                }
            for (int i = 0; i < O; ++i)
                for (int j = 0; j < O; ++j) M[i][j] = Tm[i][j];
        }
        for (int i = 0; i < O; ++i)
            for (int j = 0; j < O; ++j) {
                double acc = 0;
                for (int q = 0; q < O; ++q) acc = fma(Pw[i][q], Pw[q][j], acc);
                Tm[i][j] = acc;
            }
        for (int i = 0; i < O; ++i)
            for (int j = 0; j < O; ++j) Pw[i][j] = Tm[i][j];
    }
    double Sv[O];
#pragma unroll
    for (int k = 0; k < O; ++k) Sv[k] = ystate[(long)band * O + k];
    for (int s = 1; s < nseg; ++s) {
        double* slot = segstate + ((long)band * nseg + s) * O;
        double nS[O];
#pragma unroll
        for (int i = 0; i < O; ++i) {
            double acc = slot[i];
#pragma unroll
            for (int q = 0; q < O; ++q) acc = fma(M[i][q], Sv[q], acc);
            nS[i] = acc;
        }
#pragma unroll
        for (int i = 0; i < O; ++i) {
            Sv[i] = nS[i];
            slot[i] = nS[i];
        }
    }
}

// Fmix[j][i] = sum_n pin_n gin_n F_n[j][i]; one workgroup per entry, deterministic
// tree over bands.  F_n[j][i] = H_n[j - i + O] (0 below the diagonal) for the chunk's
// own samples (i >= O), GE_n[i][j] for the O history taps.
template <int O, int L>
__global__ __launch_bounds__(256) void fb_fmix_kernel(const double* __restrict__ rec, const double* __restrict__ pin,
                                                      const double* __restrict__ gin, int nbands,
                                                      double* __restrict__ fmix) {
    using R = RecL<O, L>;
    __shared__ double red[256];
    const int e = blockIdx.x;
    const int j = e / R::XW, i = e % R::XW;
    double s = 0.0;
    for (int nb = threadIdx.x; nb < nbands; nb += 256) {
        const double* r = rec + (long)nb * R::SIZE;
        double f;
        if (i >= O) f = (j - i + O >= 0) ? r[R::H + j - i + O] : 0.0;
        else f = r[R::GE + i * L + j];
        s = fma(pin[nb] * gin[nb], f, s);
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) fmix[e] = red[0];
}

// out[t] = sum_g partial[g][t] + sum_i Fmix[t mod L][i] x[t - t mod L - O + i]
template <int O, int L>
__global__ __launch_bounds__(256) void fb_lti_reduce_kernel(const double* __restrict__ partial, long n_pad, int G,
                                                            long n, const double* __restrict__ x,
                                                            const double* __restrict__ xhist,
                                                            const double* __restrict__ fmix,
                                                            double* __restrict__ out) {
    constexpr int XW = L + O;
    __shared__ double red[4][64];
    __shared__ double fm[L * XW];
    for (int e = threadIdx.x; e < L * XW; e += 256) fm[e] = fmix[e];
    __syncthreads();
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    const long t = (long)blockIdx.x * 64 + tx;
    double s = 0.0;
    if (t < n) {
        for (int g = ty; g < G; g += 4) s += partial[(long)g * n_pad + t];
        // zero-state mix, split over the 4 row groups
        const int j = (int)(t % L);
        const long base = t - j - O;
        for (int i = ty; i < XW; i += 4) {
            const long idx = base + i;
            const double xv = idx >= 0 ? x[idx] : xhist[-idx - 1];
            s = fma(fm[j * XW + i], xv, s);
        }
    }
    red[ty][tx] = s;
    __syncthreads();
    if (ty == 0 && t < n) out[t] = (red[0][tx] + red[1][tx]) + (red[2][tx] + red[3][tx]);
}

// ---- kernel selection -------------------------------------------
typedef void (*CarryKernel)(const double*, const double*, double*, int, int, long);
typedef void (*LtiKernel)(const double*, LtiArgs);
typedef void (*FmixKernel)(const double*, const double*, const double*, int, double*);
typedef void (*LtiReduceKernel)(const double*, long, int, long, const double*, const double*, const double*,
                                double*);

// geometries: (L, bands per wave, waves per group)
struct LtiGeom {
    int L, nb, waves;
};
static const LtiGeom kLtiGeoms[] = {{16, 1, 16}, {32, 1, 16}, {16, 2, 8}};
constexpr int kNumLtiGeoms = 3;

template <int O, int L, int NB, int W>
LtiKernel lti_kernel_mode(int mode) {
    static_assert(lti_lds_bytes<O, L>(W, NB, true) <= 160 * 1024, "LTI kernel LDS over 160 KiB");
    return mode == MODE_SEGEND ? fb_lti_kernel<O, L, NB, W, MODE_SEGEND> : fb_lti_kernel<O, L, NB, W, MODE_MIX>;
}

template <int O>
LtiKernel lti_kernel_geom(int geom, int mode) {
    switch (geom) {
    case 1: return lti_kernel_mode<O, 32, 1, 16>(mode);
    case 2: return lti_kernel_mode<O, 16, 2, 8>(mode);
    default: return lti_kernel_mode<O, 16, 1, 16>(mode);
    }
}

static LtiKernel pick_lti(int O, int geom, int mode) {
    switch (O) {
    case 1: return lti_kernel_geom<1>(geom, mode);
    case 2: return lti_kernel_geom<2>(geom, mode);
    case 3: return lti_kernel_geom<3>(geom, mode);
    default: return lti_kernel_geom<4>(geom, mode);
    }
}

static size_t lti_lds(int O, int geom, bool mix) {
    const LtiGeom g = kLtiGeoms[geom];
#define HZ_LTI_LDS(OO)                                                                                  \
    case OO:                                                                                            \
        return g.L == 16 ? lti_lds_bytes<OO, 16>(g.waves, g.nb, mix) : lti_lds_bytes<OO, 32>(g.waves, g.nb, mix);
    switch (O) {
        HZ_LTI_LDS(1)
        HZ_LTI_LDS(2)
        HZ_LTI_LDS(3)
    default:
        return g.L == 16 ? lti_lds_bytes<4, 16>(g.waves, g.nb, mix) : lti_lds_bytes<4, 32>(g.waves, g.nb, mix);
    }
#undef HZ_LTI_LDS
}

#define HZ_LTI_OL(TEMPLATE, O, L)                                                                    \
    (L == 16 ? (O == 1 ? TEMPLATE<1, 16> : O == 2 ? TEMPLATE<2, 16> : O == 3 ? TEMPLATE<3, 16> : TEMPLATE<4, 16>) \
             : (O == 1 ? TEMPLATE<1, 32> : O == 2 ? TEMPLATE<2, 32> : O == 3 ? TEMPLATE<3, 32> : TEMPLATE<4, 32>))
static CarryKernel pick_lti_carry(int O, int L) { return HZ_LTI_OL(fb_lti_seg_carry_kernel, O, L); }
static FmixKernel pick_fmix(int O, int L) { return HZ_LTI_OL(fb_fmix_kernel, O, L); }
static LtiReduceKernel pick_lti_reduce(int O, int L) { return HZ_LTI_OL(fb_lti_reduce_kernel, O, L); }
#undef HZ_LTI_OL

}  // namespace

namespace hz_fbi {

int fb_lti_chunk(const hz_fb* h) { return kLtiGeoms[h->lti_geom].L; }

// every band's smoothers at their targets (host mirror), relative to the bank's
// largest target: the LTI engine then computes the same outputs to ~2^-60
bool fb_converged(const hz_fb* h) {
    double pmax = 0, gmax = 0;
    for (int b = 0; b < h->N; ++b) {
        pmax = std::max(pmax, std::fabs(h->pin[b]));
        gmax = std::max(gmax, std::fabs(h->gin[b]));
    }
    const double tp = 0x1p-60 * pmax, tg = 0x1p-60 * gmax;
    for (int b = 0; b < h->N; ++b) {
        if (!(std::fabs(h->pg_host[2 * (size_t)b] - h->pin[b]) <= tp)) return false;
        if (!(std::fabs(h->pg_host[2 * (size_t)b + 1] - h->gin[b]) <= tg)) return false;
    }
    return true;
}

int fb_prepare_lti(hz_fb* h) {
    const int O = h->order;
    const int L = kLtiGeoms[h->lti_geom].L;
    if (h->dirty_lti || h->lti_rec_L != L) {
        const int rs = lti_rec_size(O, L);
        const size_t need = (size_t)h->N * rs;
        h->h_rec_lti.assign(need, 0.0);
        for (int b = 0; b < h->N; ++b)
            build_record_lti_any(O, L, &h->F[(size_t)b * (O + 1)], &h->B[(size_t)b * O], &h->h_rec_lti[(size_t)b * rs]);
        if (need > h->rec_lti_cap) {
            if (h->d_rec_lti) HZ_TRY_HIP(hipFree(h->d_rec_lti));
            h->d_rec_lti = nullptr;
            HZ_TRY_HIP(hipMalloc(&h->d_rec_lti, sizeof(double) * need));
            h->rec_lti_cap = need;
        }
        if (!h->d_fmix) HZ_TRY_HIP(hipMalloc(&h->d_fmix, sizeof(double) * 32 * (32 + kMaxOrder)));
        HZ_TRY_HIP(hipMemcpyAsync(h->d_rec_lti, h->h_rec_lti.data(), sizeof(double) * need, hipMemcpyHostToDevice,
                                  h->stream));
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));  // pageable source
        h->lti_rec = rs;
        h->lti_rec_L = L;
        h->dirty_lti = false;
        h->fmix_valid = false;
    }
    if (!h->fmix_valid) {
        hipLaunchKernelGGL(pick_fmix(O, L), dim3((unsigned)(L * (L + O))), dim3(256), 0, h->stream,
                           (const double*)h->d_rec_lti, (const double*)h->d_pin, (const double*)h->d_gin, h->N,
                           h->d_fmix);
        HZ_TRY_HIP(hipGetLastError());
        h->fmix_valid = true;
    }
    return HZ_OK;
}

// the converged engine over n samples (n a positive multiple of the chunk length)
int fb_launch_lti(hz_fb* h, const double* d_in, double* d_out, long n) {
    HZ_TRY(fb_prepare_lti(h));
    const int O = h->order;
    const LtiGeom geom = kLtiGeoms[h->lti_geom];
    const int L = geom.L;
    const long T = 64L * L;
    const int per = geom.waves * geom.nb;
    const int G = (h->N + per - 1) / per;
    // partial slab <= 2^27 doubles per launch
    long chunk = std::max<long>(T, (((1L << 27) / std::max(1, G)) / T) * T);
    const long n_pad_max = std::min<long>(((n + T - 1) / T) * T, chunk);
    const size_t need = (size_t)G * n_pad_max;
    if (need > h->partial_cap) {
        if (h->d_partial) HZ_TRY_HIP(hipFree(h->d_partial));
        h->d_partial = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_partial, sizeof(double) * need));
        h->partial_cap = need;
    }
    LtiKernel kmix = pick_lti(O, h->lti_geom, MODE_MIX);
    LtiKernel kend = pick_lti(O, h->lti_geom, MODE_SEGEND);
    HZ_TRY(fb_set_lds_attr((const void*)kmix));
    HZ_TRY(fb_set_lds_attr((const void*)kend));
    const size_t lds = lti_lds(O, h->lti_geom, true);
    const size_t lds_end = lti_lds(O, h->lti_geom, false);
    for (long off = 0; off < n; off += chunk) {
        const long len = std::min(chunk, n - off);
        const long ntiles = (len + T - 1) / T;
        long nseg = std::max<long>(1, std::min<long>(ntiles, (h->target_groups + G - 1) / G));
        const long seg_tiles = (ntiles + nseg - 1) / nseg;
        nseg = (ntiles + seg_tiles - 1) / seg_tiles;
        if (nseg > 1) {
            const size_t sneed = (size_t)h->N * nseg * O;
            if (sneed > h->seg_cap) {
                if (h->d_seg) HZ_TRY_HIP(hipFree(h->d_seg));
                h->d_seg = nullptr;
                HZ_TRY_HIP(hipMalloc(&h->d_seg, sizeof(double) * sneed));
                h->seg_cap = sneed;
            }
        }
        LtiArgs a;
        a.pin = h->d_pin;
        a.gin = h->d_gin;
        a.ystate = h->d_ystate[h->scur];
        a.ystate_next = h->d_ystate[h->scur ^ 1];
        a.pgstate = h->d_pg[h->scur];
        a.pgstate_next = h->d_pg[h->scur ^ 1];
        a.x = d_in + off;
        a.xhist = h->d_xhist[h->xcur];
        a.xhist_next = h->d_xhist[h->xcur ^ 1];
        a.partial = h->d_partial;
        a.segstate = h->d_seg;
        a.n = len;
        a.n_pad = ntiles * T;
        a.seg_len = seg_tiles * T;
        a.nseg = (int)nseg;
        a.nbands = h->N;
        a.sp_n = (double)powl((long double)h->sp, (long double)len);
        a.sg_n = (double)powl((long double)h->sg, (long double)len);
        hipEvent_t* e = nullptr;
        if (h->prof) {
            if (h->ev_used + 4 > h->ev.size()) {
                for (int q = 0; q < 4 * 64; ++q) {
                    hipEvent_t ne;
                    HZ_TRY_HIP(hipEventCreate(&ne));
                    h->ev.push_back(ne);
                }
            }
            e = &h->ev[h->ev_used];
            h->ev_used += 4;
            HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        }
        if (nseg > 1) {
            hipLaunchKernelGGL(kend, dim3(G, (unsigned)(nseg - 1)), dim3(64 * geom.waves), lds_end, h->stream,
                               (const double*)h->d_rec_lti, a);
            HZ_TRY_HIP(hipGetLastError());
            hipLaunchKernelGGL(pick_lti_carry(O, L), dim3((unsigned)((h->N + 255) / 256)), dim3(256), 0, h->stream,
                               (const double*)h->d_rec_lti, (const double*)h->d_ystate[h->scur], h->d_seg, h->N,
                               (int)nseg, seg_tiles);
            HZ_TRY_HIP(hipGetLastError());
        }
        if (e) HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
        hipLaunchKernelGGL(kmix, dim3(G, (unsigned)nseg), dim3(64 * geom.waves), lds, h->stream,
                           (const double*)h->d_rec_lti, a);
        HZ_TRY_HIP(hipGetLastError());
        if (e) HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
        hipLaunchKernelGGL(pick_lti_reduce(O, L), dim3((unsigned)((len + 63) / 64)), dim3(256), 0, h->stream,
                           (const double*)h->d_partial, a.n_pad, G, len, a.x, a.xhist, (const double*)h->d_fmix,
                           d_out + off);
        HZ_TRY_HIP(hipGetLastError());
        if (e) HZ_TRY_HIP(hipEventRecord(e[3], h->stream));
        h->xcur ^= 1;
        h->scur ^= 1;
        h->prof_launches += h->prof ? 1 : 0;
        fb_mirror_advance(h, len);
    }
    return HZ_OK;
}

}  // namespace hz_fbi

extern "C" {

int hz_fb_tune_lti(hz_fb* h, int chunk, int bands_per_wave, int waves_per_group) {
    if (!h) return HZ_E_INVALID;
    if (!chunk && !bands_per_wave && !waves_per_group) {
        h->lti_geom = 0;
        return HZ_OK;
    }
    for (int g = 0; g < kNumLtiGeoms; ++g)
        if (kLtiGeoms[g].L == chunk && kLtiGeoms[g].nb == bands_per_wave && kLtiGeoms[g].waves == waves_per_group) {
            h->lti_geom = g;
            return HZ_OK;
        }
    hz::set_error("hz_fb_tune_lti: (chunk, bands/wave, waves) must be one of (16,1,16), (32,1,16), (16,2,8)");
    return HZ_E_INVALID;
}

}  // extern "C"
