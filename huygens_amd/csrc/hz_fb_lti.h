// hz_fb_lti.h -- the converged ("LTI") path of the Filterbank<double> engine.
//
// Included by hz_filterbank.hip (uses its uniform / dpp_d / readlane_d helpers).
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
#pragma once

namespace {

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
constexpr int kLtiPartPad = 66;  // per-wave partial rows [L][66]
template <int O, int L>
__host__ __device__ constexpr size_t lti_lds_bytes(int waves, bool mix) {
    return sizeof(double) * (2 * (size_t)lti_xs_pad<O, L>() + (mix ? (size_t)waves * L * kLtiPartPad : 0));
}

template <int O, int L, int NB, int W, int MODE>
__global__ __launch_bounds__(64 * W) void fb_lti_kernel(const double* __restrict__ rec, LtiArgs a) {
    using R = RecL<O, L>;
    constexpr int XW = R::XW;
    constexpr int T = 64 * L;
    constexpr int XS = lti_xs_len<O, L>();
    constexpr int XSP = lti_xs_pad<O, L>();
    constexpr int PF = (XS + 64 * W - 1) / (64 * W);  // x values staged per thread
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* part = lds + 2 * XSP;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int band0 = (blockIdx.x * W + wave) * NB;
    const long n = a.n;
    const int seg = blockIdx.y;
    const long seg_t0 = (long)seg * a.seg_len;
    const long seg_end = min(seg_t0 + a.seg_len, n);
    const int ntiles = (int)((seg_end - seg_t0 + T - 1) / T);
    const bool last_seg = seg == a.nseg - 1;
    double* my = part + (long)wave * L * kLtiPartPad;

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
        double pf[PF];
        const bool more = tile + 1 < ntiles;
        if (more) load_x(t0 + T, pf);

        // the lane's chunk window x[tc-O .. tc+L-1] (li = L lane + i -> lane (L+1) + i + i/L)
        double xw[XW];
#pragma unroll
        for (int i = 0; i < XW; ++i) xw[i] = xs[lane * (L + 1) + i + i / L];

        double v[L];
#pragma unroll
        for (int j = 0; j < L; ++j) v[j] = 0.0;

#pragma unroll
        for (int b = 0; b < NB; ++b) {
            if (!live[b]) continue;  // wave-uniform
            const double* r = rec + (long)(band0 + b) * R::SIZE;
            // zero-state end state of the lane's chunk: z[k] = y_zs[tc + L-1-k]
            double z[O];
#pragma unroll
            for (int k = 0; k < O; ++k) {
                double acc = r[R::E + k * XW] * xw[0];
#pragma unroll
                for (int i = 1; i < XW; ++i) acc = fma(r[R::E + k * XW + i], xw[i], acc);
                z[k] = pb[b] * acc;
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
            double Cr[O], st[O];
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
                // correction mix: v[j] += sum_k K[j][k] gin st[k]
                double gs[O];
#pragma unroll
                for (int k = 0; k < O; ++k) gs[k] = gb[b] * st[k];
#pragma unroll
                for (int j = 0; j < L; ++j)
#pragma unroll
                    for (int k = 0; k < O; ++k) v[j] = fma(r[R::K + j * O + k], gs[k], v[j]);
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
            // ---- workgroup reduction of the per-wave mixes --------------------------
#pragma unroll
            for (int j = 0; j < L; ++j) my[j * kLtiPartPad + lane] = v[j];
            if (more) store_x(lds + ((tile + 1) & 1) * XSP, pf);
            __syncthreads();
            for (int tl = threadIdx.x; tl < T; tl += 64 * W) {
                const int src_lane = tl / L, j = tl % L;
                const double* q = part + j * kLtiPartPad + src_lane;
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int w = 0; w < W; w += 2) {
                    s0 += q[w * L * kLtiPartPad];
                    if (w + 1 < W) s1 += q[(w + 1) * L * kLtiPartPad];
                }
                const long t = t0 + tl;
                if (t < n) a.partial[(long)blockIdx.x * a.n_pad + t] = s0 + s1;
            }
        } else {
            if (more) store_x(lds + ((tile + 1) & 1) * XSP, pf);
        }
        __syncthreads();
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

}  // namespace
