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
#include <cstdio>
#include <cstdlib>

#include "hz_dd.h"
#include "hz_fb_impl.h"
#include "hz_fb_rec.h"


namespace {

using namespace hz_fbi;

static int lti_rec_size(int O, int L) {
#define HZ_LTI_RS(LL)                                                           \
    switch (O) {                                                                \
    case 0: return RecL<0, LL>::SIZE;                                           \
    case 1: return RecL<1, LL>::SIZE;                                           \
    case 2: return RecL<2, LL>::SIZE;                                           \
    case 3: return RecL<3, LL>::SIZE;                                           \
    default: return RecL<4, LL>::SIZE;                                          \
    }
    if (L == 16) HZ_LTI_RS(16)
    if (L == 32) HZ_LTI_RS(32)
    if (L == 128) HZ_LTI_RS(128)
    HZ_LTI_RS(64)
#undef HZ_LTI_RS
}

static int lti_k_offset(int O, int L) {
#define HZ_LTI_KO(LL)                                                           \
    switch (O) {                                                                \
    case 0: return RecL<0, LL>::K;                                              \
    case 1: return RecL<1, LL>::K;                                              \
    case 2: return RecL<2, LL>::K;                                              \
    case 3: return RecL<3, LL>::K;                                              \
    default: return RecL<4, LL>::K;                                             \
    }
    if (L == 16) HZ_LTI_KO(16)
    if (L == 32) HZ_LTI_KO(32)
    if (L == 128) HZ_LTI_KO(128)
    HZ_LTI_KO(64)
#undef HZ_LTI_KO
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
        for (int m = 0; m < XW; ++m) rec[R::E0 + m] = (double)F(L - 1, m);
        for (int k = 0; k < O; ++k)
            for (int i = 0; i < O; ++i) rec[R::EH + k * O + i] = (double)F(L - 1 - k, i);
        // homogeneous responses: y[-1-k] = 1, zero input; they and the chunk transition's powers
        // in double-double, M^64 keeping its low word (the tile and segment carries apply it many
        // times: hz_dd.h)
        using hz_dd::dd;
        dd Kh[L][O];
        for (int k = 0; k < O; ++k) {
            dd yh[O];
            for (int q = 0; q < O; ++q) yh[q] = {q == k ? 1.0 : 0.0, 0.0};
            for (int j = 0; j < L; ++j) {
                dd y{0.0, 0.0};
                for (int q = 0; q < O; ++q) y = hz_dd::add(y, hz_dd::mul(yh[q], -av[q]));
                for (int q = O - 1; q > 0; --q) yh[q] = yh[q - 1];
                yh[0] = y;
                Kh[j][k] = y;
                rec[R::K + j * O + k] = y.hi;
            }
        }
        dd M[O][O], T[O][O], Qp[O][O];
        for (int r = 0; r < O; ++r)
            for (int c = 0; c < O; ++c) {
                M[r][c] = Kh[L - 1 - r][c];
                Qp[r][c] = {r == c ? 1.0 : 0.0, 0.0};
            }
        for (int e = 0; e <= 64; ++e) {
            const int ps = e == 1 ? 0 : e == 2 ? 1 : e == 4 ? 2 : e == 8 ? 3 : e == 64 ? 4 : -1;
            for (int r = 0; r < O; ++r)
                for (int c = 0; c < O; ++c) {
                    rec[R::QC + e * O * O + r * O + c] = Qp[r][c].hi;
                    if (ps >= 0) rec[R::PS + ps * O * O + r * O + c] = Qp[r][c].hi;
                    if (e == 64) rec[R::PSL + r * O + c] = Qp[r][c].lo;
                }
            hz_dd::mat_mul<O>(Qp, M, T);
            std::memcpy(Qp, T, sizeof(Qp));
        }
    }
}

static void build_record_lti_any(int O, int L, const double* b, const double* a, double* rec) {
#define HZ_LTI_REC(OO)                                                          \
    case OO:                                                                    \
        if (L == 16) build_record_lti<OO, 16>(b, a, rec);                       \
        else if (L == 32) build_record_lti<OO, 32>(b, a, rec);                  \
        else if (L == 128) build_record_lti<OO, 128>(b, a, rec);                \
        else build_record_lti<OO, 64>(b, a, rec);                               \
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
    double* partial;        // [G][n_pad] (n_pad = row stride)
    double* gs_out;         // MODE_STATE: [tile][bs_pad][64 chunks] gin x chunk start states
    int bs_pad;             // GS rows per tile: band-state rows (lti_bs_rows: every wave's O rows; pad rows
                            // written 0), then the x-window rows
    int xr0, xr;            // chunk 128, MODE_STATE: the x-window rows xr0 .. xr0 + xr - 1 of every tile,
                            // written from the LDS x buffer by one workgroup per tile (xr = 0: none)
    double* segstate;       // [N][nseg_state][O] start states of the (prepass-fine) segments
    long n;                 // samples in this launch (multiple of L)
    long n_pad;             // slab row stride (the tile-padded length)
    long seg_len;           // multiple of the tile (64 L)
    int nseg;
    int nseg_state;         // segments in segstate (the prepass splits a segment in seg_stride)
    long seg_skip;          // prepass only: start this many samples into the segment (horizon)
    int seg_stride;         // segstate index of segment s: s * seg_stride
    int nbands;
    double sp_n, sg_n;      // sp^n, sg^n (closed-form smoother end state)
};

// LDS: x tile x[t0-O .. t0+64L-1] stored at pos(li) = li + P (li / L), P pad slots per chunk
// (lane c's window reads start on distinct banks); double-buffered.  Chunk 128 (one buffer,
// filled by LDS-DMA 1-KiB pieces, one per chunk): P = 2 keeps every chunk 16-B aligned.
template <int L>
__host__ __device__ constexpr int lti_xs_padc() { return L >= 128 ? 2 : 1; }
template <int O, int L>
__host__ __device__ constexpr int lti_xs_len() { return 64 * L + O; }
template <int O, int L>
__host__ __device__ constexpr int lti_xs_pad() {
    return L >= 128 ? 65 * (L + 2)   // 64 chunks + the O-sample tail piece, whole DMA pieces
                    : ((lti_xs_len<O, L>() + lti_xs_len<O, L>() / L + 1) + 1) & ~1;
}
// Workgroup geometry: one band per wave; 16 waves (bands) per workgroup for O <= 2,
// 8 for O >= 3 (LDS).  BS = band states of a group, padded to the 16-wide MFMA blocks.
__host__ __device__ constexpr int lti_waves(int O) { return O <= 2 ? 16 : 8; }
__host__ __device__ constexpr int lti_bsp(int O) { return (lti_waves(O) * O + 15) / 16 * 16; }
// GS / Kt rows (band states) of a bank: O rows for every wave of every group, so the state
// kernel's stores need no row guard (a conditional store makes the compiler's x-staging
// waits drain them: vmcnt(0) instead of vmcnt(2)); rounded up to 32 (whole pairs of 16-row
// GEMM stages), the rows past the groups' zeroed per call (fb_launch_lti)
static inline int lti_group_rows(int N, int O) { return (N + lti_waves(O) - 1) / lti_waves(O) * lti_waves(O) * O; }
static inline int lti_bs_rows(int N, int O) { return (lti_group_rows(N, O) + 31) / 32 * 32; }
// GEMM path: the bank-wide zero-state term joins the correction GEMM as XW = L + O extra K rows
// (rounded to 32): GS rows = the chunk's input window x[tc - O + r], K rows = Fmix[j][r]
static inline int lti_x_rows(int L, int O) { return (L + O + 31) / 32 * 32; }
constexpr int kZRow = 65;   // z rows [BSP][64 chunks + 1]: E-block writes hit 16 banks apart
constexpr int kGsRow = 80;  // gs rows [BSP][64 chunks + 16]: mix A-operand reads on disjoint bank halves
// chunk 64: the mix B operands (K rows) live in LDS instead of registers (the chunk's 17-step E
// operands leave no room for them below 128 VGPRs); K rows [BSP][L + 16]: the two 16-lane
// halves of a ds_read_b64 hit disjoint banks
template <int O, int L>
__host__ __device__ constexpr bool lti_k_lds() { return L == 64; }
template <int L>
__host__ __device__ constexpr int lti_krow() { return L + 16; }
// chunk 128 (8192-sample tiles, state / prepass modes only): ONE x buffer (two barriers per
// tile) and the E operands in LDS ([taps][BSP + 8]) -- their 33 k-steps do not fit registers
template <int L>
__host__ __device__ constexpr bool lti_x1() { return L >= 128; }
// E rows [tap][BSP + 16]: a row stride of 32 banks, so the two taps a half-wave reads (lanes
// 0-15, 16-31) land on disjoint banks
template <int O, int L>
__host__ __device__ constexpr int lti_ebr() { return lti_bsp(O) + 16; }
template <int O, int L>
__host__ __device__ constexpr size_t lti_lds_bytes(bool mix) {
    if (lti_x1<L>())
        return sizeof(double) * ((size_t)lti_xs_pad<O, L>() + 2 * (size_t)lti_bsp(O) * kZRow +
                                 (size_t)((L + O + 3) / 4 * 4) * lti_ebr<O, L>());
    return sizeof(double) * (2 * (size_t)lti_xs_pad<O, L>() + 2 * (size_t)lti_bsp(O) * kZRow +
                             (mix ? 2 * (size_t)lti_bsp(O) * kGsRow : 0) +
                             (mix && lti_k_lds<O, L>() ? (size_t)lti_bsp(O) * lti_krow<L>() : 0));
}

typedef double hz_f64x4 __attribute__((ext_vector_type(4)));

// DPP move of a double with a row mask: rows outside ROWMASK keep 0 (old), lanes whose
// source is outside the pattern read 0 (bound_ctrl).
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_dm(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), CTRL, ROWMASK, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWMASK, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// the same move with an explicit old value for the rows outside ROWMASK (a dead register of the
// caller: no zero materialised; the caller's coefficients for those rows are 0)
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_dm_old(double old, double v) {
    const long long b = __double_as_longlong(v), o = __double_as_longlong(old);
    const int lo = __builtin_amdgcn_update_dpp((int)(o & 0xffffffff), (int)(b & 0xffffffff), CTRL, ROWMASK, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp((int)(o >> 32), (int)(b >> 32), CTRL, ROWMASK, 0xf, true);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kDppWaveShr1 = 0x138;   // lane l <- lane l-1 across rows (gfx950: probed)
constexpr int kDppRowBcast15 = 0x142; // rows 1, 3 <- lane 15 of the row below (row_mask 0xa)
constexpr int kDppRowBcast31 = 0x143; // rows 2, 3 <- lane 31 (row_mask 0xc)

// One workgroup = W waves = W bands (group g = blockIdx.x) over one time segment
// (blockIdx.y).  Per tile of 64 lane chunks x L samples, three phases run one tile
// apart (one barrier per tile, every LDS image double-buffered):
//  (E) zero-state end states of every chunk for every band of the group, on the FP64
//      matrix cores: Z[chunk][bs] = X[chunk][tap] . E[tap][bs]  (v_mfma_f64_16x16x4f64;
//      A = the chunk windows read from the staged x tile, B = the group's E rows, held
//      in registers for the whole launch), written to LDS as z[bs][chunk];
//  (S) per band (wave) and chunk (lane): the inclusive 64-lane prefix of the chunk
//      recurrence s' = M s + pin z, entirely in VGPRs (row_shr 1,2,4,8 with M^(2^s),
//      row_bcast:15 with M^(p+1), row_bcast:31 with M^(l-31)), the chunk start states
//      st = Z(l-1) + M^l S (wave_shr:1) and the tile end state S' = Z(63) + M^64 S;
//      gs = gin st to LDS;
//  (M) the group's correction mix D[chunk][j] = sum_bs gs[bs][chunk] K[bs][j] on the
//      matrix cores, stored as this group's row of the partial slab.
// The (E) and (M) blocks are spread over the waves as independent work items.
template <int O, int L, int MODE>
__global__ __launch_bounds__(64 * lti_waves(O)) void fb_lti_kernel(const double* __restrict__ rec, LtiArgs a) {
    using R = RecL<O, L>;
    constexpr int W = lti_waves(O);
    constexpr int XW = R::XW;
    constexpr int T = 64 * L;
    constexpr int XS = lti_xs_len<O, L>();
    constexpr int XSP = lti_xs_pad<O, L>();
    constexpr int PF = (XS + 64 * W - 1) / (64 * W);  // x values staged per thread
    constexpr int BSP = lti_bsp(O);
    constexpr int KE = (XW + 3) / 4;                  // E k-steps (taps, zero padded)
    constexpr int NE = 4 * (BSP / 16);                // E blocks (4 chunk blocks x state blocks)
    constexpr int KM = BSP / 4;                       // mix k-steps (band states)
    constexpr int NM = (MODE == MODE_MIX) ? 4 * (L / 16) : 0;  // mix blocks (chunk blocks x sample blocks)
    // work items: E block e on wave e % W (slot e / W); mix block m on wave (NE + m) % W (slot
    // (NE % W + m) / W ... see m_item), so a wave holds at most IPE + IPM B operands
    // (Measured slower on the C2 state kernel, 0.283 ms: splitting the E blocks' k-steps over
    // two waves, 0.351 ms; wave roles -- waves 0-7 E blocks only, waves 8-15 two scans each in
    // separate loops -- 0.320 ms.  FP64 MFMA and FP64 VALU share a pipe, so overlapping them
    // across waves buys little; what the roles lose is the scan latency hidden behind the E
    // chains of the same SIMD's other waves.)
    constexpr int IPE = (NE + W - 1) / W;
    constexpr int IPM = (NM + W - 1) / W;
    // MODE_STATE with fewer E blocks than half the waves: the waves without E blocks stage the
    // x tiles alone, at the top of the iteration, from registers loaded one iteration earlier, so
    // the E waves (the critical path: MFMA chain, then their scan) never wait on x staging
    constexpr bool X1 = lti_x1<L>();   // chunk 128: one x buffer, E operands in LDS
    static_assert(!X1 || MODE != MODE_MIX, "chunk 128 runs the state / prepass modes only");
    constexpr bool kSplit = (MODE == MODE_STATE || MODE == MODE_SEGEND) && NE <= W / 2 &&
                            (64 * (W - NE)) % L == 0;
    constexpr int WS = kSplit ? W - NE : W;                  // staging waves
    constexpr int PF2 = (XS + 64 * WS - 1) / (64 * WS);      // x values per staging thread
    constexpr int EBR = lti_ebr<O, L>();
    constexpr int KER = X1 ? 1 : KE;                         // E k-steps held in registers
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* zb = lds + (X1 ? 1 : 2) * XSP;      // [2][BSP][kZRow]
    double* eb = zb + 2 * BSP * kZRow;          // X1: E rows [4 KE][EBR]
    double* gsb = zb + 2 * BSP * kZRow;  // [2][BSP][kGsRow]
    constexpr bool KL = lti_k_lds<O, L>() && MODE == MODE_MIX;
    constexpr int KR = lti_krow<L>();
    double* kb = gsb + 2 * BSP * kGsRow;  // [BSP][KR] (KL only)
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp_band0 = blockIdx.x * W;
    const int band = grp_band0 + wave;
    const bool live = band < a.nbands;
    const int bandc = live ? band : a.nbands - 1;  // dead waves run a live band's numbers, gs = 0
    const double* r = rec + (long)bandc * R::SIZE;
    const long n = a.n;
    const int seg = blockIdx.y;
    const long seg_base = (long)seg * a.seg_len;
    // the prepass may start past the segment's head: older input reaches the end state only
    // through M^k with ||M^k|| < 2^-64 (fb_lti_horizon)
    const long seg_t0 = seg_base + (MODE == MODE_SEGEND ? a.seg_skip : 0);
    const long seg_end = min(seg_base + a.seg_len, n);
    const int ntiles = (int)((seg_end - seg_t0 + T - 1) / T);
    const bool last_seg = seg == a.nseg - 1;

    double S[O];
    {
        const double* s0 = (MODE == MODE_SEGEND) ? nullptr
                         : (seg == 0) ? a.ystate + (long)bandc * O
                                      : a.segstate + ((long)bandc * a.nseg_state + (long)seg * a.seg_stride) * O;
#pragma unroll
        for (int k = 0; k < O; ++k) S[k] = (live && s0) ? s0[k] : 0.0;
    }
    const double pb = live ? a.pin[band] : 0.0;
    const double gb = live ? a.gin[band] : 0.0;

    // per-lane chunk-transition powers: M^l (carry-in), M^(p+1) (row_bcast:15), M^(l-31)
    // (row_bcast:31); loop-invariant
    // (qa is 0 on rows 0, 2 and qb on rows 0, 1: the bcast moves leave those rows' old values,
    // which are finite, and the FMAs then add exactly 0)
    double qc[O * O], qa[O * O], qb[O * O];
    {
        const int ea = (lane & 15) + 1, eb = lane >= 32 ? lane - 31 : 0;
        const bool wa = (lane >> 4) & 1, wb = lane >= 32;
#pragma unroll
        for (int e = 0; e < O * O; ++e) {
            qc[e] = r[R::QC + lane * O * O + e];
            qa[e] = wa ? r[R::QC + ea * O * O + e] : 0.0;
            qb[e] = wb ? r[R::QC + eb * O * O + e] : 0.0;
        }
    }
    // MODE_SEGEND needs only the tile's end state: sum_l M^(63-l) pin z_l (lane l = chunk l), a
    // weighted wave sum instead of the prefix scan
    double qr[O * O];
#pragma unroll
    for (int e = 0; e < O * O; ++e) qr[e] = MODE == MODE_SEGEND ? r[R::QC + (63 - lane) * O * O + e] : 0.0;

    // MFMA B operands of this wave's work items: E items hold E[tap][bs] (tap = 4q + (l >> 4),
    // bs = 16 sb + (l & 15)), mix items K[bs][j] (bs = 4q + (l >> 4), j = 16 jb + (l & 15));
    // zero outside the group / taps.  Loop-invariant: held in registers for the whole launch.
    auto e_item = [&](int v) { return wave + W * v; };                         // < NE: valid
    auto m_item = [&](int v) { return (wave - NE % W + W) % W + W * v; };     // < NM: valid
    constexpr int IPMR = KL ? 0 : IPM;   // mix B operands held in registers
    double bop_e[IPE > 0 ? IPE : 1][KER], bop_m[IPMR > 0 ? IPMR : 1][KM > 0 ? KM : 1];
    // E[tap][bs] with pin folded in: the E blocks produce pin z (the scan's input) directly
    auto e_val = [&](int tap, int bs) {
        const int bl = bs / O, k = bs % O, bnd = grp_band0 + bl;
        if (bl < W && bnd < a.nbands && tap < XW) {
            const double* rb = rec + (long)bnd * R::SIZE;
            return a.pin[bnd] * (tap < O ? rb[R::EH + k * O + tap] : (tap + k < XW ? rb[R::E0 + tap + k] : 0.0));
        }
        return 0.0;
    };
    if constexpr (X1) {   // every record / pin load of the thread issued before its LDS stores
        constexpr int NEF = 4 * KE * BSP, PTE = (NEF + 64 * W - 1) / (64 * W);
        double ev[PTE];
#pragma unroll
        for (int i = 0; i < PTE; ++i) {
            const int e = (int)threadIdx.x + i * 64 * W;
            ev[i] = e < NEF ? e_val(e / BSP, e % BSP) : 0.0;
        }
#pragma unroll
        for (int i = 0; i < PTE; ++i) {
            const int e = (int)threadIdx.x + i * 64 * W;
            if (e < NEF) eb[(e / BSP) * EBR + e % BSP] = ev[i];
        }
    }
#pragma unroll
    for (int v = 0; v < (X1 ? 0 : IPE); ++v) {
        const int item = e_item(v);
#pragma unroll
        for (int q = 0; q < KER; ++q) {
            const int sb = item >> 2, tap = 4 * q + (lane >> 4), bs = 16 * sb + (lane & 15);
            bop_e[v][q] = item < NE ? e_val(tap, bs) : 0.0;
        }
    }
    if constexpr (KL) {
        for (int e = threadIdx.x; e < BSP * L; e += 64 * W) {
            const int bs = e / L, j = e % L, bl = bs / O, k = bs % O, bnd = grp_band0 + bl;
            kb[bs * KR + j] = (bl < W && bnd < a.nbands) ? rec[(long)bnd * R::SIZE + R::K + j * O + k] : 0.0;
        }
    }
#pragma unroll
    for (int v = 0; v < IPMR; ++v) {
        const int item = m_item(v);
#pragma unroll
        for (int q = 0; q < KM; ++q) {
            double val = 0.0;
            const int jb = item >> 2, bs = 4 * q + (lane >> 4), j = 16 * jb + (lane & 15);
            const int bl = bs / O, k = bs % O, bnd = grp_band0 + bl;
            if (item < NM && bl < W && bnd < a.nbands) val = rec[(long)bnd * R::SIZE + R::K + j * O + k];
            bop_m[v][q] = val;
        }
    }

    // x staging through a buffer descriptor over x[0 .. seg_end): one 32-bit lane offset per
    // load, the segment's zero tail and the samples before the call (offsets that wrap past
    // 2^32) come back as 0 from the range check; the O history taps before the call's first
    // sample are patched in at store time.  (No 64-bit addresses or clamps in registers.)
    const __amdgpu_buffer_rsrc_t xrsrc = [&] {
        const unsigned long long xb = (unsigned long long)a.x;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)xb);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(xb >> 32));
        const int bytes = __builtin_amdgcn_readfirstlane((int)(seg_end * (long)sizeof(double)));
        return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, bytes,
                                                 0x00020000);
    }();
    auto load_x = [&](long t0x, double (&pf)[PF]) {
        const int v0 = (int)((t0x - O) * (long)sizeof(double)) + (int)threadIdx.x * (int)sizeof(double);
#pragma unroll
        for (int q = 0; q < PF; ++q)
            pf[q] = __builtin_bit_cast(   // the whole offset in voffset: soffset is outside the range check
                double, __builtin_amdgcn_raw_buffer_load_b64(xrsrc, v0 + q * 64 * W * (int)sizeof(double), 0, 0));
    };
    // in-loop tiles (t0x >= O): a descriptor based at x[t0x - O] (scalar math per tile) with
    // loop-invariant lane offsets; records past seg_end read 0
    // staging thread index: all threads, or (kSplit) the threads of waves NE .. W-1
    const int sid = kSplit ? (int)threadIdx.x - 64 * NE : (int)threadIdx.x;
    const int vq0 = sid * (int)sizeof(double);
    auto load_x_loop = [&](long t0x, double (&pf)[PF2]) {
        const unsigned long long xb = (unsigned long long)(a.x + (t0x - O));
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)xb);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(xb >> 32));
        const long rem = (seg_end - (t0x - O)) * (long)sizeof(double);
        const int bytes = __builtin_amdgcn_readfirstlane((int)(rem > 0 ? rem : 0));
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(((unsigned long long)hi << 32) | lo), (short)0, bytes, 0x00020000);
#pragma unroll
        for (int q = 0; q < PF2; ++q)
            pf[q] = __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(rs, vq0 + q * 64 * WS * (int)sizeof(double), 0, 0));
    };
    // LDS position of x[t0x - O + li] is li + P (li / L); li = tid + q 64 W with 64 W a multiple
    // of L, so position = (tid + P tid / L) + q (64 W + P 64 W / L): one base, immediate offsets
    constexpr int PC = lti_xs_padc<L>();
    const int xpos0 = (int)threadIdx.x + PC * ((int)threadIdx.x / L);
    const int xposs = sid + PC * (sid / L);
    auto store_x_loop = [&](double* xbuf, const double (&pf)[PF2]) {   // in-loop tiles (t0x > 0)
        double* xb = xbuf + xposs;
#pragma unroll
        for (int q = 0; q < PF2; ++q) {
            const int li = sid + q * 64 * WS;
            if (li < XS) xb[q * (64 * WS + PC * (64 * WS / L))] = pf[q];
        }
    };
    auto store_x = [&](double* xbuf, const double (&pf)[PF], long t0x) {
        static_assert((64 * W) % L == 0, "x staging stride must be a multiple of the chunk");
        double* xb = xbuf + xpos0;
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            const int li = threadIdx.x + q * 64 * W;
            if (li < XS) xb[q * (64 * W + PC * (64 * W / L))] = pf[q];
        }
        if (t0x == 0 && threadIdx.x < O) xbuf[threadIdx.x] = a.xhist[O - 1 - threadIdx.x];  // x[-O+li]
    };
    // chunk 128, in-loop tiles (t0x > 0): the staging waves fill the x buffer by LDS-DMA, one
    // 1-KiB piece (128 doubles = one chunk, 16 B per lane) per instruction, no registers and no
    // ds_write; the range check returns 0 past seg_end; __syncthreads() waits for the pieces
    auto dma_x = [&](double* xbuf, long t0x) {
        if constexpr (X1) {
            const unsigned long long xb = (unsigned long long)(a.x + (t0x - O));
            const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)xb);
            const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(xb >> 32));
            const long rem = (seg_end - (t0x - O)) * (long)sizeof(double);
            const int bytes = __builtin_amdgcn_readfirstlane((int)(rem > 0 ? rem : 0));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(((unsigned long long)hi << 32) | lo), (short)0, bytes, 0x00020000);
            const int sw = kSplit ? wave - NE : wave;   // staging wave index
            for (int c = sw; c <= 64; c += WS)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(xbuf + c * (L + 2)), 16,
                    (c * L + 2 * lane) * (int)sizeof(double), 0, 0, 0);
        }
    };

    // chunk 128, MODE_STATE: the GEMM's x-window rows of tile itx while the x buffer holds it
    // (row r, chunk c = x[t0 - O + c L + r] for r < L + O, else 0: piece c slot r, or piece c + 1
    // slot r - L), by the staging threads of workgroup (global tile) mod G -- the work of
    // fb_lti_xrows_kernel without its launch or a second read of x
    // (this workgroup's tiles are tg = blockIdx.x mod G: the next one is tracked, no division)
    long xr_next = (seg_t0 / T + (long)gridDim.x - 1 - (long)blockIdx.x) / (long)gridDim.x * (long)gridDim.x +
                   (long)blockIdx.x;   // first tg >= seg_t0 / T with tg mod G = blockIdx.x
    auto write_xrows = [&](int itx) {
        if constexpr (X1 && MODE == MODE_STATE) {
            constexpr int XRC = (L + O + 31) / 32 * 32;   // = lti_x_rows(L, O)
            constexpr int B = 5;   // LDS reads of a batch issued together, then their stores
            constexpr int PER = (XRC * 64 + 64 * WS * B - 1) / (64 * WS * B) * B;   // values per staging thread
            const long tg = seg_t0 / T + itx;
            if (a.xr == 0 || itx >= ntiles || tg != xr_next) return;
            xr_next += gridDim.x;
            double* g = a.gs_out + (tg * a.bs_pad + a.xr0) * 64;
#pragma unroll
            for (int q0 = 0; q0 < PER; q0 += B) {
                double v[B];
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    const int e = sid + (q0 + q) * 64 * WS;
                    const int r = e >> 6, c = e & 63;
                    v[q] = 0.0;
                    if (r < L + O) v[q] = r < L ? lds[c * (L + 2) + r] : lds[(c + 1) * (L + 2) + (r - L)];
                }
#pragma unroll
                for (int q = 0; q < B; ++q) {
                    const int e = sid + (q0 + q) * 64 * WS;
                    if (e < XRC * 64) __builtin_nontemporal_store(v[q], g + e);
                }
            }
        }
    };

    // (E) for tile te: this wave's E blocks -> z buffer (te & 1)
    auto phase_e = [&](int te) {
        const double* xs = lds + (X1 ? 0 : (te & 1) * XSP);
        double* z = zb + (te & 1) * BSP * kZRow;
#pragma unroll
        for (int v = 0; v < IPE; ++v) {
            const int item = e_item(v);  // wave-uniform
            if (item < NE) {
                const int m = item & 3, sb = item >> 2;
                // A: lane l holds X[chunk 16m + (l & 15)][tap 4q + (l >> 4)]
                const int li0 = (16 * m + (lane & 15)) * L + (lane >> 4);
                hz_f64x4 acc = {0.0, 0.0, 0.0, 0.0};
                // A operands read EP k-steps ahead of their MFMA (LDS latency under the chain)
                constexpr int EP = 4;
                auto xa_at = [&](int q) {
                    const int li = li0 + 4 * q;
                    return (4 * q + (lane >> 4) < XW) ? xs[li + PC * (li / L)] : 0.0;
                };
                // X1: B = E[tap 4q + (l >> 4)][bs 16 sb + (l & 15)] from LDS, read with A
                const double* ebl = eb + (lane >> 4) * EBR + 16 * sb + (lane & 15);
                auto eb_at = [&](int q) { return X1 ? ebl[4 * q * EBR] : 0.0; };
                double xq[EP], bq[EP];
#pragma unroll
                for (int q = 0; q < EP && q < KE; ++q) {
                    xq[q] = xa_at(q);
                    if constexpr (X1) bq[q] = eb_at(q);
                }
                __builtin_amdgcn_sched_barrier(0);   // keep the reads ahead (the scheduler sinks them)
#pragma unroll
                for (int q = 0; q < KE; ++q) {
                    const double xa = xq[q % EP];
                    const double bb = X1 ? bq[q % EP] : bop_e[v][X1 ? 0 : q];
                    if (q + EP < KE) {
                        xq[q % EP] = xa_at(q + EP);
                        if constexpr (X1) bq[q % EP] = eb_at(q + EP);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, bb, acc, 0, 0, 0);
                }
                // D: col = band state 16 sb + (l & 15), row = chunk 16 m + (l >> 4) + 4 rr
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    z[(16 * sb + (lane & 15)) * kZRow + 16 * m + (lane >> 4) + 4 * rr] = acc[rr];
            }
        }
    };
    // (M) for tile tm: this wave's mix blocks -> partial slab
    auto phase_m = [&](int tm) {
        const double* gs = gsb + (tm & 1) * BSP * kGsRow;
        const long t0m = seg_t0 + (long)tm * T;
#pragma unroll
        for (int v = 0; v < IPM; ++v) {
            const int item = m_item(v);  // wave-uniform
            if (item < NM) {
                const int m = item & 3, jb = item >> 2;
                const double* ga = gs + (lane >> 4) * kGsRow + 16 * m + (lane & 15);
                const double* kbl = kb + (lane >> 4) * KR + 16 * jb + (lane & 15);
                auto bm = [&](int q) { return KL ? kbl[4 * q * KR] : bop_m[KL ? 0 : v][q]; };
                // two accumulation chains (ILP) while registers allow; one for L = 64
                constexpr bool kTwo = L <= 32;
                hz_f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int q = 0; q < KM; q += 2) {
                    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[4 * q * kGsRow], bm(q), acc0, 0, 0, 0);
                    if (q + 1 < KM) {
                        if constexpr (kTwo)
                            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[4 * (q + 1) * kGsRow], bm(q + 1), acc1, 0,
                                                                       0, 0);
                        else
                            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ga[4 * (q + 1) * kGsRow], bm(q + 1), acc0, 0,
                                                                       0, 0);
                    }
                }
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const int chunk = 16 * m + (lane >> 4) + 4 * rr;
                    const long t = t0m + (long)chunk * L + 16 * jb + (lane & 15);
                    if (t < n) __builtin_nontemporal_store(acc0[rr] + acc1[rr], &a.partial[(long)blockIdx.x * a.n_pad + t]);
                }
            }
        }
    };

    // prologue: x tiles 0 and 1 staged (chunk 128: tile 1 after (E) of tile 0, one buffer), gs
    // padding rows zeroed, (E) of tile 0
    {
        double pf0[PF];
        load_x(seg_t0, pf0);
        store_x(lds, pf0, seg_t0);
        if constexpr (!X1) {
            double pf1[PF];
            if (ntiles > 1) {
                load_x(seg_t0 + T, pf1);
                store_x(lds + XSP, pf1, seg_t0 + T);
            }
        }
        if constexpr (MODE == MODE_MIX && BSP > W * O) {
            for (int e = threadIdx.x; e < 2 * BSP * kGsRow; e += 64 * W)
                if ((e % (BSP * kGsRow)) / kGsRow >= W * O) gsb[e] = 0.0;
        }
        __syncthreads();
        if (!kSplit || wave >= NE) write_xrows(0);
        phase_e(0);
        __syncthreads();
        if constexpr (X1) {
            if (ntiles > 1) {
                double pf1[PF];
                load_x(seg_t0 + T, pf1);
                store_x(lds, pf1, seg_t0 + T);
            }
            __syncthreads();
        }
    }
    const bool stager = !kSplit || wave >= NE;
    double pf[PF2];   // staging registers: x tile it + 2, loaded during iteration it - 1 (kSplit, X1)
    if (kSplit && !X1 && stager && ntiles > 2) load_x_loop(seg_t0 + 2 * T, pf);

    double st[O];
    double* go_run = MODE == MODE_STATE ? a.gs_out + ((seg_t0 / T) * a.bs_pad + (long)band * O) * 64 + lane : nullptr;
    const int niter = (MODE == MODE_MIX) ? ntiles + 1 : ntiles;
    auto phase_s = [&](int it, long t0) {
        if constexpr (MODE == MODE_SEGEND) {
            if (it < ntiles) {   // S' = M^64 S + sum_l M^(63-l) pin z_l
                const double* z = zb + (it & 1) * BSP * kZRow;
                double zz[O], v[O];
#pragma unroll
                for (int k = 0; k < O; ++k) zz[k] = z[(wave * O + k) * kZRow + lane];
#pragma unroll
                for (int k = 0; k < O; ++k) {
                    v[k] = 0.0;
#pragma unroll
                    for (int c = 0; c < O; ++c) v[k] = fma(qr[k * O + c], zz[c], v[k]);
                }
#pragma unroll
                for (int k = 0; k < O; ++k) {   // inclusive wave sum: lane 63 holds the total
                    v[k] += dpp_dm<kDppRowShr + 1, 0xf>(v[k]);
                    v[k] += dpp_dm<kDppRowShr + 2, 0xf>(v[k]);
                    v[k] += dpp_dm<kDppRowShr + 4, 0xf>(v[k]);
                    v[k] += dpp_dm<kDppRowShr + 8, 0xf>(v[k]);
                    v[k] += dpp_dm<kDppRowBcast15, 0xa>(v[k]);
                    v[k] += dpp_dm<kDppRowBcast31, 0xc>(v[k]);
                }
                double Sn[O];
#pragma unroll
                for (int k = 0; k < O; ++k) {
                    double sn = readlane_d(v[k], 63);
#pragma unroll
                    for (int c = 0; c < O; ++c) sn = fma(r[R::PSL + k * O + c], S[c], sn);
#pragma unroll
                    for (int c = 0; c < O; ++c) sn = fma(r[R::PS + 4 * O * O + k * O + c], S[c], sn);
                    Sn[k] = sn;
                }
#pragma unroll
                for (int k = 0; k < O; ++k) S[k] = Sn[k];
            }
            return;
        }
        if (it < ntiles) {
            // ---- (S) tile it: this wave's band ----
            const double* z = zb + (it & 1) * BSP * kZRow;
            double zz[O];
#pragma unroll
            for (int k = 0; k < O; ++k) zz[k] = z[(wave * O + k) * kZRow + lane];   // pin z (E operands)
#define HZ_LTI_SCAN_STEP(CTRL, RM, MAT)                                                               \
{                                                                                                 \
    _Pragma("unroll") for (int k = 0; k < O; ++k) nb_[k] = RM == 0xf ? dpp_dm<CTRL, RM>(zz[k])    \
                                                                   : dpp_dm_old<CTRL, RM>(nb_[k], zz[k]); \
    _Pragma("unroll") for (int rr = 0; rr < O; ++rr)                                              \
        _Pragma("unroll") for (int c = 0; c < O; ++c) zz[rr] = fma(MAT[rr * O + c], nb_[c], zz[rr]); \
}
            double nb_[O];
            const double* p1 = r + R::PS;
            const double* p2 = r + R::PS + O * O;
            const double* p4 = r + R::PS + 2 * O * O;
            const double* p8 = r + R::PS + 3 * O * O;
            HZ_LTI_SCAN_STEP(kDppRowShr + 1, 0xf, p1)
            HZ_LTI_SCAN_STEP(kDppRowShr + 2, 0xf, p2)
            HZ_LTI_SCAN_STEP(kDppRowShr + 4, 0xf, p4)
            HZ_LTI_SCAN_STEP(kDppRowShr + 8, 0xf, p8)
            HZ_LTI_SCAN_STEP(kDppRowBcast15, 0xa, qa)
            HZ_LTI_SCAN_STEP(kDppRowBcast31, 0xc, qb)
#undef HZ_LTI_SCAN_STEP
            double Sn[O];
#pragma unroll
            for (int k = 0; k < O; ++k) {
                double vv = dpp_dm<kDppWaveShr1, 0xf>(zz[k]);  // Z(l-1), 0 at lane 0
                double sn = readlane_d(zz[k], 63);
#pragma unroll
                for (int c = 0; c < O; ++c) sn = fma(r[R::PSL + k * O + c], S[c], sn);
#pragma unroll
                for (int c = 0; c < O; ++c) {
                    vv = fma(qc[k * O + c], S[c], vv);
                    sn = fma(r[R::PS + 4 * O * O + k * O + c], S[c], sn);
                }
                st[k] = vv;
                Sn[k] = sn;
            }
#pragma unroll
            for (int k = 0; k < O; ++k) S[k] = Sn[k];
            if constexpr (MODE != MODE_SEGEND) {
                if constexpr (MODE == MODE_MIX) {
                    double* gs = gsb + (it & 1) * BSP * kGsRow;
#pragma unroll
                    for (int k = 0; k < O; ++k) gs[(wave * O + k) * kGsRow + lane] = gb * st[k];
                } else {   // MODE_STATE: tile-major rows of 64 chunks, row band O + k (dead
                           // waves write the zero pad rows: gb = 0; every wave has its rows)
                    double* go = go_run;   // = gs_out + ((t0 / T) bs_pad + band O) 64 + lane
                    go_run += (long)a.bs_pad * 64;
#pragma unroll
                    for (int k = 0; k < O; ++k)
                        // unconditional: the x staging waits below count them exactly
                        __builtin_nontemporal_store(gb * st[k], go + 64 * k);   // count them exactly
                }
                if (last_seg && it == ntiles - 1 && live) {
                    // end-of-call y history = the start state of the chunk beginning at n
                    // (n is a multiple of L; chunks past n see zero input)
                    const int cn = (int)((n - t0) / L);  // in [1, 64]
                    if (cn < 64) {
                        if (lane == cn)
#pragma unroll
                            for (int k = 0; k < O; ++k) a.ystate_next[(long)band * O + k] = st[k];
                    } else if (lane == 0) {
#pragma unroll
                        for (int k = 0; k < O; ++k) a.ystate_next[(long)band * O + k] = S[k];
                    }
                }
            }
        }
    };

    if constexpr (X1) {
        // chunk 128, one x buffer, two barriers per tile: the E waves run (E) of tile it + 1 while
        // the others scan tile it; after the first barrier (x buffer free) the E waves scan and the
        // staging waves start the LDS-DMA of tile it + 2
        const bool isE = !kSplit || wave < NE;
        for (int it = 0; it < ntiles; ++it) {
            const long t0 = seg_t0 + (long)it * T;
            // (every wave scanning first, then the E chains: 0.465 vs 0.454 ms per C2 step)
            if (isE) {
                if (it + 1 < ntiles) phase_e(it + 1);
            } else {
                phase_s(it, t0);
            }
            if (!kSplit || !isE) write_xrows(it + 1);   // the buffer holds tile it + 1 until the barrier
            __syncthreads();
            if (isE) phase_s(it, t0);
            if (stager && it + 2 < ntiles) dma_x(lds, t0 + 2 * T);
            __syncthreads();
        }
    } else {
        for (int it = 0; it < niter; ++it) {
            const long t0 = seg_t0 + (long)it * T;
            const bool stage = it + 2 < ntiles;
            if constexpr (kSplit) {
                if (stager) {
                    if (stage) store_x_loop(lds + (it & 1) * XSP, pf);   // tile it + 2 (its buffer's tile it is done)
                    if (it + 3 < ntiles) load_x_loop(t0 + 3 * T, pf);
                }
            } else {
                if (stage) load_x_loop(t0 + 2 * T, pf);
            }
            // the three phases of an iteration touch disjoint LDS images.  Order E, M, S for every
            // wave: measured against scan-first orders for the E waves (0.554 vs 0.522 ms per C2
            // step) and for the mix-only waves (0.581); scan-first on the state kernel: 0.308 vs
            // 0.304 ms
            if (it + 1 < ntiles) phase_e(it + 1);
            if constexpr (MODE == MODE_MIX) {
                if (it >= 1) phase_m(it - 1);
            }
            phase_s(it, t0);
            if constexpr (!kSplit) {
                if (stage) store_x_loop(lds + (it & 1) * XSP, pf);
            }
            __syncthreads();
        }
    }

    if constexpr (MODE == MODE_SEGEND) {
        if (lane == 0 && !last_seg && live) {
#pragma unroll
            for (int k = 0; k < O; ++k) a.segstate[((long)band * a.nseg_state + seg + 1) * O + k] = S[k];
        }
    } else {
        if (last_seg && lane == 0 && live) {
            const double P0 = a.pgstate[2 * (long)band], G0 = a.pgstate[2 * (long)band + 1];
            a.pgstate_next[2 * (long)band] = pb + a.sp_n * (P0 - pb);
            a.pgstate_next[2 * (long)band + 1] = gb + a.sg_n * (G0 - gb);
        }
        if (last_seg && blockIdx.x == 0 && threadIdx.x < O) {
            const int k = threadIdx.x;
            const long idx = n - 1 - k;
            a.xhist_next[k] = idx >= 0 ? a.x[idx] : a.xhist[-idx - 1];
        }
    }
}

// Sequential carry over time segments (one thread per band), LTI records:
//   start(s+1) = M_tile^seg_tiles start(s) + zsr_end(s), M_tile = M^64 = QC[64]; the power in
//   double-double, applied as hi S + lo S (hz_dd.h).
template <int O, int L>
__global__ __launch_bounds__(256) void fb_lti_seg_carry_kernel(const double* __restrict__ rec,
                                                               const double* __restrict__ ystate,
                                                               double* __restrict__ segstate, int nbands,
                                                               int nseg, long seg_tiles) {
    using R = RecL<O, L>;
    const int band = blockIdx.x * blockDim.x + threadIdx.x;
    if (band >= nbands) return;
    const double* r = rec + (long)band * R::SIZE;
    double M[O][O], Ml[O][O];
    {
        hz_dd::dd B[O][O], Cp[O][O];
        hz_dd::load<O>(r + R::QC + 64 * O * O, r + R::PSL, B);
        hz_dd::mat_pow<O>(B, seg_tiles, Cp);
        for (int i = 0; i < O; ++i)
            for (int j = 0; j < O; ++j) {
                M[i][j] = Cp[i][j].hi;
                Ml[i][j] = Cp[i][j].lo;
            }
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
            for (int q = 0; q < O; ++q) acc = fma(Ml[i][q], Sv[q], acc);
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
// One thread per pair of samples (16-B loads down the slab's columns, kRedRows rows in flight),
// 128 threads = 256 samples per block; the group order of the sum is fixed (deterministic).
// The block's input window x[t0 - O .. t0 + 255] is staged in LDS once (every chunk window of
// the zero-state term reads it there: L + O taps per sample).
constexpr int kRedRows = 32;

template <int O, int L>
__global__ __launch_bounds__(128) void fb_lti_reduce_kernel(const double* __restrict__ partial, long n_pad, int G,
                                                            long n, const double* __restrict__ x,
                                                            const double* __restrict__ xhist,
                                                            const double* __restrict__ fmix,
                                                            double* __restrict__ out) {
    constexpr int XW = L + O;
    constexpr int NS = 256;   // samples per block (a multiple of L)
    __shared__ double fm[L * XW];
    __shared__ double xs[NS + O];
    const long t0 = (long)blockIdx.x * NS;
    for (int e = threadIdx.x; e < L * XW; e += 128) fm[e] = fmix[e];
    for (int e = threadIdx.x; e < NS + O; e += 128) {
        const long idx = t0 - O + e;
        // before the launch's first sample: the call's x history (first chunk) or the previous
        // chunk of the same input buffer (xhist == nullptr); past n: never read
        xs[e] = idx >= n ? 0.0 : (idx >= 0 || !xhist) ? x[idx] : xhist[-idx - 1];
    }
    __syncthreads();
    const long t = t0 + 2 * threadIdx.x;
    if (t >= n) return;
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 s0 = {0.0, 0.0}, s1 = {0.0, 0.0};
    const double* col = partial + t;  // n_pad is a multiple of the tile: t + 1 < n_pad
    int g = 0;
    // kRedRows slab rows in flight per thread; the slab is read once, so the loads are
    // non-temporal (no L2 / MALL allocation for data nobody reads again)
    for (; g + kRedRows <= G; g += kRedRows) {
        d2 v[kRedRows];
#pragma unroll
        for (int u = 0; u < kRedRows; ++u)
            v[u] = __builtin_nontemporal_load((const d2*)(col + (long)(g + u) * n_pad));
#pragma unroll
        for (int u = 0; u < kRedRows; u += 2) {
            s0 += v[u];
            s1 += v[u + 1];
        }
    }
    for (; g < G; ++g) s0 += *(const d2*)(col + (long)g * n_pad);
    d2 acc = s0 + s1;
    // zero-state mix (t and t + 1 are in the same chunk: L even, t even)
    const int j = (int)(t % L);
    const double* xw = xs + (t - j - t0);   // x[t - j - O + i] = xw[i]
#pragma unroll 6
    for (int i = 0; i < XW; ++i) {
        const double xv = xw[i];
        acc[0] = fma(fm[j * XW + i], xv, acc[0]);
        acc[1] = fma(fm[(j + 1) * XW + i], xv, acc[1]);
    }
    out[t] = acc[0];
    if (t + 1 < n) out[t + 1] = acc[1];
}

// Short calls (a streaming block is 4 x 256 samples): the kernel above would run on a
// handful of workgroups, each walking all G slab rows.  Here a workgroup takes 32 samples
// and splits the G rows over 16 slices (16 x 16 threads), summing the slices in a fixed
// order through LDS (deterministic; a different order than the long-call kernel).
// GEMM path, per launch: GS rows bs_pad + r (r < XR) of every tile hold the chunk input windows
// x[tc - O + r] (r < L + O; 0 above), so the GEMM's K dimension carries the zero-state term.
template <int L>
__global__ __launch_bounds__(256) void fb_lti_xrows_kernel(const double* __restrict__ x,
                                                           const double* __restrict__ xhist, int O, long n,
                                                           double* __restrict__ gs, int bs_pad, int bs_tot, int XR,
                                                           int ntiles) {
    const long e = (long)blockIdx.x * 256 + threadIdx.x;   // (tile, r, chunk)
    if (e >= (long)ntiles * XR * 64) return;
    const int c = (int)(e & 63);
    const long tr = e >> 6;
    const int r = (int)(tr % XR);
    const long tile = tr / XR;
    double v = 0.0;
    if (r < L + O) {
        const long idx = (tile * 64 + c) * L - O + r;
        v = idx >= n ? 0.0 : (idx >= 0 || !xhist) ? x[idx] : xhist[-idx - 1];
    }
    gs[(tile * bs_tot + bs_pad + r) * 64 + c] = v;
}
// ... and K rows bs_pad + r = Fmix[j][r] (0 for r >= L + O), written when Fmix changes
template <int O, int L>
__global__ __launch_bounds__(256) void fb_lti_kt_fmix_kernel(const double* __restrict__ fmix, double* __restrict__ kt,
                                                             int bs_pad, int XR) {
    const int e = blockIdx.x * 256 + threadIdx.x;   // (r, j)
    if (e >= XR * L) return;
    const int r = e / L, j = e % L;
    kt[(long)(bs_pad + r) * L + j] = r < L + O ? fmix[j * (L + O) + r] : 0.0;
}
// GEMM path: out[t] = sum over the S slices of part[s][t] (fixed order)
__global__ __launch_bounds__(256) void fb_lti_sum_kernel(const double* __restrict__ part, long n_pad, int S, long n,
                                                         double* __restrict__ out) {
    typedef double d2 __attribute__((ext_vector_type(2)));
    const long t = 2 * ((long)blockIdx.x * 256 + threadIdx.x);
    if (t >= n) return;
    const double* col = part + t;
    d2 s0 = {0.0, 0.0}, s1 = {0.0, 0.0};
    int g = 0;
    for (; g + 8 <= S; g += 8) {
        d2 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load((const d2*)(col + (long)(g + u) * n_pad));
#pragma unroll
        for (int u = 0; u < 8; u += 2) {
            s0 += v[u];
            s1 += v[u + 1];
        }
    }
    for (; g < S; ++g) s0 += __builtin_nontemporal_load((const d2*)(col + (long)g * n_pad));
    const d2 acc = s0 + s1;
    out[t] = acc[0];
    if (t + 1 < n) out[t + 1] = acc[1];
}

template <int O, int L>
__global__ __launch_bounds__(256) void fb_lti_reduce_short_kernel(const double* __restrict__ partial, long n_pad,
                                                                  int G, long n, const double* __restrict__ x,
                                                                  const double* __restrict__ xhist,
                                                                  const double* __restrict__ fmix,
                                                                  double* __restrict__ out) {
    constexpr int XW = L + O;
    constexpr int SL = 16;   // group slices
    __shared__ double fm[L * XW];
    typedef double d2 __attribute__((ext_vector_type(2)));
    __shared__ d2 part[SL][16];
    for (int e = threadIdx.x; e < L * XW; e += 256) fm[e] = fmix[e];
    const int pr = threadIdx.x & 15, sl = threadIdx.x >> 4;
    const long t = 2 * ((long)blockIdx.x * 16 + pr);
    d2 s = {0.0, 0.0};
    if (t < n) {
        // every slice row's load issued before the first add (the rolled loop waited for each
        // batch of 4 in turn); rows past 16 per slice (banks over 4096 bands) in a second pass
        const double* col = partial + t;
        constexpr int R = 16;
        d2 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int g = sl + r * SL;
            v[r] = g < G ? *(const d2*)(col + (long)g * n_pad) : d2{0.0, 0.0};
        }
#pragma unroll
        for (int r = 0; r < R; ++r) s += v[r];
        for (int g = sl + R * SL; g < G; g += SL) s += *(const d2*)(col + (long)g * n_pad);
    }
    part[sl][pr] = s;
    __syncthreads();
    if (sl != 0 || t >= n) return;
    d2 acc = part[0][pr];
#pragma unroll
    for (int q = 1; q < SL; ++q) acc += part[q][pr];
    const int j = (int)(t % L);
    const long base = t - j - O;
#pragma unroll 4
    for (int i = 0; i < XW; ++i) {
        const long idx = base + i;
        const double xv = idx >= 0 || !xhist ? x[idx] : xhist[-idx - 1];
        acc[0] = fma(fm[j * XW + i], xv, acc[0]);
        acc[1] = fma(fm[(j + 1) * XW + i], xv, acc[1]);
    }
    out[t] = acc[0];
    if (t + 1 < n) out[t + 1] = acc[1];
}

// ---- kernel selection -------------------------------------------
typedef void (*CarryKernel)(const double*, const double*, double*, int, int, long);
typedef void (*LtiKernel)(const double*, LtiArgs);
typedef void (*FmixKernel)(const double*, const double*, const double*, int, double*);
typedef void (*LtiReduceKernel)(const double*, long, int, long, const double*, const double*, const double*,
                                double*);

// geometries: (L, bands per wave, waves per group); one band per wave, 16 waves
struct LtiGeom {
    int L, nb, waves;
};
static const LtiGeom kLtiGeoms[] = {{16, 1, 16}, {32, 1, 16}, {64, 1, 16}, {128, 1, 16}};  // waves: lti_waves(O)
static_assert(kLtiGeomChunk128 == 3, "kLtiGeoms[3] is chunk 128");
constexpr int kNumLtiGeoms = 4;
static_assert(kNumLtiGeoms <= hz_fb::kLtiSets, "one record set per geometry");

template <int O, int L>
LtiKernel lti_kernel_mode(int mode) {
    static_assert(lti_lds_bytes<O, L>(true) <= 160 * 1024, "LTI kernel LDS over 160 KiB");
    if constexpr (lti_x1<L>())   // chunk 128: state and prepass modes only
        return mode == MODE_SEGEND ? fb_lti_kernel<O, L, MODE_SEGEND> : fb_lti_kernel<O, L, MODE_STATE>;
    else
        return mode == MODE_SEGEND ? fb_lti_kernel<O, L, MODE_SEGEND>
             : mode == MODE_STATE  ? fb_lti_kernel<O, L, MODE_STATE>
                                   : fb_lti_kernel<O, L, MODE_MIX>;
}

template <int O>
LtiKernel lti_kernel_geom(int geom, int mode) {
    const int L = kLtiGeoms[geom].L;
    return L == 128 ? lti_kernel_mode<O, 128>(mode)
         : L == 64  ? lti_kernel_mode<O, 64>(mode)
         : L == 32  ? lti_kernel_mode<O, 32>(mode)
                    : lti_kernel_mode<O, 16>(mode);
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
    const int L = kLtiGeoms[geom].L;
#define HZ_LTI_LDS(LL)                                                          \
    switch (O) {                                                                \
    case 1: return lti_lds_bytes<1, LL>(mix);                                   \
    case 2: return lti_lds_bytes<2, LL>(mix);                                   \
    case 3: return lti_lds_bytes<3, LL>(mix);                                   \
    default: return lti_lds_bytes<4, LL>(mix);                                  \
    }
    if (L == 16) HZ_LTI_LDS(16)
    if (L == 32) HZ_LTI_LDS(32)
    if (L == 128) HZ_LTI_LDS(128)
    HZ_LTI_LDS(64)
#undef HZ_LTI_LDS
}

#define HZ_LTI_O(TEMPLATE, O, LL) \
    (O == 1 ? TEMPLATE<1, LL> : O == 2 ? TEMPLATE<2, LL> : O == 3 ? TEMPLATE<3, LL> : TEMPLATE<4, LL>)
#define HZ_LTI_OL(TEMPLATE, O, L)                                                                    \
    (L == 16 ? HZ_LTI_O(TEMPLATE, O, 16) : L == 32 ? HZ_LTI_O(TEMPLATE, O, 32) : HZ_LTI_O(TEMPLATE, O, 64))
static CarryKernel pick_lti_carry(int O, int L) {
    return L == 128 ? HZ_LTI_O(fb_lti_seg_carry_kernel, O, 128) : HZ_LTI_OL(fb_lti_seg_carry_kernel, O, L);
}
static FmixKernel pick_fmix(int O, int L) {
    return L == 128 ? HZ_LTI_O(fb_fmix_kernel, O, 128) : HZ_LTI_OL(fb_fmix_kernel, O, L);
}
// (chunk 64 / 128 calls sum the GEMM slices with fb_lti_sum_kernel: the zero-state term is in the GEMM)
static LtiReduceKernel pick_lti_reduce(int O, int L) { return HZ_LTI_OL(fb_lti_reduce_kernel, O, L); }
static LtiReduceKernel pick_lti_reduce_short(int O, int L) { return HZ_LTI_OL(fb_lti_reduce_short_kernel, O, L); }
typedef void (*KtFmixKernel)(const double*, double*, int, int);
static KtFmixKernel pick_kt_fmix(int O, int L) {
    return L == 128 ? HZ_LTI_O(fb_lti_kt_fmix_kernel, O, 128) : HZ_LTI_O(fb_lti_kt_fmix_kernel, O, 64);
}
typedef void (*XrowsKernel)(const double*, const double*, int, long, double*, int, int, int, int);
static XrowsKernel pick_xrows(int L) { return L == 128 ? fb_lti_xrows_kernel<128> : fb_lti_xrows_kernel<64>; }
#undef HZ_LTI_OL
#undef HZ_LTI_O

}  // namespace

namespace hz_fbi {

// geometry by call length unless pinned (hz_fb_tune_lti): chunk 64 for calls of at least two of
// its 4096-sample tiles (C2: mix 0.609 -> 0.522 ms per 10 s step against chunk 32: half the scan
// work and barriers per sample), chunk 32 from two 2048-sample tiles, chunk 16 (1024-sample
// tiles) for the short streaming blocks
int fb_lti_geom(const hz_fb* h, long n) {
    if (h->lti_geom >= 0) return h->lti_geom;
    // chunk 128 from four of its 8192-sample tiles, for banks that fill the chip with at most two
    // time segments (C2: 256 groups; its 2-GPU shard 0.294 -> 0.279 ms); smaller shards keep
    // chunk 64 (finer tiles for the prepass and the GEMM: 4-GPU shard equal, 8-GPU 0.141 vs 0.164)
    const int W = lti_waves(h->order);
    if (n >= 4 * 64L * 128 && h->order > 0 && 2L * ((h->N + W - 1) / W) >= h->target_groups) return 3;
    if (n >= 2 * 64L * 64) return 2;   // chunk 64 for calls of at least two of its 4096-sample tiles
    if (n >= 2 * 64L * 32) return 1;
    return 0;
}

int fb_lti_chunk(int geom) { return kLtiGeoms[geom].L; }

// chunk 64 and 128 run the bank-wide correction as a GEMM over all band states (MODE_STATE +
// the correction GEMM, hz_fb_gemm.hip) instead of per-group mixes and the G-row slab
bool fb_lti_gemm_geom(int geom) { return kLtiGeoms[geom].L >= 64; }

// every band's smoothers at their targets (host mirror), relative to the bank's
// largest target: the LTI engine then computes the same outputs to ~2^-60
bool fb_converged(hz_fb* h) {
    if (h->converged) return true;  // targets unchanged since: the smoothers only get closer
    if (h->resp.st.dmode) return false;   // a streaming gain transient: gains moving (O(1) decay check there)
    fb_mirror_sync(h);
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
    h->converged = true;
    return true;
}

// Samples K (a multiple of 4096) after which every band's state transition satisfies
// ||M^K||_inf < 2^-64 (long double, powers of M^4096); -1 if some band needs more than 2^18.
// Segment start states then depend on the last K samples of input only (to 2^-64 of the
// state), so the prepass can skip a segment's head.
static long fb_lti_horizon(const hz_fb* h, long double bound = 0x1p-64L) {
    const int O = h->order;
    if (O == 0) return 0;
    typedef long double ld;
    long K = 0;
    for (int b = 0; b < h->N; ++b) {
        ld M[kMaxOrder][kMaxOrder] = {}, P[kMaxOrder][kMaxOrder], Q[kMaxOrder][kMaxOrder], T[kMaxOrder][kMaxOrder];
        for (int k = 0; k < O; ++k) M[0][k] = -(ld)h->B[(size_t)b * O + k];
        for (int k = 1; k < O; ++k) M[k][k - 1] = 1;
        auto mul = [&](ld (*A)[kMaxOrder], ld (*B)[kMaxOrder], ld (*C)[kMaxOrder]) {
            for (int i = 0; i < O; ++i)
                for (int j = 0; j < O; ++j) {
                    ld acc = 0;
                    for (int q = 0; q < O; ++q) acc += A[i][q] * B[q][j];
                    T[i][j] = acc;
                }
            for (int i = 0; i < O; ++i)
                for (int j = 0; j < O; ++j) C[i][j] = T[i][j];
        };
        for (int i = 0; i < O; ++i)
            for (int j = 0; j < O; ++j) P[i][j] = M[i][j];
        for (int s = 0; s < 12; ++s) mul(P, P, P);   // M^4096
        for (int i = 0; i < O; ++i)
            for (int j = 0; j < O; ++j) Q[i][j] = (i == j);
        // up to 2^21 samples: R = 0.9999 resonators (tests/eigen.cpp:26) forget in ~0.5 M
        long kb = -1;
        for (int it = 1; it <= 512; ++it) {
            mul(Q, P, Q);
            ld nrm = 0;
            for (int i = 0; i < O; ++i) {
                ld r = 0;
                for (int j = 0; j < O; ++j) r += std::fabs(Q[i][j]);
                nrm = std::max(nrm, r);
            }
            if (!(nrm == nrm)) break;   // NaN: unstable
            if (nrm < bound) {
                kb = 4096L * it;
                break;
            }
        }
        if (kb < 0) return -1;
        K = std::max(K, kb);
    }
    return K;
}

int fb_prepare_lti(hz_fb* h, int gi) {
    const int O = h->order;
    const int L = kLtiGeoms[gi].L;
    hz_fb::LtiRecSet& set = h->lti_set[gi];
    if (set.dirty) {
        const int rs = lti_rec_size(O, L);
        const size_t need = (size_t)h->N * rs;
        std::vector<double> host(need, 0.0);
        for (int b = 0; b < h->N; ++b)
            build_record_lti_any(O, L, &h->F[(size_t)b * (O + 1)], &h->B[(size_t)b * O], &host[(size_t)b * rs]);
        if (need > set.cap) {
            if (set.d_rec) HZ_TRY_HIP(hipFree(set.d_rec));
            set.d_rec = nullptr;
            HZ_TRY_HIP(hipMalloc(&set.d_rec, sizeof(double) * need));
            set.cap = need;
        }
        if (!set.d_fmix) HZ_TRY_HIP(hipMalloc(&set.d_fmix, sizeof(double) * L * (L + kMaxOrder)));
        HZ_TRY_HIP(hipMemcpyAsync(set.d_rec, host.data(), sizeof(double) * need, hipMemcpyHostToDevice, h->stream));
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));  // pageable source
        if (fb_lti_gemm_geom(gi) && O > 0) {   // K rows of every band state (+ the Fmix rows, below)
            const int bs_pad = lti_bs_rows(h->N, O), ko = lti_k_offset(O, L);
            const size_t rows = (size_t)bs_pad + lti_x_rows(L, O);
            std::vector<double> kt((size_t)bs_pad * L, 0.0);
            for (int b = 0; b < h->N; ++b)
                for (int k = 0; k < O; ++k)
                    for (int j = 0; j < L; ++j)
                        kt[((size_t)b * O + k) * L + j] = host[(size_t)b * rs + ko + j * O + k];
            if (rows * L > set.kt_cap) {
                if (set.d_kt) HZ_TRY_HIP(hipFree(set.d_kt));
                set.d_kt = nullptr;
                HZ_TRY_HIP(hipMalloc(&set.d_kt, sizeof(double) * rows * L));
                set.kt_cap = rows * L;
            }
            HZ_TRY_HIP(hipMemcpyAsync(set.d_kt, kt.data(), sizeof(double) * kt.size(), hipMemcpyHostToDevice,
                                      h->stream));
            HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        }
        set.rs = rs;
        set.dirty = false;
        set.horizon = -2;
        set.fmix_valid = false;
    }
    if (!set.fmix_valid) {
        hipLaunchKernelGGL(pick_fmix(O, L), dim3((unsigned)(L * (L + O))), dim3(256), 0, h->stream,
                           (const double*)set.d_rec, (const double*)h->d_pin, (const double*)h->d_gin, h->N,
                           set.d_fmix);
        HZ_TRY_HIP(hipGetLastError());
        if (fb_lti_gemm_geom(gi) && O > 0) {   // the GEMM's zero-state K rows
            const int XR = lti_x_rows(L, O);
            hipLaunchKernelGGL(pick_kt_fmix(O, L), dim3((unsigned)((XR * L + 255) / 256)), dim3(256), 0, h->stream,
                               (const double*)set.d_fmix, set.d_kt, lti_bs_rows(h->N, O), XR);
            HZ_TRY_HIP(hipGetLastError());
        }
        set.fmix_valid = true;
    }
    return HZ_OK;
}

// the converged engine over n samples (n a positive multiple of the chunk length)
constexpr long kShortReduce = 1L << 16;   // calls up to this length use the sliced reduce

int fb_launch_lti(hz_fb* h, int gi, const double* d_in, double* d_out, long n) {
    HZ_TRY(fb_prepare_lti(h, gi));
    hz_fb::LtiRecSet& set = h->lti_set[gi];
    const int O = h->order;
    const LtiGeom geom = kLtiGeoms[gi];
    const int L = geom.L;
    const long T = 64L * L;
    const int per = lti_waves(O);
    const int G = (h->N + per - 1) / per;
    // Chunks: the partial slab is bounded to 2^27 doubles per buffer; HZ_FB_LTI_SPLIT > 1
    // splits a long call further so that each chunk's cross-group reduce (HBM-bound) runs on
    // a second stream under the next chunk's mix kernel (FP64-bound).  Measured on MI355X
    // (C2, 480k samples): split 1 0.859 ms, 2 0.868, 3 0.857, 4 0.873 -- the reduce then
    // competes with the mix kernel for CU slots, so the default is 1.
    constexpr int slab_log2 = 27, nsplit = 1;
    const long ntiles_all = (n + T - 1) / T;
    // correction GEMM path: per chunk GS [bs_pad][chunks] + part [S][n_pad] instead of two slabs
    const bool gemm = fb_lti_gemm_geom(gi) && O > 0;
    const int bs_pad = lti_bs_rows(h->N, O);
    const int XR = gemm ? lti_x_rows(L, O) : 0;
    const int bs_tot = bs_pad + XR;   // GS rows per tile: band states, then the x-window rows
    long chunk = std::max<long>(T, (((1L << slab_log2) / std::max(1, G)) / T) * T);
    if (gemm) chunk = std::max<long>(T, (((1L << slab_log2) / bs_tot * L) / T) * T);
    if (!gemm && ntiles_all >= 8 * nsplit) chunk = std::min(chunk, ((ntiles_all + nsplit - 1) / nsplit) * T);
    // (row skews of 32..2050 doubles were measured: no effect on the reduce, which moves the
    // slab plus the mix kernel's dirty write-back at about 5.4 TB/s)
    const long n_pad_max = std::min<long>(ntiles_all * T, chunk);
    const size_t slab = (size_t)G * n_pad_max;
    constexpr int kMaxSlices = 32;   // GEMM band-state slices (rows of part)
    const size_t need = gemm ? (size_t)bs_tot * (n_pad_max / L) + (size_t)kMaxSlices * n_pad_max : 2 * slab;
    if (need > h->partial_cap) {
        if (h->d_partial) HZ_TRY_HIP(hipFree(h->d_partial));
        h->d_partial = nullptr;
        HZ_TRY_HIP(hipMalloc(&h->d_partial, sizeof(double) * need));
        h->partial_cap = need;
    }
    if (!h->stream_red) HZ_TRY_HIP(hipStreamCreateWithFlags(&h->stream_red, hipStreamNonBlocking));
    if (!h->d_xhist_red) HZ_TRY_HIP(hipMalloc(&h->d_xhist_red, sizeof(double) * kMaxOrder));
    const long nchunks = (n + chunk - 1) / chunk;
    if ((size_t)(2 * nchunks) > h->sync_ev.size()) {
        while (h->sync_ev.size() < (size_t)(2 * nchunks)) {
            hipEvent_t ne;
            HZ_TRY_HIP(hipEventCreateWithFlags(&ne, hipEventDisableTiming));
            h->sync_ev.push_back(ne);
        }
    }
    hipEvent_t* ev_mix = h->sync_ev.data();
    hipEvent_t* ev_red = h->sync_ev.data() + nchunks;
    LtiKernel kmix = pick_lti(O, gi, gemm ? MODE_STATE : MODE_MIX);
    LtiKernel kend = pick_lti(O, gi, MODE_SEGEND);
    HZ_TRY(fb_set_lds_attr((const void*)kmix));
    HZ_TRY(fb_set_lds_attr((const void*)kend));
    const size_t lds = lti_lds(O, gi, !gemm);
    const size_t lds_end = lti_lds(O, gi, false);
    // with the reduce on a second stream, the first chunk's reduce reads the call's x history
    // after later mixes rotated the ping-pong buffers: keep a copy
    const double* xhist_call = h->d_xhist[h->xcur];
    if (nchunks > 1 && !gemm) {
        HZ_TRY_HIP(hipMemcpyAsync(h->d_xhist_red, xhist_call, sizeof(double) * O, hipMemcpyDeviceToDevice,
                                  h->stream));
        xhist_call = h->d_xhist_red;
    }
    long k = 0;
    for (long off = 0; off < n; off += chunk, ++k) {
        const long len = std::min(chunk, n - off);
        const long ntiles = (len + T - 1) / T;
        long nseg = std::max<long>(1, std::min<long>(ntiles, (h->target_groups + G - 1) / G));
        long seg_tiles = (ntiles + nseg - 1) / nseg;
        nseg = (ntiles + seg_tiles - 1) / seg_tiles;
        // The prepass (zero-start end states of segments 0 .. nseg-2) runs on G (nseg - 1)
        // workgroups, a fraction of the chip when few segments are needed (2 GPUs: 128 of 256
        // CUs).  Split each prepass segment in m equal parts, m minimising the prepass rounds
        // per unit of work, ceil(G (nseg-1) m / CUs) / m; the carry kernel runs over the fine
        // segments and the mix reads every m-th start.
        // (the coarse segment may grow to a multiple of m tiles, by at most 1/32: fine boundaries
        // must fall on coarse ones)
        int m = 1;
        long skip_tiles = 0;
        if (nseg > 1) {
            const long seg_tiles0 = seg_tiles, nseg0 = nseg;
            double best = 1.0;
            long best_tiles = seg_tiles;
            for (int c = 2; c <= 8; ++c) {
                const long st = (seg_tiles + c - 1) / c;   // fine segment, tiles
                if (st < 4 || (st * c - seg_tiles) * 32 > seg_tiles) continue;
                const long ns = (ntiles + st * c - 1) / (st * c);
                const double cost = (double)((G * (ns - 1) * c + h->target_groups - 1) / h->target_groups) / c *
                                    ((double)(st * c) / seg_tiles);
                if (ns > 1 && cost < best - 1e-3) {
                    best = cost;
                    m = c;
                    best_tiles = st * c;
                }
            }
            seg_tiles = best_tiles;
            nseg = (ntiles + seg_tiles - 1) / seg_tiles;
            // ... or, when every band forgets its state within a horizon K shorter than a
            // segment, a prepass over only the last ceil(K / T) + 1 tiles of each segment
            if (set.horizon == -2) set.horizon = fb_lti_horizon(h);
            if (set.horizon >= 0) {
                const long kt = (set.horizon + T - 1) / T + 1;
                const double cost =
                    (double)((G * (nseg0 - 1) + h->target_groups - 1) / h->target_groups) * kt / seg_tiles0;
                if (kt < seg_tiles0 && cost < best - 1e-3) {
                    m = 1;
                    seg_tiles = seg_tiles0;
                    nseg = nseg0;
                    skip_tiles = seg_tiles0 - kt;
                }
            }
        }
        const long nseg_state = (nseg - 1) * m + 1;
        h->plan_nseg = nseg;
        h->plan_skip_tiles = skip_tiles;
        h->plan_fine = m;
        h->plan_chunk = L;
        if (nseg > 1) {
            const size_t sneed = (size_t)h->N * nseg_state * O;
            if (sneed > h->seg_cap) {
                HZ_TRY_HIP(hipStreamSynchronize(h->stream));
                if (h->d_seg) HZ_TRY_HIP(hipFree(h->d_seg));
                h->d_seg = nullptr;
                HZ_TRY_HIP(hipMalloc(&h->d_seg, sizeof(double) * sneed));
                h->seg_cap = sneed;
            }
        }
        double* slab_k = h->d_partial + (size_t)(k & 1) * slab;
        const long nc_pad = ntiles * 64;   // chunks of the launch (GEMM path)
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
        a.partial = slab_k;
        a.gs_out = h->d_partial;
        a.bs_pad = bs_tot;
        a.xr0 = bs_pad;
        a.xr = (gemm && L >= 128) ? XR : 0;   // chunk 128: x rows from the state kernel
        a.segstate = h->d_seg;
        a.n = len;
        a.n_pad = ntiles * T;
        a.seg_len = seg_tiles * T;
        a.nseg = (int)nseg;
        a.nseg_state = (int)nseg_state;
        a.seg_stride = m;
        a.seg_skip = 0;
        a.nbands = h->N;
        a.sp_n = (double)powl((long double)h->sp, (long double)len);
        a.sg_n = (double)powl((long double)h->sg, (long double)len);
        hipEvent_t* e = nullptr;
        if (k >= 2 && !gemm) HZ_TRY_HIP(hipStreamWaitEvent(h->stream, ev_red[k - 2], 0));  // slab buffer k & 1 free
        (void)0;
        if (h->prof) {
            HZ_TRY(fb_prof_events(h, &e));
            HZ_TRY_HIP(hipEventRecord(e[0], h->stream));
        }
        if (nseg > 1) {
            LtiArgs af = a;   // the prepass over fine segments (never the last one)
            af.seg_len = seg_tiles / m * T;
            af.nseg = (int)nseg_state + 1;
            af.seg_stride = 1;
            af.seg_skip = skip_tiles * T;
            hipLaunchKernelGGL(kend, dim3(G, (unsigned)(nseg_state - 1)), dim3(64 * lti_waves(O)), lds_end,
                               h->stream, (const double*)set.d_rec, af);
            HZ_TRY_HIP(hipGetLastError());
            hipLaunchKernelGGL(pick_lti_carry(O, L), dim3((unsigned)((h->N + 255) / 256)), dim3(256), 0, h->stream,
                               (const double*)set.d_rec, (const double*)h->d_ystate[h->scur], h->d_seg, h->N,
                               (int)nseg_state, seg_tiles / m);
            HZ_TRY_HIP(hipGetLastError());
        }
        if (e && nseg > 1) HZ_TRY_HIP(hipEventRecord(e[1], h->stream));
        else if (e) h->ev_skip[(e - h->ev.data()) / 5] |= 2;
        if (gemm && bs_pad > lti_group_rows(h->N, O)) {   // GS rows no group writes: zero
            const int gr = lti_group_rows(h->N, O);
            HZ_TRY_HIP(hipMemset2DAsync(h->d_partial + (size_t)gr * 64, sizeof(double) * bs_tot * 64, 0,
                                        sizeof(double) * (bs_pad - gr) * 64, (size_t)ntiles, h->stream));
        }
        if (gemm && a.xr == 0) {   // the x-window rows (zero-state term) of every tile
            const long cnt = ntiles * XR * 64L;
            hipLaunchKernelGGL(pick_xrows(L), dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, h->stream,
                               a.x, off == 0 ? xhist_call : nullptr, O, len, h->d_partial, bs_pad, bs_tot, XR,
                               (int)ntiles);
            HZ_TRY_HIP(hipGetLastError());
        }
        hipLaunchKernelGGL(kmix, dim3(G, (unsigned)nseg), dim3(64 * lti_waves(O)), lds, h->stream,
                           (const double*)set.d_rec, a);
        HZ_TRY_HIP(hipGetLastError());
        if (e) HZ_TRY_HIP(hipEventRecord(e[2], h->stream));
        if (gemm) {
            // correction GEMM over band-state slices (>= 4 workgroups per CU), then the slice sum
            // + zero-state term in the reduce kernel; one stream, chunks in sequence
            double* part = h->d_partial + (size_t)bs_tot * nc_pad;
            if (e) h->ev_skip[(e - h->ev.data()) / 5] |= 8;   // reduce start = mix end
            int S = 1;
            HZ_TRY(fb_lti_gemm_launch(h->d_partial, set.d_kt, bs_tot, part, a.n_pad, (int)ntiles, L, h->target_groups,
                                      kMaxSlices, h->stream, &S));
            hipLaunchKernelGGL(fb_lti_sum_kernel, dim3((unsigned)((len + 511) / 512)), dim3(256), 0, h->stream,
                               (const double*)part, a.n_pad, S, len, d_out + off);
            HZ_TRY_HIP(hipGetLastError());
            if (e) HZ_TRY_HIP(hipEventRecord(e[4], h->stream));
            h->xcur ^= 1;
            h->scur ^= 1;
            h->prof_launches += h->prof ? 1 : 0;
            fb_mirror_advance(h, len);
            continue;
        }
        // one chunk: the reduce stays on the caller's stream (no cross-stream round trip)
        hipStream_t rs = nchunks > 1 ? h->stream_red : h->stream;
        if (nchunks > 1) {
            HZ_TRY_HIP(hipEventRecord(ev_mix[k], h->stream));
            HZ_TRY_HIP(hipStreamWaitEvent(rs, ev_mix[k], 0));
        }
        if (e) HZ_TRY_HIP(hipEventRecord(e[3], rs));
        if (len <= kShortReduce)   // streaming blocks: slices of the slab rows per workgroup
            hipLaunchKernelGGL(pick_lti_reduce_short(O, L), dim3((unsigned)((len + 31) / 32)), dim3(256), 0, rs,
                               (const double*)slab_k, a.n_pad, G, len, a.x, off == 0 ? xhist_call : nullptr,
                               (const double*)set.d_fmix, d_out + off);
        else
            hipLaunchKernelGGL(pick_lti_reduce(O, L), dim3((unsigned)((len + 255) / 256)), dim3(128), 0, rs,
                               (const double*)slab_k, a.n_pad, G, len, a.x, off == 0 ? xhist_call : nullptr,
                               (const double*)set.d_fmix, d_out + off);
        HZ_TRY_HIP(hipGetLastError());
        if (e) HZ_TRY_HIP(hipEventRecord(e[4], rs));
        if (nchunks > 1) HZ_TRY_HIP(hipEventRecord(ev_red[k], rs));
        h->xcur ^= 1;
        h->scur ^= 1;
        h->prof_launches += h->prof ? 1 : 0;
        fb_mirror_advance(h, len);
    }
    // the caller's stream sees the whole output
    if (nchunks > 1 && !gemm) HZ_TRY_HIP(hipStreamWaitEvent(h->stream, ev_red[nchunks - 1], 0));
    return HZ_OK;
}

long fb_horizon(const hz_fb* h, int log2_bound) { return fb_lti_horizon(h, ldexpl(1.0L, log2_bound)); }

int fb_lti_prepare_end(hz_fb* h, long len) { return fb_prepare_lti(h, len % (64L * 128) == 0 ? kLtiGeomChunk128 : 2); }

}  // namespace hz_fbi

extern "C" {

int hz_fb_lti_last_chunk(hz_fb* h, int* chunk) {
    if (!h || !chunk) return HZ_E_INVALID;
    *chunk = h->plan_chunk;
    return HZ_OK;
}

int hz_fb_lti_plan(hz_fb* h, long* nseg, long* skip_tiles, int* fine_parts) {
    if (!h) return HZ_E_INVALID;
    if (nseg) *nseg = h->plan_nseg;
    if (skip_tiles) *skip_tiles = h->plan_skip_tiles;
    if (fine_parts) *fine_parts = h->plan_fine;
    return HZ_OK;
}

int hz_fb_tune_lti(hz_fb* h, int chunk, int bands_per_wave, int waves_per_group) {
    if (!h) return HZ_E_INVALID;
    if (!chunk && !bands_per_wave && !waves_per_group) {
        h->lti_geom = -1;  // by call length
        return HZ_OK;
    }
    for (int g = 0; g < kNumLtiGeoms; ++g)
        if (kLtiGeoms[g].L == chunk && kLtiGeoms[g].nb == bands_per_wave && kLtiGeoms[g].waves == waves_per_group) {
            h->lti_geom = g;
            return HZ_OK;
        }
    hz::set_error("hz_fb_tune_lti: (chunk, bands/wave, waves) must be one of (16,1,16), (32,1,16), (64,1,16), "
                  "(128,1,16)");
    return HZ_E_INVALID;
}

}  // extern "C"
