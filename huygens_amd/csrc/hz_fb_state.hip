// hz_fb_state.hip -- the band-state pass of the stationary engine (hz_fb_resp.hip): every band's
// zero-start state after a window of len samples (len a multiple of 8192),
//     S_n = sum_c M_n^(C-1-c) pin_n E_n x_c        (c < C = len / 128 chunks of 128 samples)
// with E_n the chunk's zero-state end-state map over its L + O input taps and M_n the chunk
// transition (the chunk-128 LTI records, hz_fb_rec.h; the band recurrence of
// src/filterbank.h:178-179 restated chunk-wise).  That is N O len multiply-adds, ~0.8 GFLOP at
// C2 (4096 bands, O = 2, len = 49152): the pass is bound by the FP64 matrix cores (78.6 TFLOP/s).
//
// Work split: one workgroup = 32 band-state columns (16 bands of O = 2; OP = O padded to a power
// of two columns per band) x one time segment; 4 waves, wave m owns chunk rows 16m..16m+15 of
// every 8192-sample tile (64 chunks).  Per tile a wave runs two independent chains of 33
// v_mfma_f64_16x16x4f64 (one per 16-column block) whose accumulator starts from M^64 applied to
// the previous tiles' sum, so after the last tile accumulator row c holds
//     A_c = sum_tiles M^(64 (T-1-t)) z_{t,c},   z_{t,c} = pin E x_{t,c}
// and S = sum_c M^(63-c) A_c (one weighted reduction at the end, across lanes and waves).
//   * B operands (pin E, 66 doubles per lane) stay in registers for the whole launch;
//   * A operands (the chunk windows, X[chunk][tap] = x[t0 - O + 128 chunk + tap]) come from the
//     wave's own LDS slab of its 16 chunks, staged a tile ahead through registers with coalesced
//     buffer loads (the x window, 8 B x len, is read from HBM once per XCD and is L2-resident):
//     no barrier in the loop, the waves of a workgroup never wait for each other (the first
//     version read A straight from L2 with 16-chunk gathers: 33 us at C2 against 11 us of MFMA);
//   * the O taps before the window are the zero-start history: their offsets wrap past 2^32
//     and the buffer range check returns 0 for them (and for taps past the window's end, whose
//     E entries are 0).
// Banks too small to fill the chip split the window into time segments (grid.y): each
// segment's zero-start partial goes to a scratch row, the last segment workgroup of a band
// group to arrive (device-scope counter) combines them, S = sum_s P^(m-1-s) S_s, P = M^(len/m),
// and re-arms the counter.
#include "hz_fb_impl.h"
#include "hz_fb_rec.h"

namespace {

using namespace hz_fbi;

constexpr int kL = 128;             // chunk (samples)
constexpr int kTile = 64 * kL;      // 8192 samples per tile
constexpr int kCols = 32;           // band-state columns per workgroup (two 16-wide MFMA blocks)
constexpr int kSlab = 16 * kL + 4;  // a wave's x slab per tile: 16 chunks + the last chunk's taps past it
constexpr int kSlabPieces = 17;    // L-sample pieces of a slab (16 chunks + the taps past the last)
constexpr int kSlabPos = kSlabPieces * (kL + 2);   // with 2 pad slots per piece (16-B aligned pieces)
constexpr int kStage = (kSlab + 63) / 64;     // register staging loads per lane of tile 0 (33)

template <int O>
struct StateGeom {
    static constexpr int OP = O == 3 ? 4 : O;       // columns per band
    static constexpr int BANDS = kCols / OP;        // bands per workgroup
    static constexpr int XW = kL + O;               // chunk input taps
    static constexpr int KE = (XW + 3) / 4;         // MFMA k-steps (4 taps each)
};

typedef double f64x4 __attribute__((ext_vector_type(4)));

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

// One tile of a wave's chain: tile it + 1's pieces of the wave's share of row block m's slab go
// into `nxt` by LDS-DMA (1 KiB per instruction, 16 B per lane from the x window), then the 33
// k-steps read their A operands from `cur` (4 ahead of the MFMAs).  `cur` and `nxt` are restrict:
// inlined here, the compiler knows the DMA does not write what the reads read and issues no wait
// between them (with one plain pointer it made every read wait for the newest DMA).
template <int KE, int OP>
__device__ __forceinline__ void state_tile(const double* __restrict__ cur, double* __restrict__ nxt, bool dma,
                                           __amdgpu_buffer_rsrc_t xr, int voff, int sb, int a_pos,
                                           const double (&e)[KE], const double (&m64)[OP], bool carry, f64x4& acc) {
    if (dma) {
#pragma unroll
        for (int i = 0; i < (kSlabPieces + 1) / 2; ++i) {
            const int p = 2 * i + sb;   // wave-uniform
            if (p < kSlabPieces)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    xr, (__attribute__((address_space(3))) void*)(nxt + p * (kL + 2)), 16,
                    voff + p * kL * (int)sizeof(double), 0, 0, 0);
        }
    }
    if (carry) {   // acc <- M^64 acc (the previous tiles, one tile further back)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) acc[rr] = mix_cols<OP>(m64, acc[rr]);
    }
    auto a_at = [&](int q) {
        const int t = 4 * q;   // + (l >> 4) < 4: taps 128.. of the last k-step sit after the pad
        return t < kL ? cur[a_pos + t] : cur[a_pos + t + 2];
    };
    constexpr int EP = 4;
    double xq[EP];
#pragma unroll
    for (int q = 0; q < EP; ++q) xq[q] = a_at(q);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < KE; ++q) {
        const double xa = xq[q % EP];
        if (q + EP < KE) xq[q % EP] = a_at(q + EP);
        __builtin_amdgcn_sched_barrier(0);
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, e[q], acc, 0, 0, 0);
    }
}

struct StateArgs {
    const double* rec;     // chunk-128 records [N][rs]
    int rs;                // record size (doubles)
    const double* eop;     // [G][2][KE][64] pin E operands (fb_state_ops_kernel)
    const double* x;       // [len] the window
    long len;
    int nbands;
    int tps;               // tiles per segment
    int nseg;              // segments (grid.y)
    double* part;          // [G][nseg][kCols] segment partials (nseg > 1)
    unsigned* count;       // [G] arrival counters (nseg > 1; 0 between launches)
    double* out;           // [N][O]
};

template <int O>
__global__ __launch_bounds__(512) void fb_state_kernel(StateArgs a) {
    using R = RecL<O, kL>;
    using Gm = StateGeom<O>;
    constexpr int OP = Gm::OP, KE = Gm::KE;
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int m = w & 3;                       // chunk rows 16m .. 16m + 15 of every tile
    const int sb = w >> 2;                     // column block 16 sb .. 16 sb + 15
    const int g = blockIdx.x, seg = blockIdx.y;
    const int col = lane & 15;                 // column within the block
    const int k = col % OP;                    // state component of the column
    const int band = g * Gm::BANDS + (16 * sb + col) / OP;
    const bool live = band < a.nbands && k < O;
    // B operands, pin E[tap 4q + (l >> 4)][column] (fb_state_ops_kernel's layout: coalesced)
    double e[KE];
#pragma unroll
    for (int q = 0; q < KE; ++q) e[q] = a.eop[(((long)g * 2 + sb) * KE + q) * 64 + lane];
    // rows k of the band's M^e (QC[e], e <= 64) as weights of the columns k ^ j: M^64 (the tile
    // carry), then for the end: M^4 (rows 4 apart in a lane), M^(3 - (l >> 4)) (the lane groups)
    // and M^(16 (3 - m)) (the row blocks)
    auto qrow = [&](int ex, double (&wt)[OP]) {
        const double* rb = a.rec + (long)(live ? band : 0) * a.rs + R::QC + ex * O * O;
#pragma unroll
        for (int j = 0; j < OP; ++j) wt[j] = (live && (k ^ j) < O) ? rb[k * O + (k ^ j)] : 0.0;
    };
    double m64[OP], m4[OP], mg[OP], mw[OP];
    qrow(64, m64);
    qrow(4, m4);
    qrow(3 - (lane >> 4), mg);
    qrow(16 * (3 - m), mw);
    // row block m's slab of every tile: x[t0 + it T + 16m L - O + e], e < kSlab (its 16 chunks'
    // taps) at LDS pos(e) = e + 2 (e / L): 17 pieces of L samples, piece p at p (L + 2) (A reads of
    // 16 chunks x 4 taps hit distinct banks per half-wave); waves m and m + 4 (the two column
    // blocks) share it.  Two slab sets: tile it + 1 arrives by LDS-DMA (state_tile) while tile it
    // is read; one barrier per tile.  Tile 0 of the window (its O taps before the window read as
    // 0, at any O) is staged through registers.
    const __amdgpu_buffer_rsrc_t xr = [&] {
        const unsigned long long xb = (unsigned long long)a.x;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)xb);
        const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(xb >> 32));
        const int bytes = __builtin_amdgcn_readfirstlane((int)(a.len * (long)sizeof(double)));
        return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), (short)0, bytes,
                                                 0x00020000);
    }();
    __shared__ __attribute__((aligned(16))) double slab_a[4][kSlabPos];
    __shared__ __attribute__((aligned(16))) double slab_b[4][kSlabPos];
    const long t0 = (long)seg * a.tps * kTile;
    {   // tile 0 through registers (element-wise range check: the taps before the window are 0)
        constexpr int kHalf = (kStage + 1) / 2;
        const int i0 = sb * kHalf;
        const int v = (int)((t0 - O + (long)(16 * m) * kL + lane + 64 * i0) * (long)sizeof(double));
        double st[kHalf];
#pragma unroll
        for (int i = 0; i < kHalf; ++i)
            st[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, v + 512 * i, 0, 0));
#pragma unroll
        for (int i = 0; i < kHalf; ++i) {
            const int e = lane + 64 * (i0 + i);
            if (e < kSlab) slab_a[m][e + 2 * (e / kL)] = st[i];
        }
    }
    // tile it's DMA offset (16 B per lane: piece p = x[t0 + it T + 16m L - O + p L + 2 lane (+1)])
    auto voff = [&](int it) {
        return (int)((t0 + (long)it * kTile - O + (long)(16 * m) * kL + 2 * lane) * (long)sizeof(double));
    };
    // A operand of k-step q: X[chunk c = l & 15][tap t = 4q + (l >> 4)] = slab element 128 c + t
    const int a_pos = (lane & 15) * (kL + 2) + (lane >> 4);
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    __syncthreads();   // tile 0's ds_writes
    // tile it in slab set it & 1, tile it + 1 arriving in the other; after a tile, this wave's
    // pieces of the next have landed (vmcnt) and every wave is past this one (barrier)
    for (int it = 0; it < a.tps; it += 2) {
        state_tile<KE, OP>(slab_a[m], slab_b[m], it + 1 < a.tps, xr, voff(it + 1), sb, a_pos, e, m64, it > 0, acc);
        if (it + 1 >= a.tps) break;
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0); expcnt, lgkmcnt at their maxima (no wait)
        __syncthreads();
        state_tile<KE, OP>(slab_b[m], slab_a[m], it + 2 < a.tps, xr, voff(it + 2), sb, a_pos, e, m64, true, acc);
        if (it + 2 >= a.tps) break;
        __builtin_amdgcn_s_waitcnt(0x0f70);
        __syncthreads();
    }
    // S = sum_c M^(63-c) A_c, lane rows c = 16m + g + 4 rr (g = l >> 4), by Horner steps: over rr
    // with M^4 (anchored at row 16m + g + 12), M^(3-g) (row 16m + 15), the sum over g, M^(16(3-m))
    // (row 63), then the sum over the row blocks
    double T = acc[0];
#pragma unroll
    for (int rr = 1; rr < 4; ++rr) T = mix_cols<OP>(m4, T) + acc[rr];
    T = mix_cols<OP>(mg, T);
    T += __shfl_xor(T, 16);
    T += __shfl_xor(T, 32);
    const double v = mix_cols<OP>(mw, T);
    __shared__ double red[4][kCols];
    __shared__ int is_last;
    if (lane < 16) red[m][16 * sb + lane] = v;
    __syncthreads();
    const int t = threadIdx.x;
    if (t < kCols) {
        const double S = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
        const int b = g * Gm::BANDS + t / OP, kk = t % OP;
        if (a.nseg == 1) {
            if (b < a.nbands && kk < O) a.out[(long)b * O + kk] = S;
        } else {
            a.part[((long)g * a.nseg + seg) * kCols + t] = S;
            __threadfence();   // the partial visible at agent scope before the arrival below
        }
    }
    if (a.nseg == 1) return;
    // segments: the last workgroup of this band group to arrive combines the partials
    __syncthreads();
    if (t == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.count + g, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        is_last = prev == (unsigned)(a.nseg - 1);
    }
    __syncthreads();
    if (!is_last) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    if (t < Gm::BANDS) {
        const int b = g * Gm::BANDS + t;
        if (b < a.nbands) {
            // P = (M^64)^tps, by squaring
            const double* M64 = a.rec + (long)b * a.rs + R::QC + 64 * O * O;
            double P[O][O], Pw[O][O], Tm[O][O];
            for (int i = 0; i < O; ++i)
                for (int j = 0; j < O; ++j) {
                    Pw[i][j] = M64[i * O + j];
                    P[i][j] = i == j ? 1.0 : 0.0;
                }
            for (int ex = a.tps; ex > 0; ex >>= 1) {
                if (ex & 1) {
                    for (int i = 0; i < O; ++i)
                        for (int j = 0; j < O; ++j) {
                            double s = 0.0;
                            for (int q = 0; q < O; ++q) s = fma(P[i][q], Pw[q][j], s);
                            Tm[i][j] = s;
                        }
                    for (int i = 0; i < O; ++i)
                        for (int j = 0; j < O; ++j) P[i][j] = Tm[i][j];
                }
                for (int i = 0; i < O; ++i)
                    for (int j = 0; j < O; ++j) {
                        double s = 0.0;
                        for (int q = 0; q < O; ++q) s = fma(Pw[i][q], Pw[q][j], s);
                        Tm[i][j] = s;
                    }
                for (int i = 0; i < O; ++i)
                    for (int j = 0; j < O; ++j) Pw[i][j] = Tm[i][j];
            }
            double S[O];
            const double* p0 = a.part + (long)g * a.nseg * kCols + t * OP;
            for (int i = 0; i < O; ++i) S[i] = p0[i];
            for (int s = 1; s < a.nseg; ++s) {
                const double* ps = p0 + (long)s * kCols;
                double nS[O];
                for (int i = 0; i < O; ++i) {
                    double acc2 = ps[i];
                    for (int q = 0; q < O; ++q) acc2 = fma(P[i][q], S[q], acc2);
                    nS[i] = acc2;
                }
                for (int i = 0; i < O; ++i) S[i] = nS[i];
            }
            for (int i = 0; i < O; ++i) a.out[(long)b * O + i] = S[i];
        }
    }
    if (t == 0) __hip_atomic_store(a.count + g, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// pin E in the state kernel's B-operand order, eop[((g 2 + sb) KE + q) 64 + lane] =
// pin E[tap 4q + (lane >> 4)][column 16 sb + (lane & 15)] of band group g (zero outside the bank,
// the taps and O): one coalesced load per operand instead of 8 records per load
template <int O>
__global__ __launch_bounds__(256) void fb_state_ops_kernel(const double* __restrict__ rec, int rs,
                                                           const double* __restrict__ pin, int nbands, int G,
                                                           double* __restrict__ eop) {
    using R = RecL<O, kL>;
    using Gm = StateGeom<O>;
    constexpr int OP = Gm::OP, KE = Gm::KE, XW = Gm::XW;
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)G * 2 * KE * 64) return;
    const int lane = (int)(i & 63), q = (int)((i >> 6) % KE), sb = (int)((i / (64 * KE)) % 2);
    const int g = (int)(i / (128L * KE));
    const int col = lane & 15, k = col % OP, tap = 4 * q + (lane >> 4);
    const int band = g * Gm::BANDS + (16 * sb + col) / OP;
    double v = 0.0;
    if (band < nbands && k < O && tap < XW) {
        const double* rb = rec + (long)band * rs;
        v = pin[band] * (tap < O ? rb[R::EH + k * O + tap] : (tap + k < XW ? rb[R::E0 + tap + k] : 0.0));
    }
    eop[i] = v;
}

typedef void (*StateOpsKernel)(const double*, int, const double*, int, int, double*);
StateOpsKernel pick_state_ops(int O) {
    switch (O) {
    case 1: return fb_state_ops_kernel<1>;
    case 2: return fb_state_ops_kernel<2>;
    case 3: return fb_state_ops_kernel<3>;
    default: return fb_state_ops_kernel<4>;
    }
}

int state_ke(int O) { return (kL + O + 3) / 4; }

typedef void (*StateKernel)(StateArgs);
StateKernel pick_state(int O) {
    switch (O) {
    case 1: return fb_state_kernel<1>;
    case 2: return fb_state_kernel<2>;
    case 3: return fb_state_kernel<3>;
    default: return fb_state_kernel<4>;
    }
}

int bands_per_group(int O) { return kCols / (O == 3 ? 4 : O); }

}  // namespace

namespace hz_fbi {

// the records and the pin E operands for the current coefficients and pre-amp targets, on h->stream
int fb_state_prepare(hz_fb* h) {
    const int O = h->order;
    HZ_TRY(fb_lti_prepare_end(h, kTile));   // the chunk-128 records
    hz_fb::LtiRecSet& set = h->lti_set[kLtiGeomChunk128];
    hz_fb::Resp& R = h->resp;
    const int G = (h->N + bands_per_group(O) - 1) / bands_per_group(O);
    const size_t need = (size_t)G * 2 * state_ke(O) * 64;
    if (need > R.sop_cap) {
        HZ_TRY_HIP(hipStreamSynchronize(h->stream));
        if (R.d_sop) HZ_TRY_HIP(hipFree(R.d_sop));
        R.d_sop = nullptr;
        HZ_TRY_HIP(hipMalloc(&R.d_sop, sizeof(double) * need));
        R.sop_cap = need;
    }
    hipLaunchKernelGGL(pick_state_ops(O), dim3((unsigned)((need + 255) / 256)), dim3(256), 0, h->stream,
                       (const double*)set.d_rec, set.rs, (const double*)h->d_pin, h->N, G, R.d_sop);
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

int fb_state_window(hz_fb* h, const double* x, long len, double* out, hipStream_t st) {
    const int O = h->order;
    if (O == 0 || len <= 0 || len % kTile != 0 || len > (1L << 27) || !h->resp.d_sop) {
        hz::set_error("fb_state_window: order %d, window %ld (a positive multiple of 8192), operands %s", O, len,
                      h->resp.d_sop ? "ready" : "missing");
        return HZ_E_INVALID;
    }
    hz_fb::LtiRecSet& set = h->lti_set[kLtiGeomChunk128];
    const int G = (h->N + bands_per_group(O) - 1) / bands_per_group(O);
    const int ntiles = (int)(len / kTile);
    // time segments while the band groups leave CUs idle: the largest m <= target / G dividing
    // the tile count
    int nseg = std::max(1, std::min(ntiles, h->target_groups / G));
    while (ntiles % nseg != 0) --nseg;
    hz_fb::Resp& R = h->resp;
    if (nseg > 1) {
        const size_t need = (size_t)G * nseg * kCols;
        if (need > R.spart_cap) {
            HZ_TRY_HIP(hipStreamSynchronize(st));
            if (R.d_spart) HZ_TRY_HIP(hipFree(R.d_spart));
            R.d_spart = nullptr;
            HZ_TRY_HIP(hipMalloc(&R.d_spart, sizeof(double) * need));
            R.spart_cap = need;
        }
        if ((size_t)G > R.scount_cap) {
            HZ_TRY_HIP(hipStreamSynchronize(st));
            if (R.d_scount) HZ_TRY_HIP(hipFree(R.d_scount));
            R.d_scount = nullptr;
            HZ_TRY_HIP(hipMalloc(&R.d_scount, sizeof(unsigned) * G));
            HZ_TRY_HIP(hipMemset(R.d_scount, 0, sizeof(unsigned) * G));
            R.scount_cap = G;
        }
    }
    StateArgs a;
    a.rec = set.d_rec;
    a.rs = set.rs;
    a.eop = R.d_sop;
    a.x = x;
    a.len = len;
    a.nbands = h->N;
    a.tps = ntiles / nseg;
    a.nseg = nseg;
    a.part = R.d_spart;
    a.count = R.d_scount;
    a.out = out;
    hipLaunchKernelGGL(pick_state(O), dim3((unsigned)G, (unsigned)nseg), dim3(512), 0, st, a);
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

}  // namespace hz_fbi
