// hz_fb_gemm.hip -- the converged Filterbank engine's bank-wide correction as one GEMM
// (chunk-64 calls; hz_fb_lti.hip runs MODE_STATE before it and the slice/zero-state reduce
// after it).  Built with -mllvm -amdgpu-mfma-vgpr-form=1 (Makefile): the accumulators stay in
// VGPRs instead of being copied between AGPRs and VGPRs around the k loop.
//
// With GS[bs][c] = gin_n x (start state k of band n at chunk c), bs = n O + k, and K[bs][j] the
// bands' homogeneous responses (the K rows of the LTI records), the correction of chunk c is
//     D[c][j] = sum_bs GS[bs][c] K[bs][j]      (j < 64)
// Reducing over ALL band states inside the MFMA K dimension leaves no per-group slab: the only
// intermediate is GS, N O (n / 64) doubles -- 4x fewer bytes than the G x n slab of the
// per-group mix at chunk 64.
#include <cstdlib>

#include "hz_fb_impl.h"

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// Workgroup = 4 waves x 16 chunks (64 chunks = one tile) x the 64 samples of a chunk (4 MFMA
// blocks), over one slice of the band states (blockIdx.y).  GS is tile-major
// ([tile][bs_pad][64 chunks]): a wave's A operands are one contiguous 128-B run per band state,
// read once (non-temporal) straight into registers.  The B operands (K rows, shared by the 4
// waves) are staged once per workgroup in LDS, kD k-steps (16 band states) per stage, double
// buffered: the next stage's A and B loads are in flight under this stage's MFMAs.
// GS and K rows past N O are zero (bs_pad is a multiple of 4); part[slice][t] is summed, with
// the zero-state term, by fb_lti_reduce_kernel.
constexpr int kBRow = 64 + 16;        // LDS row: the two 16-lane halves of a ds_read_b64 on disjoint banks

// RB: tiles (16-chunk row blocks per wave) per workgroup; kD: k-steps (4 band states each) per stage;
// ABL (diagnostics, HZ_FB_GEMM_ABL; wrong results): bit 0 skips the GS loads, bit 1 the K loads
template <int RB, int kD, int ABL = 0>
__global__ __launch_bounds__(256) void fb_lti_gemm_kernel(const double* __restrict__ gs,
                                                          const double* __restrict__ kt, int kslice, int bs_pad,
                                                          int ntiles, double* __restrict__ part, long n_pad) {
    constexpr int L = 64;
    constexpr int kRows = 4 * kD;         // band states per stage
    __shared__ __attribute__((aligned(16))) double bsh[2][kRows * kBRow];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int tile0 = blockIdx.x * RB;
    const int b0 = blockIdx.y * kslice;
    const int b1 = min(bs_pad, b0 + kslice);
    const int nst = (b1 - b0 + kRows - 1) / kRows;       // stages; rows past b1 read as 0
    f64x4 acc[RB][4];
#pragma unroll
    for (int t = 0; t < RB; ++t)
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) acc[t][jb] = f64x4{0.0, 0.0, 0.0, 0.0};
    // A: lane (r = l >> 4, c = l & 15) of k-step u in stage s, tile t: GS row b0 + 16 s + 4 u + r
    // of tile tile0 + t (a last odd tile reads tile0's rows again and is not stored)
    const double* ap[RB];
#pragma unroll
    for (int t = 0; t < RB; ++t) {
        const int tt = tile0 + t < ntiles ? tile0 + t : tile0;
        ap[t] = gs + ((long)tt * bs_pad + b0 + (lane >> 4)) * 64 + 16 * wave + (lane & 15);
    }
    // B staging: thread t moves K[b0 + kRows s + 16 h + (t >> 4)][4 (t & 15) .. + 3], h < kD / 4
    constexpr int BH = kD / 4;
    const int brow = threadIdx.x >> 4, bcol = 4 * (threadIdx.x & 15);
    const double* bp = kt + (long)(b0 + brow) * L + bcol;
    typedef double d2 __attribute__((ext_vector_type(2)));
    // full stages load unguarded; only a slice's last stage can hold rows past b1
    const int nfull = (b1 - b0) / kRows;
    auto load_a = [&](int s, double (&av)[RB][kD]) {
        if constexpr ((ABL & 1) != 0) {
#pragma unroll
            for (int t = 0; t < RB; ++t)
#pragma unroll
                for (int u = 0; u < kD; ++u) av[t][u] = 1e-3 * (u + s);
            return;
        }
#pragma unroll
        for (int t = 0; t < RB; ++t) {
            if (s < nfull) {
#pragma unroll
                for (int u = 0; u < kD; ++u)
                    av[t][u] = __builtin_nontemporal_load(ap[t] + (long)(kRows * s + 4 * u) * 64);
            } else {
#pragma unroll
                for (int u = 0; u < kD; ++u) {
                    const int row = kRows * s + 4 * u + (lane >> 4);
                    av[t][u] = b0 + row < b1 ? __builtin_nontemporal_load(ap[t] + (long)(kRows * s + 4 * u) * 64)
                                             : 0.0;
                }
            }
        }
    };
    auto load_b = [&](int s, d2 (&bv)[BH][2]) {
        if constexpr ((ABL & 2) != 0) {
#pragma unroll
            for (int h = 0; h < BH; ++h) bv[h][0] = bv[h][1] = d2{1e-3 * s, 2e-3};
            return;
        }
#pragma unroll
        for (int h = 0; h < BH; ++h) {
            const bool ok = s < nfull || b0 + kRows * s + 16 * h + brow < b1;
            const d2 z = {0.0, 0.0};
            const double* q = bp + (long)(kRows * s + 16 * h) * L;
            bv[h][0] = ok ? *(const d2*)q : z;
            bv[h][1] = ok ? *(const d2*)(q + 2) : z;
        }
    };
    auto store_b = [&](int buf, const d2 (&bv)[BH][2]) {
#pragma unroll
        for (int h = 0; h < BH; ++h) {
            *(d2*)&bsh[buf][(16 * h + brow) * kBRow + bcol] = bv[h][0];
            *(d2*)&bsh[buf][(16 * h + brow) * kBRow + bcol + 2] = bv[h][1];
        }
    };
    double an[RB][kD];
    d2 bn[BH][2];
    if (nst > 0) {
        load_a(0, an);
        load_b(0, bn);
        store_b(0, bn);
    }
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
        double ac[RB][kD];
#pragma unroll
        for (int t = 0; t < RB; ++t)
#pragma unroll
            for (int u = 0; u < kD; ++u) ac[t][u] = an[t][u];
        const bool more = s + 1 < nst;
        if (more) {
            load_a(s + 1, an);
            load_b(s + 1, bn);
        }
        const double* bs = bsh[s & 1] + (lane >> 4) * kBRow + (lane & 15);
#pragma unroll
        for (int u = 0; u < kD; ++u) {
            const double* bu = bs + 4 * u * kBRow;
            double bv[4];
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) bv[jb] = bu[16 * jb];
#pragma unroll
            for (int t = 0; t < RB; ++t)
#pragma unroll
                for (int jb = 0; jb < 4; ++jb)
                    acc[t][jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[t][u], bv[jb], acc[t][jb], 0, 0, 0);
        }
        if (more) store_b((s + 1) & 1, bn);
        __syncthreads();
    }
    // D: row = chunk (tile 64 + 16 wave) + (l >> 4) + 4 rr, column = sample 16 jb + (l & 15)
#pragma unroll
    for (int t = 0; t < RB; ++t) {
        if (tile0 + t >= ntiles) break;
        const long c0 = (long)(tile0 + t) * 64 + 16 * wave;
        double* out = part + (long)blockIdx.y * n_pad + (c0 + (lane >> 4)) * L + (lane & 15);
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) out[4 * rr * L + 16 * jb] = acc[t][jb][rr];
    }
}

// Full-stage variant: every slice is an even number of 16-band-state stages (bs_pad and kslice
// multiples of 32), so no load is guarded, and the loop is unrolled by two over ping-pong A
// registers and B buffers with no exit between the halves (no register copies between stages).
// L = 64 or 128 samples per chunk (L / 16 accumulator blocks per wave).
// PADB: LDS row padding of the B stage (doubles; HZ_FB_GEMM_PADB experiments: C2 GEMM + sum
// 0.190 / 0.191 / 0.181 / 0.182 / 0.185 ms for 16 / 8 / 4 / 2 / 1).  The staging
// writes are interleaved (d2 v of a thread at column 2 (t & 15) + 32 v) so that one ds_write_b128
// covers 256 consecutive bytes of a row.
// WJ: sample-column parts per chunk block: the workgroup is 4 WJ waves, wave (cb, jh) = (w & 3,
// w >> 2) computes chunks 16 cb .. 16 cb + 15 x samples jh L / WJ .. (jh + 1) L / WJ (L / (16 WJ)
// accumulators): fewer registers per wave (more waves per CU) and one B stage shared by more waves.
// Measured at C2 (HZ_FB_GEMM_WJ=2, 2 / 3 / 4 workgroups per CU): GEMM + sum 0.234 / 0.193 / 0.190
// ms against 0.181 for WJ = 1 -- the default stays 1
template <int L, int PADB = 4, int WJ = 1>
__global__ __launch_bounds__(256 * WJ) void fb_lti_gemm_pp_kernel(const double* __restrict__ gs,
                                                                  const double* __restrict__ kt, int kslice,
                                                                  int bs_pad, int ntiles, double* __restrict__ part,
                                                                  long n_pad) {
    constexpr int kD = 4, kRows = 16, JB = L / (16 * WJ), BR = L + PADB;
    constexpr int TPR = 16 * WJ, BV = L / (2 * TPR);   // threads per B row, d2 per thread
    __shared__ __attribute__((aligned(16))) double bsh[2][kRows * BR];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cb = wave & 3, j0 = (wave >> 2) * (L / WJ);
    const int tile = blockIdx.x;
    const int b0 = blockIdx.y * kslice;
    const int nst = (min(bs_pad, b0 + kslice) - b0) / kRows;
    f64x4 acc[JB];
#pragma unroll
    for (int jb = 0; jb < JB; ++jb) acc[jb] = f64x4{0.0, 0.0, 0.0, 0.0};
    const double* ap = gs + ((long)tile * bs_pad + b0 + (lane >> 4)) * 64 + 16 * cb + (lane & 15);
    const int brow = threadIdx.x / TPR, bcol = 2 * (threadIdx.x % TPR);
    const double* bp = kt + (long)(b0 + brow) * L + bcol;
    typedef double d2 __attribute__((ext_vector_type(2)));
    auto load_a = [&](int st, double (&av)[kD]) {
#pragma unroll
        for (int u = 0; u < kD; ++u) av[u] = __builtin_nontemporal_load(ap + (long)(kRows * st + 4 * u) * 64);
    };
    auto load_b = [&](int st, d2 (&bv)[BV]) {
        const double* q = bp + (long)(kRows * st) * L;
#pragma unroll
        for (int v = 0; v < BV; ++v) bv[v] = *(const d2*)(q + 2 * TPR * v);
    };
    auto store_b = [&](int buf, const d2 (&bv)[BV]) {
#pragma unroll
        for (int v = 0; v < BV; ++v) *(d2*)&bsh[buf][brow * BR + bcol + 2 * TPR * v] = bv[v];
    };
    auto compute = [&](int buf, const double (&av)[kD]) {
        const double* bs = bsh[buf] + (lane >> 4) * BR + j0 + (lane & 15);
#pragma unroll
        for (int u = 0; u < kD; ++u) {
            const double* bu = bs + 4 * u * BR;
            double bv[JB];
#pragma unroll
            for (int jb = 0; jb < JB; ++jb) bv[jb] = bu[16 * jb];
#pragma unroll
            for (int jb = 0; jb < JB; ++jb) acc[jb] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[jb], acc[jb], 0, 0, 0);
        }
    };
    double a0[kD], a1[kD];
    d2 bq[BV];
    if (nst > 0) {
        load_a(0, a0);
        load_b(0, bq);
        store_b(0, bq);
    }
    if (nst > 1) {
        load_a(1, a1);
        load_b(1, bq);
    }
    __syncthreads();
    for (int st = 0; st < nst; st += 2) {   // nst is even
        compute(0, a0);   // stage st
        if (st + 2 < nst) load_a(st + 2, a0);
        store_b(1, bq);
        if (st + 2 < nst) load_b(st + 2, bq);
        __syncthreads();
        compute(1, a1);   // stage st + 1
        if (st + 3 < nst) load_a(st + 3, a1);
        if (st + 2 < nst) store_b(0, bq);
        if (st + 3 < nst) load_b(st + 3, bq);
        __syncthreads();
    }
    const long c0 = (long)tile * 64 + 16 * cb;
    double* out = part + (long)blockIdx.y * n_pad + (c0 + (lane >> 4)) * L + j0 + (lane & 15);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
        for (int jb = 0; jb < JB; ++jb) out[4 * rr * L + 16 * jb] = acc[jb][rr];
}

}  // namespace

namespace hz_fbi {

int fb_lti_gemm_launch(const double* gs, const double* kt, int bs_pad, double* part, long n_pad, int ntiles, int L,
                       int target_groups, int max_slices, hipStream_t stream, int* slices_out) {
    static const int rb = [] {   // tuning experiments: HZ_FB_GEMM_RB = 1 or 2 tiles per workgroup
        const char* e = std::getenv("HZ_FB_GEMM_RB");
        return e && e[0] == '2' ? 2 : 1;
    }();
    // (measured on C2: 2 tiles per workgroup, 8-step stages and 2 or 8 workgroups per CU were all
    // slower than 1 / 4 / 4: 0.224 / 0.224 / 0.237 / 0.219 vs 0.219 ms with the reduce)
    static const int kd = [] {   // HZ_FB_GEMM_KD = 4 or 8 k-steps per stage
        const char* e = std::getenv("HZ_FB_GEMM_KD");
        return e && e[0] == '8' ? 8 : 4;
    }();
    static const int occ = [] {  // HZ_FB_GEMM_OCC: workgroups wanted per CU (slice count)
        const char* e = std::getenv("HZ_FB_GEMM_OCC");
        const int v = e ? std::atoi(e) : 6;   // (C2, full-stage kernel: 3 / 4 / 5 / 6 per CU ->
        return v >= 1 && v <= 16 ? v : 6;      //  0.222 / 0.215 / 0.214 / 0.210 ms with the reduce)
    }();
    if (bs_pad % 4 != 0 || ntiles <= 0) {
        hz::set_error("fb_lti_gemm_launch: bad geometry (bs_pad %d, tiles %d)", bs_pad, ntiles);
        return HZ_E_INVALID;
    }
    // band-state slices: >= occ workgroups per CU, each slice a multiple of 4 band states
    const int gx = (ntiles + rb - 1) / rb;
    // at least 512 band states per slice: shard-sized banks (bs_pad 1024-4096) gain from fewer
    // slices for the reduce to sum (emulated 2 / 4 / 8-GPU shard steps 0.323 / 0.206 / 0.155 ->
    // 0.313 / 0.204 / 0.148 ms); C2 on one GPU keeps 9 slices
    static const int mink = [] {  // HZ_FB_GEMM_MINK: fewest band states per slice
        const char* e = std::getenv("HZ_FB_GEMM_MINK");
        const int v = e ? std::atoi(e) : 512;
        return v >= 0 ? v : 512;
    }();
    int S = std::min(max_slices, std::max(1, (occ * target_groups + gx - 1) / gx));
    if (mink > 0) S = std::max(1, std::min(S, bs_pad / mink));
    S = std::min(S, bs_pad / 4);
    // full-stage kernel (default): slices of whole 16-row stages; HZ_FB_GEMM_PP=0 keeps the guarded one
    static const bool pp = !(std::getenv("HZ_FB_GEMM_PP") && std::getenv("HZ_FB_GEMM_PP")[0] == '0');
    const bool full = (pp && rb == 1 && kd == 4) || L != 64;   // chunk 128: the full-stage kernel only
    if (bs_pad % 32 != 0 || (L != 64 && L != 128)) {
        hz::set_error("fb_lti_gemm_launch: bad geometry (bs_pad %d, chunk %d)", bs_pad, L);
        return HZ_E_INVALID;
    }
    const int kslice = full ? ((bs_pad + S - 1) / S + 31) & ~31
                            : ((bs_pad + S - 1) / S + 3) & ~3;   // (stages past b1 read as 0)
    S = (bs_pad + kslice - 1) / kslice;
    static const int abl = std::getenv("HZ_FB_GEMM_ABL") ? std::atoi(std::getenv("HZ_FB_GEMM_ABL")) : 0;
    auto k = rb == 2 ? (kd == 8 ? fb_lti_gemm_kernel<2, 8> : fb_lti_gemm_kernel<2, 4>)
                     : (kd == 8 ? fb_lti_gemm_kernel<1, 8> : fb_lti_gemm_kernel<1, 4>);
    if (abl == 1) k = fb_lti_gemm_kernel<1, 4, 1>;
    if (abl == 2) k = fb_lti_gemm_kernel<1, 4, 2>;
    if (abl == 3) k = fb_lti_gemm_kernel<1, 4, 3>;
    static const int padb = std::getenv("HZ_FB_GEMM_PADB") ? std::atoi(std::getenv("HZ_FB_GEMM_PADB")) : 4;
    static const int wj = std::getenv("HZ_FB_GEMM_WJ") ? std::atoi(std::getenv("HZ_FB_GEMM_WJ")) : 1;
    int threads = 256;
    if (full && abl == 0) {
        k = L == 128 ? fb_lti_gemm_pp_kernel<128> : fb_lti_gemm_pp_kernel<64>;
        if (wj == 2) {
            k = L == 128 ? fb_lti_gemm_pp_kernel<128, 4, 2> : fb_lti_gemm_pp_kernel<64, 4, 2>;
            threads = 512;
        }
        if (padb == 16) k = L == 128 ? fb_lti_gemm_pp_kernel<128, 16> : fb_lti_gemm_pp_kernel<64, 16>;
        if (padb == 8) k = L == 128 ? fb_lti_gemm_pp_kernel<128, 8> : fb_lti_gemm_pp_kernel<64, 8>;
        if (padb == 2) k = L == 128 ? fb_lti_gemm_pp_kernel<128, 2> : fb_lti_gemm_pp_kernel<64, 2>;
        if (padb == 1) k = L == 128 ? fb_lti_gemm_pp_kernel<128, 1> : fb_lti_gemm_pp_kernel<64, 1>;
    }
    hipLaunchKernelGGL(k, dim3((unsigned)gx, (unsigned)S), dim3(threads), 0, stream, gs, kt, kslice, bs_pad, ntiles,
                       part, n_pad);
    HZ_TRY_HIP(hipGetLastError());
    *slices_out = S;
    return HZ_OK;
}

}  // namespace hz_fbi
