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

// Every slice is an even number of 16-band-state stages (bs_pad and kslice multiples of 32), so
// no load is guarded, and the loop is unrolled by two over ping-pong A registers and B buffers with
// no exit between the halves (no register copies between stages).  L = 64 or 128 samples per
// chunk (L / 16 accumulator blocks per wave).  The B stage rows are padded by 4 doubles and
// written interleaved (d2 v of a thread at column 2 (t & 15) + 32 v), so one ds_write_b128 covers
// 256 consecutive bytes of a row and the reads hit no bank conflicts.  (Measured and dropped in
// round 2, C2 GEMM + sum: row padding 16 / 8 / 2 / 1 -- 0.190 / 0.191 / 0.182 / 0.185 vs 0.181 ms;
// 8-wave workgroups splitting the sample columns -- 0.190-0.234 ms; a guarded kernel with 2 tiles
// per workgroup or 8-step stages, 2 or 8 workgroups per CU -- 0.219-0.237 vs 0.210 ms.)
template <int L>
__global__ __launch_bounds__(256) void fb_lti_gemm_pp_kernel(const double* __restrict__ gs,
                                                                  const double* __restrict__ kt, int kslice,
                                                                  int bs_pad, int ntiles, double* __restrict__ part,
                                                                  long n_pad) {
    constexpr int kD = 4, kRows = 16, JB = L / 16, BR = L + 4;
    constexpr int TPR = 16, BV = L / (2 * TPR);   // threads per B row, d2 per thread
    __shared__ __attribute__((aligned(16))) double bsh[2][kRows * BR];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int cb = wave & 3, j0 = 0;
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
    if (bs_pad % 32 != 0 || ntiles <= 0 || (L != 64 && L != 128)) {
        hz::set_error("fb_lti_gemm_launch: bad geometry (bs_pad %d, tiles %d, chunk %d)", bs_pad, ntiles, L);
        return HZ_E_INVALID;
    }
    // band-state slices: >= 6 workgroups per CU (C2: 3 / 4 / 5 / 6 per CU -> 0.222 / 0.215 / 0.214
    // / 0.210 ms with the reduce), at least 512 band states each (shard-sized banks gain from fewer
    // slices for the reduce to sum: emulated 2 / 4 / 8-GPU shard steps 0.323 / 0.206 / 0.155 ->
    // 0.313 / 0.204 / 0.148 ms), each slice a whole number of 32-row stage pairs
    constexpr int kOcc = 6, kMinRows = 512;
    int S = std::min(max_slices, std::max(1, (kOcc * target_groups + ntiles - 1) / ntiles));
    S = std::max(1, std::min(S, bs_pad / kMinRows));
    const int kslice = ((bs_pad + S - 1) / S + 31) & ~31;
    S = (bs_pad + kslice - 1) / kslice;
    hipLaunchKernelGGL(L == 128 ? fb_lti_gemm_pp_kernel<128> : fb_lti_gemm_pp_kernel<64>, dim3((unsigned)ntiles,
                       (unsigned)S), dim3(256), 0, stream, gs, kt, kslice, bs_pad, ntiles, part, n_pad);
    HZ_TRY_HIP(hipGetLastError());
    *slices_out = S;
    return HZ_OK;
}

}  // namespace hz_fbi
