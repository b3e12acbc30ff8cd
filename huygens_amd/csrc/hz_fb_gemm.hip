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
constexpr int kD = 4;                 // k-steps (4 band states each) per stage
constexpr int kRows = 4 * kD;         // band states per stage
constexpr int kBRow = 64 + 16;        // LDS row: the two 16-lane halves of a ds_read_b64 on disjoint banks

__global__ __launch_bounds__(256) void fb_lti_gemm_kernel(const double* __restrict__ gs,
                                                          const double* __restrict__ kt, int kslice, int bs_pad,
                                                          double* __restrict__ part, long n_pad) {
    constexpr int L = 64;
    __shared__ __attribute__((aligned(16))) double bsh[2][kRows * kBRow];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const long c0 = (long)blockIdx.x * 64 + 16 * wave;   // this wave's 16 chunks
    const int b0 = blockIdx.y * kslice;
    const int b1 = min(bs_pad, b0 + kslice);
    const int nst = (b1 - b0 + kRows - 1) / kRows;       // stages; rows past b1 read as 0
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    // A: lane (r = l >> 4, c = l & 15) of k-step u in stage s: GS row b0 + 16 s + 4 u + r
    const double* ap = gs + ((long)blockIdx.x * bs_pad + b0 + (lane >> 4)) * 64 + 16 * wave + (lane & 15);
    // B staging: thread t moves K[b0 + 16 s + (t >> 4)][4 (t & 15) .. + 3] (two 16-B loads)
    const int brow = threadIdx.x >> 4, bcol = 4 * (threadIdx.x & 15);
    const double* bp = kt + (long)(b0 + brow) * L + bcol;
    typedef double d2 __attribute__((ext_vector_type(2)));
    // full stages load unguarded; only a slice's last stage can hold rows past b1
    const int nfull = (b1 - b0) / kRows;
    auto load_a = [&](int s, double (&av)[kD]) {
        if (s < nfull) {
#pragma unroll
            for (int u = 0; u < kD; ++u) av[u] = __builtin_nontemporal_load(ap + (long)(16 * s + 4 * u) * 64);
        } else {
#pragma unroll
            for (int u = 0; u < kD; ++u) {
                const int row = 16 * s + 4 * u + (lane >> 4);
                av[u] = b0 + row < b1 ? __builtin_nontemporal_load(ap + (long)(16 * s + 4 * u) * 64) : 0.0;
            }
        }
    };
    auto load_b = [&](int s, d2 (&bv)[2]) {
        const bool ok = s < nfull || b0 + 16 * s + brow < b1;
        const d2 z = {0.0, 0.0};
        bv[0] = ok ? *(const d2*)(bp + (long)16 * s * L) : z;
        bv[1] = ok ? *(const d2*)(bp + (long)16 * s * L + 2) : z;
    };
    auto store_b = [&](int buf, const d2 (&bv)[2]) {
        *(d2*)&bsh[buf][brow * kBRow + bcol] = bv[0];
        *(d2*)&bsh[buf][brow * kBRow + bcol + 2] = bv[1];
    };
    double an[kD];
    d2 bn[2];
    if (nst > 0) {
        load_a(0, an);
        load_b(0, bn);
        store_b(0, bn);
    }
    __syncthreads();
    for (int s = 0; s < nst; ++s) {
        double ac[kD];
#pragma unroll
        for (int u = 0; u < kD; ++u) ac[u] = an[u];
        const bool more = s + 1 < nst;
        if (more) {
            load_a(s + 1, an);
            load_b(s + 1, bn);
        }
        const double* bs = bsh[s & 1] + (lane >> 4) * kBRow + (lane & 15);
#pragma unroll
        for (int u = 0; u < kD; ++u) {
            const double* bu = bs + 4 * u * kBRow;
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[u], bu[0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[u], bu[16], acc1, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[u], bu[32], acc2, 0, 0, 0);
            acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(ac[u], bu[48], acc3, 0, 0, 0);
        }
        if (more) store_b((s + 1) & 1, bn);
        __syncthreads();
    }
    // D: row = chunk c0 + (l >> 4) + 4 rr, column = sample 16 jb + (l & 15) of the chunk
    double* out = part + (long)blockIdx.y * n_pad + (c0 + (lane >> 4)) * L + (lane & 15);
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
        out[4 * rr * L] = acc0[rr];
        out[4 * rr * L + 16] = acc1[rr];
        out[4 * rr * L + 32] = acc2[rr];
        out[4 * rr * L + 48] = acc3[rr];
    }
}

}  // namespace

namespace hz_fbi {

int fb_lti_gemm_launch(const double* gs, const double* kt, int kslice, int bs_pad, double* part, long n_pad,
                       int ntiles, int slices, hipStream_t stream) {
    if (bs_pad % 4 != 0 || kslice % 4 != 0 || ntiles <= 0 || slices <= 0) {
        hz::set_error("fb_lti_gemm_launch: bad geometry (bs_pad %d, kslice %d)", bs_pad, kslice);
        return HZ_E_INVALID;
    }
    hipLaunchKernelGGL(fb_lti_gemm_kernel, dim3((unsigned)ntiles, (unsigned)slices), dim3(256), 0, stream, gs, kt,
                       kslice, bs_pad, part, n_pad);
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

}  // namespace hz_fbi
