// hz_fb_state.hip -- the stationary engine's band-state pass (hz_fb_state.h): the B-operand
// preparation, the standalone kernel (calls shorter than the horizon, LAZY states, orders 3-4) and
// the host side of both launch forms (standalone, or pieces inside the transform kernels).
#include "hz_fb_state.h"

#ifdef HZ_DIAG_STAMPS
#include <cstdio>
#include <map>
#endif

namespace {

using namespace hz_fbi;
using namespace hz_state;

template <int O>
__global__ __launch_bounds__(kThreads) void fb_state_kernel(StateArgs a) {
    __shared__ StateLds L;
    state_group<O>(a, blockIdx.x, blockIdx.y, L);
}

// orders <= 2 within 256 registers: two waves per SIMD, room for other kernels' waves beside it
// the pieces' partials of a pass run inside another kernel, combined per band
template <int O>
__global__ __launch_bounds__(256) void fb_state_combine_kernel(StateArgs a) {
    using Gm = StateGeom<O>;
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= a.nbands) return;
    const int g = b / Gm::BANDS, t = b % Gm::BANDS;
    combine_pieces<O>(a, b, a.part + (long)g * a.nseg * kCols + t * Gm::OP, a.tps);
}

template <int O>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2))) void fb_state_kernel_w2(StateArgs a) {
    __shared__ StateLds L;
    state_group<O>(a, blockIdx.x, blockIdx.y, L);
}

// a band group's block for the state pass (hz_fb_state.h, grp_doubles<O>): per band its row --
// pin E_0[i] (i < XW; zeros to kEh), pin E_H[k O + i] (k, i < O) -- then the M^e weights
// W[sb][col][p][j] = row k of M^pow_of(p) at column k ^ j (the chunk-128 records' QC powers;
// zero where k ^ j >= O or past the bank): one coalesced block per workgroup instead of record
// gathers from HBM at its start and end
template <int O>
__global__ __launch_bounds__(256) void fb_state_ops_kernel(const double* __restrict__ rec, int rs,
                                                           const double* __restrict__ pin, int nbands, int G,
                                                           double* __restrict__ eop) {
    using R = RecL<O, kL>;
    using Gm = StateGeom<O>;
    constexpr int OP = Gm::OP, XW = Gm::XW, kGrpO = grp_doubles<O>(), kEO = grp_e<O>();
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long)G * kGrpO) return;
    const int g = (int)(i / kGrpO), r = (int)(i % kGrpO);
    double v = 0.0;
    if (r < kEO) {
        const int band = g * Gm::BANDS + r / kEs, e = r % kEs;
        if (band < nbands) {
            const double* rb = rec + (long)band * rs;
            if (e < XW) v = pin[band] * rb[R::E0 + e];
            else if (e >= kEh && e - kEh < O * O) v = pin[band] * rb[R::EH + (e - kEh)];
        }
    } else {
        const int w = r - kEO, j = w & 3, p = (w >> 2) % kPows, sc = w / (4 * kPows);   // sc = sb 16 + col
        const int sb = sc / 16, col = sc % 16, k = col % OP;
        const int band = g * Gm::BANDS + (16 * sb + col) / OP;
        if (sb < 2 && j < OP && band < nbands && k < O && (k ^ j) < O)
            v = p == 9 ? rec[(long)band * rs + R::PSL + k * O + (k ^ j)]
                       : rec[(long)band * rs + R::QC + pow_of(p) * O * O + k * O + (k ^ j)];
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

typedef void (*StateKernel)(StateArgs);
StateKernel pick_state(int O) {
    switch (O) {
    case 1: return fb_state_kernel_w2<1>;
    case 2: return fb_state_kernel_w2<2>;
    case 3: return fb_state_kernel<3>;
    default: return fb_state_kernel<4>;
    }
}

}  // namespace

namespace hz_fbi {

// the records and the pin E operands for the current coefficients and pre-amp targets, on h->stream
int fb_state_prepare(hz_fb* h) {
    const int O = h->order;
    HZ_TRY(fb_lti_prepare_end(h, kTile));   // the chunk-128 records
    hz_fb::LtiRecSet& set = h->lti_set[kLtiGeomChunk128];
    hz_fb::Resp& R = h->resp;
    const int G = (h->N + bands_per_group(O) - 1) / bands_per_group(O);
    const size_t need = (size_t)G * grp_doubles(O);
    if (need > R.sop_cap) {
        HZ_TRY_HIP(hipDeviceSynchronize());
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

// the pass's arguments and piece count (time pieces while the band groups leave CUs idle: the
// largest m <= target / G dividing the tile count)
static int state_args(hz_fb* h, const double* x, long len, double* out, StateArgs* a) {
    const int O = h->order;
    if (O == 0 || len <= 0 || len % kTile != 0 || len > (1L << 27) || !h->resp.d_sop) {
        hz::set_error("fb_state_window: order %d, window %ld (a positive multiple of 8192), operands %s", O, len,
                      h->resp.d_sop ? "ready" : "missing");
        return HZ_E_INVALID;
    }
    hz_fb::LtiRecSet& set = h->lti_set[kLtiGeomChunk128];
    const int G = (h->N + bands_per_group(O) - 1) / bands_per_group(O);
    const int ntiles = (int)(len / kTile);
    int nseg = std::max(1, std::min(ntiles, h->target_groups / G));
    while (ntiles % nseg != 0) --nseg;
    hz_fb::Resp& R = h->resp;
    if (nseg > 1) {
        const size_t need = (size_t)G * nseg * kCols;
        if (need > R.spart_cap) {
            HZ_TRY_HIP(hipDeviceSynchronize());
            if (R.d_spart) HZ_TRY_HIP(hipFree(R.d_spart));
            R.d_spart = nullptr;
            HZ_TRY_HIP(hipMalloc(&R.d_spart, sizeof(double) * need));
            R.spart_cap = need;
        }
        if ((size_t)G > R.scount_cap) {
            HZ_TRY_HIP(hipDeviceSynchronize());
            if (R.d_scount) HZ_TRY_HIP(hipFree(R.d_scount));
            R.d_scount = nullptr;
            HZ_TRY_HIP(hipMalloc(&R.d_scount, sizeof(unsigned) * G));
            HZ_TRY_HIP(hipMemset(R.d_scount, 0, sizeof(unsigned) * G));
            R.scount_cap = G;
        }
    }
    *a = StateArgs();
    a->rec = set.d_rec;
    a->rs = set.rs;
    a->eop = R.d_sop;
    a->x = x;
    a->len = len;
    a->nbands = h->N;
    a->G = G;
    a->tps = ntiles / nseg;
    a->nseg = nseg;
    a->part = R.d_spart;
    a->count = R.d_scount;
    a->out = out;
    a->deferred = 0;
    a->stamps = nullptr;
#ifdef HZ_DIAG_STAMPS
    static long long* d_st = nullptr;
    if (!d_st) HZ_TRY_HIP(hipMalloc(&d_st, sizeof(long long) * 4 * 64 * 8192));
    a->stamps = d_st;
#endif
    return HZ_OK;
}

#ifdef HZ_DIAG_STAMPS
// (diagnostic builds) the last launch's workgroup stamps: state workgroups [0, G nseg) (start,
// loop start, loop end, HW id), then the inverse kernel's nfft transform workgroups (start, end, end,
// HW id); which of them shared a CU while running
void fb_state_stamps_dump(const StateArgs& a, int nfft, long call) {
    const int n = a.G * a.nseg, nt = n + nfft;
    std::vector<long long> v((size_t)nt * 4);
    if (hipDeviceSynchronize() != hipSuccess) return;
    if (hipMemcpy(v.data(), a.stamps, sizeof(long long) * v.size(), hipMemcpyDeviceToHost) != hipSuccess) return;
    long long t0 = v[0];
    for (int i = 0; i < nt; ++i) t0 = std::min(t0, v[(size_t)i * 4]);
    // CU key: XCC, SE, SH, CU (HW_ID bits 15:8)
    auto cu = [&](int i) { const long long hw = v[(size_t)i * 4 + 3]; return ((hw >> 32) & 0xf) << 8 | ((hw >> 8) & 0xff); };
    auto overlap = [&](int i, int j) { return v[(size_t)i * 4] < v[(size_t)j * 4 + 2] && v[(size_t)j * 4] < v[(size_t)i * 4 + 2]; };
    std::map<long long, int> scu, fcu;
    int ss = 0, sf = 0, ff = 0;
    for (int i = 0; i < nt; ++i) (i < n ? scu : fcu)[cu(i)]++;
    for (int i = 0; i < n; ++i) {
        bool s2 = false, f2 = false;
        for (int j = 0; j < nt; ++j)
            if (j != i && cu(j) == cu(i) && overlap(i, j)) (j < n ? s2 : f2) = true;
        ss += s2;
        sf += f2;
    }
    for (int i = n; i < nt; ++i)
        for (int j = n; j < nt; ++j)
            if (j != i && cu(j) == cu(i) && overlap(i, j)) { ++ff; break; }
    double pro = 0, loop = 0, st_max = 0, loop_max = 0, fs_max = 0, fe_max = 0, fdur = 0;
    for (int i = 0; i < n; ++i) {
        const long long* s = &v[(size_t)i * 4];
        pro += (s[1] - s[0]) * 0.01;
        loop += (s[2] - s[1]) * 0.01;
        st_max = std::max(st_max, (s[0] - t0) * 0.01);
        loop_max = std::max(loop_max, (s[2] - t0) * 0.01);
    }
    for (int i = n; i < nt; ++i) {
        const long long* s = &v[(size_t)i * 4];
        fs_max = std::max(fs_max, (s[0] - t0) * 0.01);
        fe_max = std::max(fe_max, (s[2] - t0) * 0.01);
        fdur += (s[2] - s[0]) * 0.01;
    }
    std::fprintf(stderr, "[state stamps call %ld] %d state workgroups (%d pieces x %d groups, %d tiles each) on %zu CUs; "
                 "%d overlapped another state workgroup on their CU, %d a transform workgroup; mean prologue %.2f us, "
                 "loop %.2f us; starts up to %.2f us, last loop end %.2f us | %d transform workgroups on %zu CUs, %d "
                 "beside another; mean %.2f us, starts up to %.2f us, last end %.2f us\n", call, n, a.nseg, a.G,
                 a.tps, scu.size(), ss, sf, pro / n, loop / n, st_max, loop_max, nfft, fcu.size(), ff,
                 nfft ? fdur / nfft : 0.0, fs_max, fe_max);
}
#endif

int fb_state_window(hz_fb* h, const double* x, long len, double* out, hipStream_t st) {
    StateArgs a;
    HZ_TRY(state_args(h, x, len, out, &a));
    hipLaunchKernelGGL(pick_state(h->order), dim3((unsigned)a.G, (unsigned)a.nseg), dim3(kThreads), 0, st, a);
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

int fb_state_chained(hz_fb* h, const double* x, long len, double* out, hz_state::StateArgs* a) {
    if (h->order > 2) {
        hz::set_error("fb_state_chained: order %d (at most 2 fit beside another kernel)", h->order);
        return HZ_E_INVALID;
    }
    HZ_TRY(state_args(h, x, len, out, a));
    a->deferred = a->nseg > 1 ? 1 : 0;
    return HZ_OK;
}

int fb_state_combine(hz_fb* h, const hz_state::StateArgs& a, hipStream_t st) {
    if (a.nseg <= 1) return HZ_OK;
    const unsigned grid = (unsigned)((h->N + 255) / 256);
    switch (h->order) {
    case 1: hipLaunchKernelGGL(fb_state_combine_kernel<1>, dim3(grid), dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL(fb_state_combine_kernel<2>, dim3(grid), dim3(256), 0, st, a); break;
    default:
        hz::set_error("fb_state_combine: order %d", h->order);
        return HZ_E_INVALID;
    }
    HZ_TRY_HIP(hipGetLastError());
    return HZ_OK;
}

}  // namespace hz_fbi
