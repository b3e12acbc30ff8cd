// Probe: where a workgroup of the stationary engine's forward transform (resp_fwd_kernel: one
// 4096-sample real window = 2048-point complex FFT + split, 256 threads) spends its time --
// s_memtime stamps after the global loads, the LDS store, each FFT pass and the split, for 258
// workgroups (the C2 call) and for 24 (the partition spectra).  Same code path as
// hz_fb_resp.hip's real_window_fwd, instrumented.
// Build: hipcc --offload-arch=gfx950 -O3 -I huygens_amd/csrc -o scripts/probe/fft_phase_probe scripts/probe/fft_phase_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "hz_fft.h"
#include "hz_fft2k.h"

constexpr int kLgH = 11, kH = 1 << kLgH, kP = kH, kThreads = 256, kPT = kH / kThreads;
constexpr int kSplit = (kH / 2 + kThreads) / kThreads;
constexpr int kStamps = 12;   // slots 9: hw id, 10 / 11: s_memrealtime at start / end

struct FftLds {
    double re[hz::padded_len(kH)], im[hz::padded_len(kH)];
    double2 T[hz::twc_len(kLgH)];
};

__device__ __forceinline__ long long stamp() {
    __builtin_amdgcn_sched_barrier(0);
    const long long t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

template <int MODE>   // 0: full; 1: loads + stores only (no FFT passes, no split math)
__global__ __launch_bounds__(kThreads) void fwd_probe(const double* __restrict__ u, const double2* __restrict__ tw,
                                                     double2* __restrict__ Z, double* __restrict__ Zn,
                                                     long long* __restrict__ st) {
    __shared__ FftLds s;
    long long ts[kStamps];
    int ns = 0;
    ts[ns++] = stamp();
    const int t = threadIdx.x;
    const long m0 = (long)blockIdx.x * kP;
    double vr[kPT], vi[kPT];
#pragma unroll
    for (int i = 0; i < kPT; ++i) {
        const int n = t + i * kThreads;
        vr[i] = u[m0 + 2 * n];
        vi[i] = u[m0 + 2 * n + 1];
    }
    double2 w[kSplit];
#pragma unroll
    for (int i = 0; i < kSplit; ++i) {
        const int k = t + i * kThreads;
        w[i] = k <= kH / 2 ? tw[k] : make_double2(1.0, 0.0);
    }
    for (int k = t; k < hz::twc_len(kLgH); k += kThreads) s.T[k] = tw[2 * k];
#pragma unroll
    for (int i = 0; i < kPT; ++i) {
        const int e = hz::pad16(t + i * kThreads);
        s.re[e] = vr[i];
        s.im[e] = vi[i];
    }
    ts[ns++] = stamp();   // 1: loads landed (the stores needed them)
    __syncthreads();
    ts[ns++] = stamp();   // 2: barrier
    if constexpr (MODE == 0) {
        // fft_fwd_lead<3>(lg 11): a radix-4 pass, then three radix-8 passes, stamped
        hz::fft_pass_r<3, false>(2, s.re, s.im, kLgH, kLgH - 1, s.T);
        __syncthreads();
        ts[ns++] = stamp();
        int lh = kLgH - 1 - 2;
        for (int p = 0; p < 3; ++p, lh -= 3) {
            hz::fft_pass_r<3, false>(3, s.re, s.im, kLgH, lh, s.T);
            __syncthreads();
            ts[ns++] = stamp();
        }
    }
    double2* zrow = Z + (long)blockIdx.x * kH;
#pragma unroll
    for (int i = 0; i < kSplit; ++i) {
        const int k = t + i * kThreads;
        if (k > kH / 2) break;
        if (k == 0) {
            zrow[0] = make_double2(s.re[0] + s.im[0], 0.0);
            Zn[blockIdx.x] = s.re[0] - s.im[0];
            continue;
        }
        const int pa = hz::pad16(hz::bitrev(k, kLgH)), pb = hz::pad16(hz::bitrev(kH - k, kLgH));
        const double ar = s.re[pa], ai = s.im[pa], br = s.re[pb], bi = s.im[pb];
        const double er = 0.5 * (ar + br), ei = 0.5 * (ai - bi);
        const double orr = 0.5 * (ai + bi), oi = -0.5 * (ar - br);
        const double wr = w[i].x * orr - w[i].y * oi, wi = w[i].x * oi + w[i].y * orr;
        zrow[k] = make_double2(er + wr, ei + wi);
        if (k != kH / 2) zrow[kH - k] = make_double2(er - wr, wi - ei);
    }
    ts[ns++] = stamp();   // split issued
    __builtin_amdgcn_s_waitcnt(0);   // stores acknowledged
    ts[ns++] = stamp();
    if (t == 0)
        for (int i = 0; i < kStamps; ++i) st[(long)blockIdx.x * kStamps + i] = i < ns ? ts[i] : 0;
}

// the shipped forward path (hz_fft2k.h + the split of hz_fb_resp.hip's real_window_fwd), stamped:
// 0 start, 1 loads landed + P1 (registers) + LDS store, 2 barrier, 3-5 LDS passes, 6 split issued,
// 7 stores acknowledged
__global__ __launch_bounds__(kThreads) void fwd2k_probe(const double* __restrict__ u, const double2* __restrict__ tw,
                                                       double2* __restrict__ Z, double* __restrict__ Zn,
                                                       long long* __restrict__ st) {
    __shared__ hz2k::Lds s;
    long long ts[kStamps];
    const long long rt0 = __builtin_amdgcn_s_memrealtime();
    int ns = 0;
    ts[ns++] = stamp();
    const int t = threadIdx.x;
    const long m0 = (long)blockIdx.x * kP;
    double vr[kPT], vi[kPT];
#pragma unroll
    for (int i = 0; i < kPT; ++i) {
        const int n = t + i * kThreads;
        vr[i] = u[m0 + 2 * n];
        vi[i] = u[m0 + 2 * n + 1];
    }
    hz2k::FwdTw ft;
    ft.load(tw);
    double2 w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = tw[t + i * kThreads];
    // hz2k::fwd, stamped
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        double xr[4], xi[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            xr[j] = vr[g + 2 * j];
            xi[j] = vi[g + 2 * j];
        }
        hz2k::Dif<2, 10>::regs(xr, xi, ft.p1[g]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            vr[g + 2 * j] = xr[j];
            vi[g + 2 * j] = xi[j];
        }
    }
#pragma unroll
    for (int i = 0; i < kPT; ++i) {
        const int e = hz::pad16(t + kThreads * i);
        s.re[e] = vr[i];
        s.im[e] = vi[i];
    }
    ts[ns++] = stamp();
    __syncthreads();
    ts[ns++] = stamp();
    hz2k::Dif<3, 8>::lds(s, t, ft.p2);
    __syncthreads();
    ts[ns++] = stamp();
    hz2k::Dif<3, 5>::lds(s, t, ft.p3);
    __syncthreads();
    ts[ns++] = stamp();
    const double2 one[3] = {make_double2(1.0, 0.0), make_double2(1.0, 0.0), make_double2(1.0, 0.0)};
    hz2k::Dif<3, 2>::lds(s, t, one);
    __syncthreads();
    ts[ns++] = stamp();
    double2* zrow = Z + (long)blockIdx.x * kH;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int k = t + i * kThreads, kb = (kH - k) & (kH - 1);
        const int pa = hz::pad16(hz::bitrev(k, kLgH)), pb = hz::pad16(hz::bitrev(kb, kLgH));
        const double ar = s.re[pa], ai = s.im[pa], br = s.re[pb], bi = s.im[pb];
        const double er = 0.5 * (ar + br), ei = 0.5 * (ai - bi);
        const double orr = 0.5 * (ai + bi), oi = -0.5 * (ar - br);
        const double wr = w[i].x * orr - w[i].y * oi, wi = w[i].x * oi + w[i].y * orr;
        zrow[k] = make_double2(er + wr, ei + wi);
        if (k) zrow[kb] = make_double2(er - wr, wi - ei);
        else Zn[blockIdx.x] = er - wr;
    }
    ts[ns++] = stamp();
    __builtin_amdgcn_s_waitcnt(0);
    ts[ns++] = stamp();
    // where the workgroup ran: HW_ID (cu [11:8], sh [12], se [15:13]) and XCC_ID
    const unsigned hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
    if (t == 0) {
        for (int i = 0; i < kStamps; ++i) st[(long)blockIdx.x * kStamps + i] = i < ns ? ts[i] : 0;
        st[(long)blockIdx.x * kStamps + 9] = ((long long)(xcc & 0xf) << 32) | hwid;
        st[(long)blockIdx.x * kStamps + 10] = rt0;
        st[(long)blockIdx.x * kStamps + 11] = __builtin_amdgcn_s_memrealtime();
    }
}

int main() {
    const int maxw = 258;
    const long nu = (long)(maxw + 1) * kP;
    double* u;
    double2 *tw, *Z;
    double* Zn;
    long long* st;
    hipMalloc(&u, nu * sizeof(double));
    hipMalloc(&tw, kH * sizeof(double2));
    hipMalloc(&Z, (long)maxw * kH * sizeof(double2));
    hipMalloc(&Zn, maxw * sizeof(double));
    hipMalloc(&st, (long)maxw * kStamps * sizeof(long long));
    std::vector<double> hu(nu);
    for (long i = 0; i < nu; ++i) hu[i] = std::sin(0.001 * i);
    hipMemcpy(u, hu.data(), nu * sizeof(double), hipMemcpyHostToDevice);
    std::vector<double2> htw(kH);
    for (int k = 0; k < kH; ++k) htw[k] = make_double2(std::cos(-2 * M_PI * k / (2 * kH)), std::sin(-2 * M_PI * k / (2 * kH)));
    hipMemcpy(tw, htw.data(), kH * sizeof(double2), hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // mode 3: mode 2 with 90 KB of unused dynamic LDS per workgroup, so at most one fits a CU
    hipFuncSetAttribute((const void*)fwd2k_probe, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    for (int mode = 0; mode < 4; ++mode)
        for (int wg : {24, 258}) {
            auto k = mode == 0 ? fwd_probe<0> : mode == 1 ? fwd_probe<1> : fwd2k_probe;
            const size_t dyn = mode == 3 ? 90 * 1024 : 0;
            for (int rep = 0; rep < 200; ++rep) hipLaunchKernelGGL(k, dim3(wg), dim3(kThreads), dyn, 0, u, tw, Z, Zn, st);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k, dim3(wg), dim3(kThreads), dyn, 0, u, tw, Z, Zn, st);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            std::vector<long long> hs((long)wg * kStamps);
            hipMemcpy(hs.data(), st, hs.size() * sizeof(long long), hipMemcpyDeviceToHost);
            const int nst = mode == 0 ? 9 : mode == 1 ? 5 : 8;   // modes 2, 3: the hz_fft2k path
            std::vector<double> avg(nst, 0.0);
            long long first = hs[0], lastend = 0;
            for (int b = 0; b < wg; ++b) {
                for (int i = 1; i < nst; ++i) avg[i] += (double)(hs[b * kStamps + i] - hs[b * kStamps + i - 1]) / wg;
                first = std::min(first, hs[b * kStamps]);
                lastend = std::max(lastend, hs[b * kStamps + nst - 1]);
            }
            std::printf("mode %d (%s), %3d workgroups: event %.2f us; span first start -> last end %.0f ticks; "
                        "per-WG phase ticks (s_memtime):", mode, mode == 3 ? "hz_fft2k, 1/CU" : mode == 2 ? "hz_fft2k" : mode ? "no FFT" : "full", wg, 1e3 * ms,
                        (double)(lastend - first));
            for (int i = 1; i < nst; ++i) std::printf(" %.0f", avg[i]);
            std::printf("\n");
            if (mode >= 2) {   // workgroups per CU (XCC, SE, SH, CU)
                std::vector<int> cnt(8 * 8 * 2 * 16, 0);
                for (int b = 0; b < wg; ++b) {
                    const long long v = hs[b * kStamps + 9];
                    const unsigned hw = (unsigned)v, xc = (unsigned)(v >> 32);
                    const int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
                    ++cnt[((xc * 8 + se) * 2 + sh) * 16 + cu];
                }
                int used = 0, mx = 0;
                for (int c : cnt) {
                    used += c > 0;
                    mx = std::max(mx, c);
                }
                long long r0 = hs[10], r1 = 0, rmax = 0;
                double rsum = 0;
                for (int b = 0; b < wg; ++b) {
                    r0 = std::min(r0, hs[b * kStamps + 10]);
                    r1 = std::max(r1, hs[b * kStamps + 11]);
                }
                for (int b = 0; b < wg; ++b) {
                    rmax = std::max(rmax, hs[b * kStamps + 10] - r0);
                    rsum += hs[b * kStamps + 11] - hs[b * kStamps + 10];
                }
                std::printf("    %d workgroups on %d distinct CUs, at most %d per CU; real time: first start -> last end "
                            "%.2f us, last start %.2f us after the first, mean workgroup life %.2f us\n",
                            wg, used, mx, 0.01 * (r1 - r0), 0.01 * rmax, 0.01 * rsum / wg);
            }
        }
    return 0;
}
