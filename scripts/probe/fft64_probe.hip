// probe: lane-exchange primitives and the 64-point transforms of hz_fb_col.h against direct sums
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../../huygens_amd/csrc/hz_fb_col.h"

using namespace hz_col;

__global__ void xor_kernel(double* out) {
    const int l = threadIdx.x;
    const double v = 1000.0 + l;
    out[0 * 64 + l] = xor_d<1>(v, l);
    out[1 * 64 + l] = xor_d<2>(v, l);
    out[2 * 64 + l] = xor_d<4>(v, l);
    out[3 * 64 + l] = xor_d<8>(v, l);
    out[4 * 64 + l] = xor_d<16>(v, l);
    out[5 * 64 + l] = xor_d<32>(v, l);
}

__global__ void fft_kernel(const double2* tw, const double2* in, double2* fo, double2* io) {
    const int l = threadIdx.x;
    Fft64 f;
    f.init(tw, l);
    double2 v[2] = {in[l], in[64 + l]};
    f.fwd(v, l);
    fo[l] = v[0];
    fo[64 + l] = v[1];
    double2 y[1] = {in[l]};
    f.inv(y, l);
    io[l] = y[0];
}

int main() {
    double* d;
    hipMalloc(&d, 6 * 64 * sizeof(double));
    hipLaunchKernelGGL(xor_kernel, dim3(1), dim3(64), 0, 0, d);
    std::vector<double> h(6 * 64);
    hipMemcpy(h.data(), d, h.size() * sizeof(double), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int k = 0; k < 6; ++k)
        for (int l = 0; l < 64; ++l)
            if (h[k * 64 + l] != 1000.0 + (l ^ (1 << k))) {
                if (bad < 20) printf("xor %d lane %d: got %g want %d\n", 1 << k, l, h[k * 64 + l] - 1000.0, l ^ (1 << k));
                ++bad;
            }
    printf("xor mismatches: %d\n", bad);
    std::vector<double2> tw(4096), in(128);
    for (int k = 0; k < 4096; ++k) {
        const long double a = -2.0L * acosl(-1.0L) * k / 4096;
        tw[k] = make_double2((double)cosl(a), (double)sinl(a));
    }
    for (int i = 0; i < 128; ++i) in[i] = make_double2(sin(0.37 * i + 0.1), cos(1.3 * i * i));
    double2 *dtw, *din, *dfo, *dio;
    hipMalloc(&dtw, 4096 * 16);
    hipMalloc(&din, 128 * 16);
    hipMalloc(&dfo, 128 * 16);
    hipMalloc(&dio, 64 * 16);
    hipMemcpy(dtw, tw.data(), 4096 * 16, hipMemcpyHostToDevice);
    hipMemcpy(din, in.data(), 128 * 16, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(fft_kernel, dim3(1), dim3(64), 0, 0, dtw, din, dfo, dio);
    std::vector<double2> fo(128), io(64);
    hipMemcpy(fo.data(), dfo, 128 * 16, hipMemcpyDeviceToHost);
    hipMemcpy(io.data(), dio, 64 * 16, hipMemcpyDeviceToHost);
    double ef = 0, ei = 0;
    for (int g = 0; g < 2; ++g)
        for (int l = 0; l < 64; ++l) {
            const int k = (int)(__builtin_bitreverse32((unsigned)l) >> 26);
            long double sr = 0, si = 0;
            for (int n = 0; n < 64; ++n) {
                const long double a = -2.0L * acosl(-1.0L) * ((n * k) % 64) / 64;
                sr += in[64 * g + n].x * cosl(a) - in[64 * g + n].y * sinl(a);
                si += in[64 * g + n].x * sinl(a) + in[64 * g + n].y * cosl(a);
            }
            ef = fmax(ef, fabs((double)sr - fo[64 * g + l].x) + fabs((double)si - fo[64 * g + l].y));
        }
    for (int n = 0; n < 64; ++n) {   // inverse: lane l holds Y[brev6(l)] = in[l]
        long double sr = 0, si = 0;
        for (int l = 0; l < 64; ++l) {
            const int k = (int)(__builtin_bitreverse32((unsigned)l) >> 26);
            const long double a = 2.0L * acosl(-1.0L) * ((n * k) % 64) / 64;
            sr += in[l].x * cosl(a) - in[l].y * sinl(a);
            si += in[l].x * sinl(a) + in[l].y * cosl(a);
        }
        ei = fmax(ei, fabs((double)sr - io[n].x) + fabs((double)si - io[n].y));
    }
    printf("fft64 fwd max err %.3e, inv max err %.3e\n", ef, ei);
    return bad || ef > 1e-12 || ei > 1e-12;
}
