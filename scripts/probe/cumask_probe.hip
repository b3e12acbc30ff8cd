// cumask_probe.hip -- where do the workgroups of a CU-masked stream land (XCC, SE, CU), and do two
// streams with complementary masks run side by side?  hipcc --offload-arch=gfx950 -O2 -o cumask_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

#define CK(x)                                                                                    \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) {                                                                  \
            std::printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));        \
            return 1;                                                                            \
        }                                                                                        \
    } while (0)

__global__ void where_kernel(unsigned* out, long long spin) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
        const long long t1 = __builtin_amdgcn_s_memrealtime();
        out[4 * blockIdx.x] = xcc;
        out[4 * blockIdx.x + 1] = hw;
        out[4 * blockIdx.x + 2] = (unsigned)t0;
        out[4 * blockIdx.x + 3] = (unsigned)t1;
    }
}

static void report(const char* name, const std::vector<unsigned>& h, int n) {
    std::set<std::tuple<int, int, int, int>> cus;
    std::set<int> xccs;
    int per_xcc[8] = {0};
    for (int i = 0; i < n; ++i) {
        const unsigned xcc = h[4 * i] & 0xf, hw = h[4 * i + 1];
        const int cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        if (cus.insert({(int)xcc, se, sh, cu}).second) per_xcc[xcc & 7]++;
        xccs.insert(xcc);
    }
    std::printf("%s: %d WGs on %zu CUs, %zu XCCs; CUs per XCC:", name, n, cus.size(), xccs.size());
    for (int x = 0; x < 8; ++x) std::printf(" %d", per_xcc[x]);
    std::printf("\n");
}

int main() {
    const int n = 1024;
    unsigned *dA, *dB, *dC;
    CK(hipMalloc(&dA, 16 * n));
    CK(hipMalloc(&dB, 16 * n));
    CK(hipMalloc(&dC, 16 * n));
    hipStream_t s0, sA, sB;
    CK(hipStreamCreate(&s0));
    std::vector<unsigned> m0(8, 0);
    CK(hipExtStreamGetCUMask(s0, 8, m0.data()));
    std::printf("default mask:");
    for (unsigned w : m0) std::printf(" %08x", w);
    std::printf("\n");
    std::vector<unsigned> mA(8, 0x00FF00FFu), mB(8, 0xFF00FF00u);
    CK(hipExtStreamCreateWithCUMask(&sA, 8, mA.data()));
    CK(hipExtStreamCreateWithCUMask(&sB, 8, mB.data()));
    std::vector<unsigned> g(8, 0);
    CK(hipExtStreamGetCUMask(sA, 8, g.data()));
    std::printf("mask A read back:");
    for (unsigned w : g) std::printf(" %08x", w);
    std::printf("\n");
    const long long spin = 100 * 20;   // memrealtime 100 MHz: 20 us
    hipLaunchKernelGGL(where_kernel, dim3(n), dim3(64), 0, s0, dC, spin);
    CK(hipStreamSynchronize(s0));
    hipLaunchKernelGGL(where_kernel, dim3(n), dim3(64), 0, sA, dA, spin);
    hipLaunchKernelGGL(where_kernel, dim3(n), dim3(64), 0, sB, dB, spin);
    CK(hipStreamSynchronize(sA));
    CK(hipStreamSynchronize(sB));
    std::vector<unsigned> hA(4 * n), hB(4 * n), hC(4 * n);
    CK(hipMemcpy(hA.data(), dA, 16 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hB.data(), dB, 16 * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hC.data(), dC, 16 * n, hipMemcpyDeviceToHost));
    report("default", hC, n);
    report("mask A", hA, n);
    report("mask B", hB, n);
    // overlap: A's and B's time ranges
    unsigned a0 = ~0u, a1 = 0, b0 = ~0u, b1 = 0;
    for (int i = 0; i < n; ++i) {
        a0 = std::min(a0, hA[4 * i + 2]), a1 = std::max(a1, hA[4 * i + 3]);
        b0 = std::min(b0, hB[4 * i + 2]), b1 = std::max(b1, hB[4 * i + 3]);
    }
    std::printf("A [%u, %u] B [%u, %u] (10 ns ticks, rel A start: B %d..%d, A ends %d)\n", a0, a1, b0, b1,
                (int)(b0 - a0), (int)(b1 - a0), (int)(a1 - a0));
    // disjointness
    std::set<std::tuple<int, int, int, int>> sa, sb;
    for (int i = 0; i < n; ++i) {
        unsigned hw = hA[4 * i + 1];
        sa.insert({(int)(hA[4 * i] & 0xf), (int)(hw >> 13) & 7, (int)(hw >> 12) & 1, (int)(hw >> 8) & 0xf});
        hw = hB[4 * i + 1];
        sb.insert({(int)(hB[4 * i] & 0xf), (int)(hw >> 13) & 7, (int)(hw >> 12) & 1, (int)(hw >> 8) & 0xf});
    }
    int common = 0;
    for (auto& c : sa) common += sb.count(c);
    std::printf("CUs in both A and B: %d\n", common);
    std::printf("cumask probe ok\n");
    return 0;
}
