// Probe: the 1024-sample streaming rate of the C2 bank from a C++ caller of the C ABI (no Python
// between calls), to separate the Python caller's per-call cost from the GPU's.
//   python3 scripts/probe/stream_cpp_coef.py coef.bin && ./stream_cpp coef.bin
// coef.bin: 4096 x (3 fwd + 2 back) doubles (the bench's resonant_coefficients(4096, 0.999, 1.0)).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "huygens_hip.h"

#define CK(x)                                                                      \
    do {                                                                           \
        int rc_ = (x);                                                             \
        if (rc_ != 0) {                                                            \
            std::fprintf(stderr, "%s -> %d (%s)\n", #x, rc_, hz_last_error());     \
            return 1;                                                              \
        }                                                                          \
    } while (0)

int main(int argc, char** argv) {
    const int N = 4096, B = 1024;
    std::vector<double> coef((size_t)N * 5);
    FILE* f = std::fopen(argc > 1 ? argv[1] : "coef.bin", "rb");
    if (!f || std::fread(coef.data(), sizeof(double), coef.size(), f) != coef.size()) {
        std::fprintf(stderr, "coefficients file\n");
        return 1;
    }
    std::fclose(f);
    hz_fb* h = nullptr;
    CK(hz_fb_create(2, N, 0.1, 1.0, 0, &h));
    for (int n = 0; n < N; ++n) CK(hz_fb_coefficients(h, n, &coef[(size_t)n * 5], 3, &coef[(size_t)n * 5 + 3], 2));
    std::vector<double> ones(N, 1.0);
    CK(hz_fb_boost_all(h, ones.data(), N));
    CK(hz_fb_open(h));
    const long S = 480000;
    std::vector<double> xh(S);
    srand(1234);
    for (long i = 0; i < S; ++i) xh[i] = 2.0 * rand() / RAND_MAX - 1.0;
    double *x = nullptr, *y = nullptr;
    if (hipMalloc(&x, sizeof(double) * S) != hipSuccess || hipMalloc(&y, sizeof(double) * S) != hipSuccess) return 1;
    if (hipMemcpy(x, xh.data(), sizeof(double) * S, hipMemcpyHostToDevice) != hipSuccess) return 1;
    // converge the smoothers (k_g = 1 s), as the bench's priming calls do
    for (int i = 0; i < 3; ++i) CK(hz_fb_process_device(h, x, y, S));
    const int nb = S / B;
    for (int i = 0; i < 8; ++i) CK(hz_fb_process_device(h, x + (long)B * i, y + (long)B * i, B));
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    for (int rep = 0; rep < 3; ++rep) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < nb; ++i) CK(hz_fb_process_device(h, x + (long)B * i, y + (long)B * i, B));
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        int path = -1;
        CK(hz_fb_last_path(h, &path));
        std::printf("C++ caller: %d blocks of %d samples, %.2f us per block, %.3e band-samples/s (path %d)\n", nb, B,
                    1e6 * s / nb, (double)N * B * nb / s, path);
    }
    CK(hz_fb_destroy(h));
    return 0;
}
