// Setter churn from a C++ caller (the reference's language): the C2 bank streamed in 1024-sample
// calls on device buffers, mix() on 9 bands every 4800 samples (tests/filterbank.cpp:217-252 retunes
// the courses of a note from its MIDI thread), against the same calls without setters.
// argv: <dir> -- reads coef.bin ([N] x {3 forward, 2 back}), x.bin ([n] input); prints one JSON line.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdio>
#include <string>
#include <vector>

#include "huygens_hip.h"

static std::vector<double> slurp(const std::string& path) {
    std::vector<double> v;
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return v;
    double d;
    while (std::fread(&d, sizeof d, 1, f) == 1) v.push_back(d);
    std::fclose(f);
    return v;
}

#define CHECK(e)                                                                     \
    do {                                                                             \
        int rc_ = (e);                                                               \
        if (rc_) {                                                                   \
            std::fprintf(stderr, "%s: %d %s\n", #e, rc_, hz_last_error());           \
            return 1;                                                                \
        }                                                                            \
    } while (0)

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    const std::vector<double> coef = slurp(dir + "/coef.bin"), x = slurp(dir + "/x.bin");
    const int N = (int)(coef.size() / 5);
    const long n = (long)x.size(), B = 1024, nb = n / B;
    hz_fb* h = nullptr;
    CHECK(hz_fb_create(2, N, 0.1, 1.0, 0, &h));
    for (int b = 0; b < N; ++b) CHECK(hz_fb_coefficients(h, b, &coef[5 * b], 3, &coef[5 * b + 3], 2));
    std::vector<double> ones(N, 1.0);
    CHECK(hz_fb_boost_all(h, ones.data(), N));
    CHECK(hz_fb_open(h));
    double *dx = nullptr, *dy = nullptr;
    if (hipMalloc((void**)&dx, sizeof(double) * n) || hipMalloc((void**)&dy, sizeof(double) * n)) return 3;
    if (hipMemcpy(dx, x.data(), sizeof(double) * n, hipMemcpyHostToDevice)) return 3;
    for (int i = 0; i < 3; ++i) CHECK(hz_fb_process_device(h, dx, dy, n));   // converge, fill the history
    // (diagnostic) HZ_CHURN_SPAN: the setters' bands drawn from [0, span) instead of all N
    const int span = std::getenv("HZ_CHURN_SPAN") ? std::max(9, std::min(N, std::atoi(std::getenv("HZ_CHURN_SPAN")))) : N;
    unsigned long long lcg = 12345;
    auto rnd = [&]() { lcg = lcg * 6364136223846793005ULL + 1442695040888963407ULL; return (unsigned)(lcg >> 33); };
    double us[2] = {0, 0};
    double t_mix = 0, t_setblk = 0, t_blk = 0;   // host seconds: mix() calls, calls after a setter, other calls
    long setters = 0;
    int path = 0;
    long streamed_churn = 0;
    for (int pass = 0; pass < 2; ++pass) {   // 0: converged, 1: churn
        for (long i = 0; i < 64; ++i) CHECK(hz_fb_process_device(h, dx + B * (i % nb), dy + B * (i % nb), B));
        CHECK(hz_fb_synchronize(h));
        const auto t0 = std::chrono::steady_clock::now();
        for (long i = 0; i < nb; ++i) {
            bool set = false;
            auto c0 = std::chrono::steady_clock::now();
            if (pass == 1 && (i * B) / 4800 != ((i - 1) * B) / 4800) {
                for (int j = 0; j < 9; ++j) CHECK(hz_fb_mix(h, (int)(rnd() % span), 0.5 + (rnd() % 1000) / 1000.0));
                ++setters;
                set = true;
            }
            auto c1 = std::chrono::steady_clock::now();
            CHECK(hz_fb_process_device(h, dx + B * i, dy + B * i, B));
            auto c2 = std::chrono::steady_clock::now();
            if (pass == 1) {
                t_mix += std::chrono::duration<double>(c1 - c0).count();
                (set ? t_setblk : t_blk) += std::chrono::duration<double>(c2 - c1).count();
            }
            if (pass == 1) {
                CHECK(hz_fb_last_path(h, &path));
                streamed_churn += path == HZ_FB_PATH_STREAM;
            }
        }
        CHECK(hz_fb_synchronize(h));
        us[pass] = 1e6 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / nb;
    }
    std::printf("{\"converged_us_per_block\": %.4f, \"churn_us_per_block\": %.4f, \"ratio\": %.4f, \"setters\": %ld, "
                "\"blocks\": %ld, \"blocks_streamed\": %ld, \"host_us_per_setter_mix_calls\": %.3f, "
                "\"host_us_per_call_after_setter\": %.3f, \"host_us_per_other_call\": %.3f}\n", us[0], us[1], us[1] / us[0],
                setters, nb, streamed_churn, 1e6 * t_mix / std::max(1L, setters), 1e6 * t_setblk / std::max(1L, setters),
                1e6 * t_blk / std::max(1L, nb - setters));
    hz_fb_destroy(h);
    return 0;
}
