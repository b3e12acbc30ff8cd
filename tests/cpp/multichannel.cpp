// tests/filterbanks.cpp:191-211's multi-channel loop over the C++ drop-in, with the one-line change
// INTEGRATION.md describes: the channels' operator() calls of a sample become one
// soundmath::sample_many call (one per-sample server request); tick() stays per channel.
// argv: <dir> -- reads coef.bin ([864] x {3 forward, 2 back}) and x.bin ([T][8]), writes y.bin
// ([T][8]) and lat.bin ([T] seconds per frame).
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "soundmath/filterbank.h"

constexpr int CHANELS = 8, N = 864;

static std::vector<double> slurp(const std::string& path) {
    std::vector<double> v;
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return v;
    double d;
    while (std::fread(&d, sizeof d, 1, f) == 1) v.push_back(d);
    std::fclose(f);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string dir = argv[1];
    const std::vector<double> coef = slurp(dir + "/coef.bin"), x = slurp(dir + "/x.bin");
    if (coef.size() != 5 * N || x.size() % CHANELS) return 3;
    const int T = (int)(x.size() / CHANELS);
    soundmath::FFilterbank<double, N, 2>* Fs[CHANELS];
    for (int j = 0; j < CHANELS; ++j) {
        Fs[j] = new soundmath::FFilterbank<double, N, 2>();
        for (int n = 0; n < N; ++n)
            Fs[j]->coefficients(n, {coef[5 * n], coef[5 * n + 1], coef[5 * n + 2]}, {coef[5 * n + 3], coef[5 * n + 4]});
        Fs[j]->boost(std::vector<double>(N, 1.0 + 0.1 * j));
        Fs[j]->open();
    }
    std::vector<double> y((size_t)T * CHANELS), lat(T);
    for (int i = 0; i < T; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        soundmath::sample_many(Fs, CHANELS, &x[(size_t)i * CHANELS], &y[(size_t)i * CHANELS], HZ_DIST_SOFTCLIP);
        for (int j = 0; j < CHANELS; ++j) Fs[j]->tick();
        lat[i] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    FILE* f = std::fopen((dir + "/y.bin").c_str(), "wb");
    std::fwrite(y.data(), sizeof(double), y.size(), f);
    std::fclose(f);
    f = std::fopen((dir + "/lat.bin").c_str(), "wb");
    std::fwrite(lat.data(), sizeof(double), lat.size(), f);
    std::fclose(f);
    for (int j = 0; j < CHANELS; ++j) delete Fs[j];
    std::printf("multichannel ok\n");
    return 0;
}
