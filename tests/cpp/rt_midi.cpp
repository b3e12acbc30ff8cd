// rt_midi.cpp -- the reference's filterbank demo shape (tests/filterbank.cpp:194-252): the audio
// thread runs `out = F(in); F.tick();` per sample on Filterbank<double>(2, N) while a MIDI thread
// calls boost() / mix() concurrently (the reference does that without synchronisation; the drop-in
// holds the handle's lock).  Writes, into argv[1]: the inputs and outputs, the per-sample latency
// (ns), and the setter log {served-at-call, kind (0 boost, 1 mix), band, value}; the setter applies
// from sample `served-at-call` on (hz_fb_setter_seq).  tests/test_rt_server_gpu.py replays the log
// through the C restatement.  argv[2] = bands, argv[3] = samples, argv[4] = setter period (us).
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "soundmath/filterbank.h"

using namespace soundmath;

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: rt_midi DIR BANDS SAMPLES SETTER_US\n");
        return 2;
    }
    const std::string dir = argv[1];
    const int N = std::atoi(argv[2]);
    const int S = std::atoi(argv[3]);
    const int period_us = std::atoi(argv[4]);
    Filterbank<double> F(2, N, 0.1, 1.0);
    // tests/resynthesis.cpp:48-54 recipe, R = 0.999
    const double R = 0.999;
    std::vector<double> coef(5 * (size_t)N);   // dumped: the replay uses the same values
    for (int i = 0; i < N; ++i) {
        const double f = 0.5 * (i + 1) * SR / N, th = 2 * PI * f / SR;
        const double b1 = -2 * R * std::cos(th), b2 = R * R;
        // |H(e^{j th})| of {1, 0, -1} / (1 + b1 z^-1 + b2 z^-2)
        const double cr = 1 - std::cos(2 * th), ci = std::sin(2 * th);
        const double dr = 1 + b1 * std::cos(th) + b2 * std::cos(2 * th), di = -b1 * std::sin(th) - b2 * std::sin(2 * th);
        double g = std::sqrt((cr * cr + ci * ci) / (dr * dr + di * di));
        if (!(g > 0) || !std::isfinite(g)) g = 1;
        F.coefficients(i, {1 / g, 0, -1 / g}, {b1, b2});
        const double c5[5] = {1 / g, 0, -1 / g, b1, b2};
        for (int k = 0; k < 5; ++k) coef[5 * (size_t)i + k] = c5[k];
    }
    F.boost(std::vector<double>(N, 1.0));
    F.open();
    std::vector<double> in(S), out(S);
    std::vector<long long> lat(S);
    for (int t = 0; t < S; ++t) in[t] = std::sin(0.013 * t) * 0.5 + 0.5 * (((t * 7919) % 13) - 6) / 6.0;
    std::atomic<bool> done{false};
    std::vector<double> log;   // {seq, kind, band, value}
    std::thread midi([&] {
        unsigned s = 12345;
        auto rnd = [&] {
            s = s * 1103515245u + 12345u;
            return (s >> 8) & 0xffffff;
        };
        while (!done.load()) {
            std::this_thread::sleep_for(std::chrono::microseconds(period_us));
            const int kind = rnd() & 1, band = rnd() % N;
            const double v = 0.25 + (rnd() % 1000) / 500.0;
            if (kind == 0) F.boost(band, v);
            else F.mix(band, v);
            long long seq = 0;
            hz_fb_setter_seq(F.native(), &seq);
            log.insert(log.end(), {(double)seq, (double)kind, (double)band, v});
        }
    });
    for (int t = 0; t < S; ++t) {
        const auto t0 = std::chrono::steady_clock::now();
        out[t] = F(in[t]);
        F.tick();
        lat[t] = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    }
    done = true;
    midi.join();
    auto dump = [&](const char* name, const void* p, size_t bytes) {
        FILE* f = std::fopen((dir + "/" + name).c_str(), "wb");
        std::fwrite(p, 1, bytes, f);
        std::fclose(f);
    };
    dump("coef.bin", coef.data(), sizeof(double) * coef.size());
    dump("in.bin", in.data(), sizeof(double) * S);
    dump("out.bin", out.data(), sizeof(double) * S);
    dump("lat.bin", lat.data(), sizeof(long long) * S);
    dump("log.bin", log.data(), sizeof(double) * log.size());
    std::printf("rt_midi ok: %d samples, %zu setters\n", S, log.size() / 4);
    return 0;
}
