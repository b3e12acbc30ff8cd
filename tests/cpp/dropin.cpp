// dropin.cpp -- the drop-in headers used as the reference's demos use src/*.h
// (tests/resynthesis.cpp, tests/delay.cpp, tests/bowl.cpp, tests/spectral.cpp,
// tests/fft.cpp).  Writes raw little-endian outputs into argv[1]; tests/test_cpp_gpu.py
// replays the same scenarios through the oracle.  Build: tests/test_cpp_cpu.py.
#include <chrono>
#include <cstdio>
#include <string>
#include <vector>

#include "soundmath/additive.h"
#include "soundmath/audio.h"
#include "soundmath/bowl.h"
#include "soundmath/delay.h"
#include "soundmath/filterbank.h"
#include "soundmath/fourier.h"
#include "soundmath/granulator.h"
#include "soundmath/harmbank.h"
#include "soundmath/oscbank.h"
#include "soundmath/sinusoids.h"
#include "soundmath/synth.h"

using namespace soundmath;

static std::string dir;

template <typename T>
static void dump(const char* name, const std::vector<T>& v) {
    FILE* f = std::fopen((dir + "/" + name + ".bin").c_str(), "wb");
    std::fwrite(v.data(), sizeof(T), v.size(), f);
    std::fclose(f);
}

static double input(int t) { return std::sin(0.01 * t) + 0.5 * (((t * 7919) % 13) - 6) / 6.0; }

static int hilbert64(const std::complex<double>* in, std::complex<double>* out) {
    for (int i = 0; i < 64; i++) out[i] = i < 32 ? in[i] : 0.0;
    return 0;
}

// tests/harmbank.cpp's process() callback shape: BSIZE frames of mono float in, float out
#define BSIZE 32
static Heterodyne<96>* g_het = nullptr;
static int het_process(const float* in, float* out) {
    g_het->process(in, out, BSIZE);
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    dir = argv[1];

    {   // Filterbank: per-sample operator()/tick, then process()
        Filterbank<double> fb(2, 16);
        for (int i = 0; i < 16; i++) {
            const double g = 0.01 * (i + 1), R = 0.99, th = 2 * PI * (i + 1) / 40.0;
            fb.coefficients(i, {g, 0, -g}, {-2 * R * std::cos(th), R * R});
        }
        fb.boost(std::vector<double>(16, 1.0));
        fb.open();
        std::vector<double> y(1000), x(1000);
        for (int t = 0; t < 1000; t++) x[t] = input(t);
        for (int t = 0; t < 100; t++) {
            y[t] = fb(x[t]);
            (void)fb(x[t]);   // cached until tick()
            fb.tick();
            if (t == 40 || t == 41) fb.tick();   // tick() without operator(): the stale ring row
        }
        fb.process(x.data() + 100, y.data() + 100, 600);   // block, then per sample again, then block
        for (int t = 700; t < 800; t++) {
            y[t] = fb(x[t]);
            fb.tick();
        }
        fb.process(x.data() + 800, y.data() + 800, 200);
        dump("filterbank", y);

        // the per-sample rate of a 4096-band bank (C2's size): operator() + tick() per sample,
        // the reference's execution model (tests/resynthesis.cpp:35-39)
        Filterbank<double> big(2, 4096);
        for (int i = 0; i < 4096; i++) {
            const double g = 0.001, R = 0.999, th = PI * (i + 0.5) / 4096.0;
            big.coefficients(i, {g, 0, -g}, {-2 * R * std::cos(th), R * R});
        }
        big.boost(std::vector<double>(4096, 1.0));
        big.open();
        double acc = 0;
        for (int t = 0; t < 500; t++) {
            acc += big(input(t));
            big.tick();
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 500; t < 20500; t++) {
            acc += big(input(t));
            big.tick();
        }
        const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        std::printf("per-sample Filterbank<double>(2, 4096): %.0f samples/s (%.2f us per operator()+tick(), sum %g)\n",
                    20000 / dt, 1e6 * dt / 20000, acc);

        // FFilterbank<double, 16, 2> (tests/filterbank.cpp:184,194 pattern), block form only
        FFilterbank<double, 16, 2> ff;
        for (int i = 0; i < 16; i++) {
            const double g = 0.01 * (i + 1), R = 0.99, th = 2 * PI * (i + 1) / 40.0;
            ff.coefficients(i, {g, 0, -g}, {-2 * R * std::cos(th), R * R});
        }
        ff.boost(std::vector<double>(16, 1.0));
        ff.open();
        std::vector<double> z(1000);
        ff.process(x.data(), z.data(), 1000);
        dump("ffilterbank", z);

        // Subtractive ALLINONE pattern (src/subtractive.h:215-228): every band retuned every
        // sample, here as one process_resonant() call over per-sample frequency rows
        Filterbank<double> sub(2, 16);
        sub.boost(std::vector<double>(16, 1.0));
        sub.open();
        std::vector<double> fr(1000 * 16), w(1000);
        for (int t = 0; t < 1000; t++)
            for (int b = 0; b < 16; b++) fr[t * 16 + b] = 110.0 * (b + 1) * (1 + 0.02 * std::sin(0.003 * t + b));
        sub.process_resonant(x.data(), w.data(), 1000, fr.data(), 0.999);
        dump("subtractive", w);
    }
    {   // Delay: tests/delay.cpp:18,41
        Delay<double> delay(10, 2 * SR);
        delay.coefficients({{0, 1}}, {{20000, 0.5}, {10000, 0.5}});
        std::vector<double> x(50000, 0.0), y(50000);
        x[0] = 1.0;
        for (int t = 0; t < 10; t++) {
            y[t] = delay(x[t]);
            delay.tick();
        }
        delay.tick();   // tick() without operator() (delay.h:92-97): the rings advance, nothing written
        delay.tick();
        delay.process(x.data() + 10, y.data() + 10, 49990);
        dump("delay", y);
    }
    {   // Bowl<float>: tests/bowl.cpp pattern with fill(float*, BSIZE)
        std::vector<float> f, a, d;
        for (int i = 0; i < 8; i++) {
            f.push_back(100.0f * (i + 1) * 1.01f);
            a.push_back(0.01f * (i + 1));
            d.push_back(0.5f * (i + 1));
        }
        Bowl<float> bowl(8, f, a, d);
        bowl.trigger();
        std::vector<float> y(2048);
        for (int b = 0; b < 2; b++) bowl.fill(y.data() + 1024 * b, 1024);
        dump("bowl", y);
    }
    {   // Fourier with a host processor (pointer of the reference's type), StaticSTFT
        // per sample, tests/spectral.cpp:90-108's loop, with a stretch of two writes per read
        // (the heads run apart) and one of reads alone (they catch up) -- the reference's own
        // state machine
        Fourier F(hilbert64, 64, 4);
        std::vector<double> yr, yi, x(1000);
        for (int t = 0; t < 1000; t++) x[t] = input(t);
        int w = 0;
        for (int t = 0; t < 900; t++) {
            F.write(x[w++]);
            if (t >= 300 && t < 340) F.write(x[w++]);
            if (t >= 500 && t < 540) continue;   // no read: writes only
            double r, i;
            F.read(&r, &i);
            yr.push_back(r);
            yi.push_back(i);
            if (t >= 600 && t < 640) {   // reads alone
                F.read(&r, &i);
                yr.push_back(r);
                yi.push_back(i);
            }
        }
        dump("fourier_re", yr);
        dump("fourier_im", yi);
        StaticSTFT S(64, 4);
        std::vector<double> sr(1000), si(1000);
        S.process_block(x.data(), nullptr, sr.data(), si.data(), 1000);
        dump("static_re", sr);
    }
    {   // Synth<double> / Oscillator<double>: tests/eigen.cpp:23, tests/fm.cpp:18 (host, as the reference)
        Synth<double> s(&cycle, 220.0);
        Oscillator<double> mod(3.0, 0.25, 0.01);
        std::vector<double> y;
        for (int t = 0; t < 3000; t++) {
            if (t == 1000) s.freqmod(330.0);
            if (t == 2000) s.phasemod(0.5);
            y.push_back(s());
            y.push_back(mod());
            s.tick();
            mod.tick();
        }
        Synth<double> saw_synth(&saw, 100.0, 0.1);
        for (int t = 0; t < 500; t++) {
            y.push_back(saw_synth());
            saw_synth.tick();
        }
        dump("synth", y);
    }
    {   // Cosine: tests/fft.cpp (Cosine dct(N, &dct_in, &dct_out))
        double *in, *out;
        Cosine dct(64, &in, &out);
        for (int i = 0; i < 64; i++) in[i] = input(i);
        dct.forward();
        std::vector<double> y(out, out + 64);
        dct.backward();
        y.insert(y.end(), in, in + 64);
        dump("cosine", y);
    }
    {   // Oscbank<double, 8>: per-sample operator()/mixdown/tick, then fill
        Oscbank<double, 8> osc;
        for (int i = 0; i < 8; i++) osc.freqmod(i, 110.0 * (i + 1));
        osc.open();
        std::vector<double> m;
        for (int t = 0; t < 10; t++) {
            const std::complex<double> s = osc.mixdown();
            const std::complex<double> z3 = osc()(3);
            m.push_back(s.real());
            m.push_back(s.imag());
            m.push_back(z3.real());
            osc.tick();
        }
        std::vector<std::complex<double>> mix(100);
        osc.fill(mix.data(), 100);
        for (auto& c : mix) {
            m.push_back(c.real());
            m.push_back(c.imag());
        }
        dump("oscbank", m);
    }
    {   // Additive (tests/additive.cpp shape, small) and Sinusoids
        Additive<double> add(&cycle, 4, 8, 0.75, 1.0);
        add.makenote(48, 1.0);
        add.makenote(55, 0.5);
        std::vector<double> y(2000);
        for (int t = 0; t < 50; t++) {
            y[t] = add();
            add.tick();
        }
        add.fill(y.data() + 50, 1950);
        dump("additive", y);
        Sinusoids<double> sins(&cycle, 220.0, 6, 0.8);
        std::vector<double> s(1000);
        sins.fill(s.data(), 1000);
        dump("sinusoids", s);
    }
    {   // Granulator: tests/granny.cpp:34-56 per sample (write; granny(); request; tick), then process()
        Buffer<double> source(3000);
        Granulator<double> granny(&hann, &source, true, 16);
        auto par = [](int t) {
            return hz_grain_req{0, 0.001 * (t % 7), 0.002 + 0.0005 * (t % 11), 0.5 + 0.25 * (t % 5), 0.3, 0.0};
        };
        std::vector<double> y(4000);
        std::vector<double> v;
        for (int t = 0; t < 2000; t++) {
            source.write(input(t));
            y[t] = granny();
            if (t % 97 == 0) {
                const hz_grain_req r = par(t);
                v.push_back((double)(int)granny.request(r.offset, r.size, r.speed, r.gain, r.pan));
            }
            source.tick();
            granny.tick();
        }
        std::vector<hz_grain_req> reqs;
        std::vector<double> x(2000);
        for (int i = 0; i < 2000; i++) {
            x[i] = input(2000 + i);
            if ((2000 + i) % 97 == 0) {
                reqs.push_back(par(2000 + i));
                reqs.back().at = i;
            }
        }
        std::vector<int> voices;
        granny.process(x.data(), y.data() + 2000, 2000, reqs, &voices);
        for (int vv : voices) v.push_back(vv);
        dump("granulator", y);
        dump("granulator_voices", v);
    }
    {   // Freezer<64>(4, 1): tests/freezer.cpp pattern (per-sample operator(), freeze/unfreeze), then process()
        std::srand(11);
        Freezer<64> fr(4, 1);
        std::vector<double> y(3000);
        for (int t = 0; t < 1000; t++) {
            if (t == 400) fr.freeze();
            if (t == 900) fr.unfreeze();
            y[t] = fr(input(t));
        }
        std::vector<double> x(2000);
        for (int i = 0; i < 2000; i++) x[i] = input(1000 + i);
        fr.process(x.data(), y.data() + 1000, 2000, {{300, HZ_FRZ_FREEZE}, {1500, HZ_FRZ_UNFREEZE}});
        dump("freezer", y);
    }
    {   // tests/harmbank.cpp: 96 channels, transpose() / measure(), both banks open; per-sample, then blocks
        const int octaves = 4, division = 12, parities = 2, n = parities * division * octaves;
        const double frequency = mtof(24), detune = 0.125;
        std::vector<std::complex<double>> radii(n);
        std::vector<double> fa(n), fs(n);
        for (int i = 0; i < division * octaves; i++)
            for (int l = 0; l < parities; l++) {
                const double midi = (i + detune * std::pow(2 * (0 + 0.5) / 1.0 - 1, 1)) / division;
                const double partial = frequency * std::pow(2, midi) * 1 * std::pow(-1, l);
                const int idx = parities * i + l;
                fa[idx] = partial;
                fs[idx] = -1 * partial * std::pow(2, (double)division / division);
                radii[idx] = std::min(0.999, std::exp((std::log(0.5) - 4 - 1) / (25 * SR / std::abs(partial))));
            }
        Heterodyne<96> het(4, radii);
        for (int i = 0; i < n; i++) {
            het.analysis().freqmod(i, fa[i]);
            het.synthesis().freqmod(i, fs[i]);
        }
        het.analysis().open();
        het.synthesis().open();
        std::vector<double> y(4000);
        for (int t = 0; t < 500; t++) y[t] = het(0.3 * input(t));
        std::vector<double> x(3500);
        for (int i = 0; i < 3500; i++) x[i] = 0.3 * input(500 + i);
        het.process(x.data(), y.data() + 500, 3500);
        dump("heterodyne", y);

        // the same instrument behind the offline Audio engine (src/audio.h stand-in): a
        // fresh chain, a 1000-frame float WAV in, float WAV out
        Heterodyne<96> het2(4, radii);
        for (int i = 0; i < n; i++) {
            het2.analysis().freqmod(i, fa[i]);
            het2.synthesis().freqmod(i, fs[i]);
        }
        het2.analysis().open();
        het2.synthesis().open();
        std::vector<float> xin(1000);
        for (int t = 0; t < 1000; t++) xin[t] = (float)(0.3 * input(t));
        wav::write(dir + "/audio_in.wav", xin.data(), xin.size(), 1, SR);
        g_het = &het2;
        Audio A(het_process, BSIZE);
        Audio::offline(dir + "/audio_in.wav", dir + "/audio_out.wav");
        A.startup(1, 1, false);
        A.shutdown();
    }
    std::printf("dropin ok\n");
    return 0;
}
