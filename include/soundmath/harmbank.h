// soundmath/harmbank.h -- the heterodyne bank chain of tests/harmbank.cpp:77-101 as one
// fused drop-in over the HIP engine.
//
// The reference composes seven banks per sample in user code:
//     limiter(dry * in + gain * mixdown(demodulators(synthesis(), smoothbank(latchbank(&rmsbank,
//         slidebank(modulators(in, analysis())))))));
//     analysis.tick(); synthesis.tick(); slidebank.tick(); smoothbank.tick(); rmsbank.tick();
// with Oscbank (src/oscbank.h), Modbank (modbank.h), Slidebank (slidebank.h), Latchbank
// (latchbank.h), RMSbank (rmsbank.h), Stickbank (stickbank.h) and Mixer (mixer.h).  On the
// GPU the N-wide intermediate signals never leave registers, so the chain is one object:
// Heterodyne<N>(slide order, radii, Latchbank thresh/ratio, RMSbank width, Stickbank order/rad,
// dry, gain).  analysis() / synthesis() return the two Oscbanks' controls (freqmod, activate,
// deactivate, open, close); setup() is Slidebank::setup.  process() runs n iterations of the
// loop body above; operator()(in) is one.
#pragma once

#include <complex>
#include <vector>

#include "hz.h"

namespace soundmath {

template <int N>
class Heterodyne {
public:
    // the Oscbank controls of one bank (oscbank.h:49-56, multichannel.h:90-130)
    class Bank {
    public:
        void freqmod(int index, double target) { detail::check(hz_het_freqmod(h_, b_, &index, &target, 1), "freqmod"); }
        void activate(const std::vector<int>& indices) {
            detail::check(hz_het_activate(h_, b_, indices.data(), (int)indices.size(), 1), "activate");
        }
        void deactivate(const std::vector<int>& indices) {
            detail::check(hz_het_activate(h_, b_, indices.data(), (int)indices.size(), 0), "deactivate");
        }
        void open() { detail::check(hz_het_open(h_, b_, 1), "open"); }
        void close() { detail::check(hz_het_open(h_, b_, 0), "close"); }

    private:
        friend class Heterodyne;
        Bank(hz_het* h, int b) : h_(h), b_(b) {}
        hz_het* h_;
        int b_;
    };

    // defaults: tests/harmbank.cpp:47-52 (Latchbank(0.0005), RMSbank(SR / 20), Stickbank(1, -0.9)),
    // dry 0, gain 3 (harmbank.cpp:55-56)
    Heterodyne(int order, const std::vector<std::complex<double>>& radii, double thresh = 0.0005, double ratio = 0.2,
               unsigned width = SR / 20, int stick_order = 1, double stick_rad = -0.9, double dry = 0,
               double gain = 3, int device = 0) {
        hz_het* h = nullptr;
        detail::check(hz_het_create(N, order, reinterpret_cast<const double*>(radii.data()), thresh, ratio, width,
                                    stick_order, stick_rad, dry, gain, device, &h),
                      "Heterodyne");
        h_ = decltype(h_)(h);
    }

    Bank analysis() { return Bank(h_.get(), HZ_HET_ANALYSIS); }
    Bank synthesis() { return Bank(h_.get(), HZ_HET_SYNTHESIS); }

    // Slidebank::setup (slidebank.h:63-100): new order and radii, zeroed stages
    void setup(int order, const std::vector<std::complex<double>>& radii) {
        detail::check(hz_het_setup(h_.get(), order, reinterpret_cast<const double*>(radii.data())), "setup");
    }

    double operator()(double in) {
        double y = 0;
        detail::check(hz_het_process(h_.get(), &in, &y, 1), "Heterodyne::operator()");
        return y;
    }
    void process(const double* in, double* out, std::size_t n) {
        detail::check(hz_het_process(h_.get(), in, out, n), "Heterodyne::process");
    }
    void process(const float* in, float* out, std::size_t n) {   // the Audio callback's float buffers
        std::vector<double> x(in, in + n), y(n);
        process(x.data(), y.data(), n);
        for (std::size_t i = 0; i < n; ++i) out[i] = (float)y[i];
    }
    hz_het* native() const { return h_.get(); }

private:
    handle<hz_het, hz_het_destroy> h_;
};

}  // namespace soundmath
