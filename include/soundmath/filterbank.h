// soundmath/filterbank.h -- drop-in Filterbank<T> (src/filterbank.h:16-188) over the HIP
// engine.  T = double (the engine's arithmetic).  process() is the block path; the per-sample
// operator()/tick() pair runs on the GPU's per-sample engine (hz_fb_sample: a kernel resident on
// the handle's stream, a few microseconds per sample whatever the band count) with the
// reference's exact semantics -- a repeated operator() before tick() returns the cached row
// (re-mixed with its functor), a tick() without operator() rotates the ring.
// operator()(T, T(*)(T)) takes a device functor id instead of a host function pointer
// (HZ_DIST_SOFTCLIP / SATURATE / LIMITER, see huygens_hip.h).
#pragma once

#include <cstdio>

#include "hz.h"

namespace soundmath {

template <typename T>
class Filterbank {
    static_assert(std::is_same<T, double>::value, "the HIP Filterbank computes in double");

public:
    Filterbank(int order, int N = 1, double k_p = 0.1, double k_g = 1, int device = 0) : N_(N), order_(order) {
        hz_fb* h = nullptr;
        detail::check(hz_fb_create(order, N, k_p, k_g, device, &h), "Filterbank");
        h_ = decltype(h_)(h);
    }
    void coefficients(int n, const std::vector<T>& forward, const std::vector<T>& back) {
        detail::check(hz_fb_coefficients(h_.get(), n, forward.data(), (int)forward.size(), back.data(),
                                         (int)back.size()),
                      "Filterbank::coefficients");
    }
    void boost(int n, T v) { detail::check(hz_fb_boost(h_.get(), n, v), "Filterbank::boost"); }
    void boost(const std::vector<T>& v) {
        detail::check(hz_fb_boost_all(h_.get(), v.data(), (int)v.size()), "Filterbank::boost");
    }
    void mix(int n, T v) { detail::check(hz_fb_mix(h_.get(), n, v), "Filterbank::mix"); }
    void mix(const std::vector<T>& v) {
        detail::check(hz_fb_mix_all(h_.get(), v.data(), (int)v.size()), "Filterbank::mix");
    }
    void open() { detail::check(hz_fb_open(h_.get()), "Filterbank::open"); }
    void print() { std::printf("Filterbank<double>(order %d, %d bands) on HIP\n", order_, N_); }

    T operator()(T sample) { return sample_with(sample, HZ_DIST_NONE, 0.0); }
    // F(x, &softclip) -> F(x, HZ_DIST_SOFTCLIP): the one-argument softclip's width 0.125 by default
    T operator()(T sample, int dist_id) { return sample_with(sample, dist_id, HZ_DIST_DEFAULT_PARAM(dist_id)); }
    T operator()(T sample, int dist_id, double param) { return sample_with(sample, dist_id, param); }
    void tick() { detail::check(hz_fb_sample_tick(h_.get()), "Filterbank::tick"); }

    // n x { out[i] = operator()(in[i]); tick(); }
    void process(const T* in, T* out, std::size_t n, int dist_id = HZ_DIST_NONE, double param = -1.0) {
        if (param < 0.0) param = HZ_DIST_DEFAULT_PARAM(dist_id);
        detail::check(hz_fb_set_distortion(h_.get(), dist_id, param), "Filterbank::process");
        detail::check(hz_fb_process(h_.get(), in, out, n), "Filterbank::process");
    }
    // n x { coefficients(b, row t) for every band b; out[t] = operator()(in[t]); tick(); } --
    // the Subtractive ALLINONE / ONEPERVOICE pattern (src/subtractive.h:215-228, 300-317) as one
    // call.  coeffs: [n][2*order+1][N] (forward then back, band-minor).  The last row stays set.
    void process_stream(const T* in, T* out, std::size_t n, const T* coeffs, int dist_id = HZ_DIST_NONE,
                        double param = -1.0) {
        if (param < 0.0) param = HZ_DIST_DEFAULT_PARAM(dist_id);
        detail::check(hz_fb_set_distortion(h_.get(), dist_id, param), "Filterbank::process_stream");
        detail::check(hz_fb_process_tv(h_.get(), in, out, n, HZ_FB_TV_COEFFS, coeffs, 0.0),
                      "Filterbank::process_stream");
    }
    // the same with every band retuned to resonant(freqs[t][b], R) (order 2, subtractive.h:240-264)
    void process_resonant(const T* in, T* out, std::size_t n, const T* freqs, double R,
                          int dist_id = HZ_DIST_NONE, double param = -1.0) {
        if (param < 0.0) param = HZ_DIST_DEFAULT_PARAM(dist_id);
        detail::check(hz_fb_set_distortion(h_.get(), dist_id, param), "Filterbank::process_resonant");
        detail::check(hz_fb_process_tv(h_.get(), in, out, n, HZ_FB_TV_RESONANT, freqs, R),
                      "Filterbank::process_resonant");
    }
    // (new) the stationary engine: HZ_FB_RESP_OFF / _EAGER (default) / _LAZY
    void response(int mode) { detail::check(hz_fb_set_response(h_.get(), mode), "Filterbank::response"); }
    hz_fb* native() const { return h_.get(); }

private:
    T sample_with(T sample, int dist_id, double param) {
        T y = 0;
        detail::check(hz_fb_sample(h_.get(), sample, dist_id, param, &y), "Filterbank::operator()");
        return y;
    }
    handle<hz_fb, hz_fb_destroy> h_;
    int N_, order_;
};

// FFilterbank<T, N, order> (src/filterbank.h:191-319): the fixed-size variant.  The
// reference keeps the same maths in fixed-size Eigen types (its smoothing factors are T
// rather than double: identical for T = double), so it is the same engine with N and the
// order fixed at compile time; the API is Filterbank's minus print().
template <typename T, std::size_t N, std::size_t order>
class FFilterbank : public Filterbank<T> {
public:
    explicit FFilterbank(double k_p = 0.1, double k_g = 1, int device = 0)
        : Filterbank<T>((int)order, (int)N, k_p, k_g, device) {}
    void print() = delete;
};

// (new) one sample of several banks in ONE per-sample request: out[j] = (*F[j])(in[j], dist_id, param)
// for every j (each with its own pending tick()s) -- the multi-channel loop of tests/filterbanks.cpp:
// 191-211 keeps its per-channel tick() calls and changes one line, the channels' operator() calls
// into one call per sample:
//     double ys[CHANELS];   // xs[j] = each channel's filterbank input
//     soundmath::sample_many(Fs, CHANELS, xs, ys, HZ_DIST_SOFTCLIP);
template <typename Bank>
void sample_many(Bank* const* banks, int count, const double* in, double* out, int dist_id = HZ_DIST_NONE,
                 double param = -1.0) {
    if (param < 0.0) param = HZ_DIST_DEFAULT_PARAM(dist_id);   // &softclip: width 0.125
    hz_fb* hs[12];
    if (count > 12) detail::check(HZ_E_INVALID, "sample_many: at most 12 banks");
    for (int j = 0; j < count; ++j) hs[j] = banks[j]->native();
    detail::check(hz_fb_sample_many(hs, count, in, dist_id, param, out), "sample_many");
}

}  // namespace soundmath
