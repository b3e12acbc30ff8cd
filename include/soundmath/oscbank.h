// soundmath/oscbank.h -- drop-in Oscbank<T,N> (src/oscbank.h:15-97, Multichannel
// src/multichannel.h:16-159) over the HIP engine.  T = double.  fill() is the GPU path;
// operator()() returns the current phasors (cspan instead of const ArrayCT*), mixdown()
// their sum over the active set, tick() advances one sample on the device.
#pragma once

#include "hz.h"

namespace soundmath {

template <typename T, int N>
class Oscbank {
    static_assert(std::is_same<T, double>::value, "the HIP Oscbank computes in double");

public:
    explicit Oscbank(double k = 2.0 / SR, int device = 0) : z_(2 * N) {
        hz_osc* h = nullptr;
        detail::check(hz_osc_create(N, k, device, &h), "Oscbank");
        h_ = decltype(h_)(h);
    }
    void freqmod(int index, T hz) { detail::check(hz_osc_freqmod(h_.get(), index, hz), "Oscbank::freqmod"); }
    void tick() { detail::check(hz_osc_fill(h_.get(), nullptr, nullptr, 1), "Oscbank::tick"); }
    cspan<std::complex<T>> operator()() {
        detail::check(hz_osc_phases(h_.get(), z_.data()), "Oscbank::operator()");
        return {reinterpret_cast<const std::complex<T>*>(z_.data()), (std::size_t)N};
    }
    std::complex<T> mixdown() {
        double m[2];
        detail::check(hz_osc_mixdown(h_.get(), m), "Oscbank::mixdown");
        return {m[0], m[1]};
    }
    void activate(const std::vector<int>& idx) {
        detail::check(hz_osc_activate(h_.get(), idx.data(), (int)idx.size()), "Oscbank::activate");
    }
    void deactivate(const std::vector<int>& idx) {
        detail::check(hz_osc_deactivate(h_.get(), idx.data(), (int)idx.size()), "Oscbank::deactivate");
    }
    void open() { detail::check(hz_osc_open(h_.get()), "Oscbank::open"); }
    void close() { detail::check(hz_osc_close(h_.get()), "Oscbank::close"); }
    int activity() {
        int c = 0;
        detail::check(hz_osc_active_count(h_.get(), &c), "Oscbank::activity");
        return c;
    }
    // n x { mix[t] = mixdown(); per_band[t] = operator()(); tick(); }
    void fill(std::complex<T>* mix, std::size_t n, std::complex<T>* per_band = nullptr) {
        detail::check(hz_osc_fill(h_.get(), reinterpret_cast<double*>(mix), reinterpret_cast<double*>(per_band), n),
                      "Oscbank::fill");
    }
    hz_osc* native() const { return h_.get(); }

private:
    handle<hz_osc, hz_osc_destroy> h_;
    std::vector<double> z_;
};

}  // namespace soundmath
