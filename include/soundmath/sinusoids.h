// soundmath/sinusoids.h -- drop-in Sinusoids<T> (src/sinusoids.h:10-79) over the HIP
// engine.  T = double, form = &cycle.  The modulators' smoothing is applied per call
// boundary (a step at each fill/tick), see huygens_hip.h.
#pragma once

#include "hz.h"

namespace soundmath {

template <typename T>
class Sinusoids {
    static_assert(std::is_same<T, double>::value, "the HIP Sinusoids computes in double");

public:
    Sinusoids(Wave<T>* form, T fundamental, uint overtones, T decay, T harmonicity = 1, T k = 2.0 / SR,
              int device = 0) {
        if (!form || form->kind != Shape::cycle) throw std::runtime_error("Sinusoids: only the cycle waveform runs on the device");
        hz_sin* h = nullptr;
        detail::check(hz_sin_create(fundamental, (int)overtones, decay, harmonicity, k, device, &h), "Sinusoids");
        h_ = decltype(h_)(h);
    }
    T operator()() {
        if (!computed_) {
            detail::check(hz_sin_fill(h_.get(), &last_, 1), "Sinusoids::operator()");
            computed_ = true;
        }
        return last_;
    }
    void tick() {
        if (!computed_) {
            T y;
            detail::check(hz_sin_fill(h_.get(), &y, 1), "Sinusoids::tick");
        }
        computed_ = false;
    }
    void fundmod(T target) { detail::check(hz_sin_fundmod(h_.get(), target), "Sinusoids::fundmod"); }
    void decaymod(T target) { detail::check(hz_sin_decaymod(h_.get(), target), "Sinusoids::decaymod"); }
    void harmmod(T target) { detail::check(hz_sin_harmmod(h_.get(), target), "Sinusoids::harmmod"); }
    void fill(T* out, std::size_t n) { detail::check(hz_sin_fill(h_.get(), out, n), "Sinusoids::fill"); }
    hz_sin* native() const { return h_.get(); }

private:
    handle<hz_sin, hz_sin_destroy> h_;
    bool computed_ = false;
    T last_ = 0;
};

}  // namespace soundmath
