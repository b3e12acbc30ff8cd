// soundmath/additive.h -- drop-in Additive<T> (src/additive.h:11-71) with the Minimizer
// note API (src/minimizer.h:111-187) over the HIP engine.  T = double, form = &cycle;
// physics() (Gravity between partials) is out of scope.
// operator()() / tick() keep the reference's per-sample pair: operator() renders the
// current sample once (cached until tick()), tick() advances.
#pragma once

#include "hz.h"

namespace soundmath {

template <typename T>
class Additive {
    static_assert(std::is_same<T, double>::value, "the HIP Additive computes in double");

public:
    Additive(Wave<T>* form, uint voices, uint overtones, T decay, T harmonicity = 1.0, T k = 0.1, int device = 0) {
        if (!form || form->kind != Shape::cycle) throw std::runtime_error("Additive: only the cycle waveform runs on the device");
        hz_add* h = nullptr;
        detail::check(hz_add_create((int)voices, (int)overtones, decay, harmonicity, k, device, &h), "Additive");
        h_ = decltype(h_)(h);
    }
    T operator()() {
        if (!computed_) {
            detail::check(hz_add_fill(h_.get(), &last_, 1), "Additive::operator()");
            computed_ = true;
        }
        return last_;
    }
    void tick() {
        if (!computed_) {
            T y;
            detail::check(hz_add_fill(h_.get(), &y, 1), "Additive::tick");
        }
        computed_ = false;
    }
    int request(T fundamental, T amplitude) {
        int v = -1;
        detail::check(hz_add_request(h_.get(), fundamental, amplitude, &v), "Additive::request");
        return v;
    }
    void release(int voice) { detail::check(hz_add_release(h_.get(), voice), "Additive::release"); }
    int makenote(T pitch, T amplitude) {
        int v = -1;
        detail::check(hz_add_makenote(h_.get(), pitch, amplitude, &v), "Additive::makenote");
        return v;
    }
    void endnote(T pitch) { detail::check(hz_add_endnote(h_.get(), pitch), "Additive::endnote"); }
    // n x { out[t] = operator()(); tick(); }
    void fill(T* out, std::size_t n) { detail::check(hz_add_fill(h_.get(), out, n), "Additive::fill"); }
    hz_add* native() const { return h_.get(); }

private:
    handle<hz_add, hz_add_destroy> h_;
    bool computed_ = false;
    T last_ = 0;
};

}  // namespace soundmath
