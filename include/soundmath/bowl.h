// soundmath/bowl.h -- drop-in Bowl<T> (src/bowl.h:10-74) over the HIP engine.
// T = double (form &cycle) or float (form &cycle_f, the Wave<float> sin(2 PI p) that
// &cycle cannot be for T = float).
#pragma once

#include "hz.h"

namespace soundmath {

template <typename T>
class Bowl {
    static_assert(std::is_same<T, double>::value || std::is_same<T, float>::value, "Bowl<double> or Bowl<float>");

public:
    Bowl(int overtones, const std::vector<T>& f, const std::vector<T>& a, const std::vector<T>& d,
         Wave<T>* form = default_form(), int device = 0) {
        if (!form || form->kind != Shape::cycle) throw std::runtime_error("Bowl: only sin(2 PI p) runs on the device");
        const std::vector<double> fd(f.begin(), f.end()), ad(a.begin(), a.end()), dd(d.begin(), d.end());
        const int count = (int)std::min(fd.size(), std::min(ad.size(), dd.size()));
        hz_bowl* h = nullptr;
        detail::check(hz_bowl_create(overtones, fd.data(), ad.data(), dd.data(), count,
                                     std::is_same<T, float>::value ? 1 : 0, device, &h),
                      "Bowl");
        h_ = decltype(h_)(h);
    }
    void trigger() {
        detail::check(hz_bowl_trigger(h_.get()), "Bowl::trigger");
        computed_ = false;
    }
    T operator()() {
        if (!computed_) {
            double y;
            detail::check(hz_bowl_render(h_.get(), &y, 1), "Bowl::operator()");
            last_ = (T)y;
            computed_ = true;
        }
        return last_;
    }
    void tick() {
        if (!computed_) {
            double y;
            detail::check(hz_bowl_render(h_.get(), &y, 1), "Bowl::tick");
        }
        computed_ = false;
    }
    int fill(float* buffer, int bsize) {
        detail::check(hz_bowl_fill(h_.get(), buffer, (std::size_t)bsize), "Bowl::fill");
        return 0;
    }
    hz_bowl* native() const { return h_.get(); }

private:
    static Wave<T>* default_form() {
        if constexpr (std::is_same<T, float>::value) return &cycle_f;
        else return &cycle;
    }
    handle<hz_bowl, hz_bowl_destroy> h_;
    bool computed_ = false;
    T last_ = 0;
};

}  // namespace soundmath
