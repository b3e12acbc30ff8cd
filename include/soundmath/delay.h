// soundmath/delay.h -- drop-in Delay<T> (src/delay.h:10-108) and Delaybank<T,N> (the N-line
// bank SURVEY.md a21 defines; src/delaybank.h is a stub) over the HIP engine.
// T = double or float.  Ring indexing is bit-exact with src/buffer.h:40-47.
#pragma once

#include "hz.h"

namespace soundmath {

namespace detail {
template <typename T>
inline void split_taps(const std::vector<std::pair<uint, T>>& v, std::vector<unsigned>& t, std::vector<double>& g) {
    t.clear();
    g.clear();
    for (const auto& p : v) {
        t.push_back(p.first);
        g.push_back((double)p.second);
    }
}
}  // namespace detail

template <typename T, int N>
class Delaybank {
    static_assert(std::is_same<T, double>::value || std::is_same<T, float>::value, "T = double or float");

public:
    Delaybank(uint sparsity, uint time, int device = 0) {
        hz_dly* h = nullptr;
        detail::check(hz_dly_create(N, sparsity, time, std::is_same<T, float>::value ? 1 : 0, device, &h), "Delaybank");
        h_ = decltype(h_)(h);
    }
    void coefficients(int line, const std::vector<std::pair<uint, T>>& forward,
                      const std::vector<std::pair<uint, T>>& back) {
        std::vector<unsigned> ft, bt;
        std::vector<double> fg, bg;
        detail::split_taps(forward, ft, fg);
        detail::split_taps(back, bt, bg);
        detail::check(hz_dly_coefficients(h_.get(), line, ft.data(), fg.data(), (int)ft.size(), bt.data(), bg.data(),
                                          (int)bt.size()),
                      "Delaybank::coefficients");
    }
    void modulate_forward(int line, uint n, const std::pair<uint, T>& tap) {
        detail::check(hz_dly_modulate_forward(h_.get(), line, n, tap.first, (double)tap.second),
                      "Delaybank::modulate_forward");
    }
    void modulate_back(int line, uint n, const std::pair<uint, T>& tap) {
        detail::check(hz_dly_modulate_back(h_.get(), line, n, tap.first, (double)tap.second),
                      "Delaybank::modulate_back");
    }
    // one sample of every line; in: N per-line samples
    cspan<T> operator()(const T* in) {
        if (!computed_) {
            detail::check(hz_dly_sample(h_.get(), in, out_, 1), "Delaybank::operator()");   // per-sample server
            computed_ = true;
        }
        return {out_, (std::size_t)N};
    }
    // delay.h:92-97: after operator() the engine has advanced already; without one, both rings'
    // origins move and nothing is written (hz_dly_tick)
    void tick() {
        if (!computed_) detail::check(hz_dly_tick(h_.get(), 1), "Delaybank::tick");
        computed_ = false;
    }
    // in: mono [n] (per_line false) or [N][n]; out: [N][n] or the mixdown [n]
    void process(const T* in, T* out, std::size_t n, bool mix, bool per_line_input = false) {
        detail::check(hz_dly_process(h_.get(), in, out, n, per_line_input ? 1 : 0, mix ? 1 : 0), "Delaybank::process");
    }
    hz_dly* native() const { return h_.get(); }

private:
    handle<hz_dly, hz_dly_destroy> h_;
    bool computed_ = false;
    T out_[N] = {};
};

template <typename T>
class Delay {
public:
    Delay(uint sparsity, uint time, int device = 0) : bank_(sparsity, time, device) {}
    void coefficients(const std::vector<std::pair<uint, T>>& forward, const std::vector<std::pair<uint, T>>& back) {
        bank_.coefficients(0, forward, back);
    }
    void modulate_forward(uint n, const std::pair<uint, T>& forward) { bank_.modulate_forward(0, n, forward); }
    void modulate_back(uint n, const std::pair<uint, T>& back) { bank_.modulate_back(0, n, back); }
    T operator()(T sample) { return bank_(&sample)(0); }
    void tick() { bank_.tick(); }
    void process(const T* in, T* out, std::size_t n) { bank_.process(in, out, n, false); }

private:
    Delaybank<T, 1> bank_;
};

}  // namespace soundmath
