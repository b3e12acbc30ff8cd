// soundmath/wave.h -- Wave<T> (src/wave.h:17-140) with the reference's FUNCTIONAL lookup
// (wave.h:4, 65-70: lookup(p) calls the shape directly; the 65,536-entry table is built there but
// never read, so it is not built here), and the global shapes of wave.h:142-150.
//
// A Wave also carries a `kind`: the GPU banks evaluate their shape inside the kernels (device
// code cannot call a host std::function), so Additive / Sinusoids / Bowl accept the cycle shape
// and Granulator the hann window, and refuse other Waves with an exception; host code (Synth,
// Oscillator users, demos) calls any Wave, including user lambdas, exactly as the reference.
#pragma once

#include <functional>

#include "includes.h"

namespace soundmath {

inline constexpr int TABSIZE = 65536;   // wave.h:10 (the table size of the non-FUNCTIONAL build)

enum Interp { none = 0, linear = 1, quadratic = 2, cubic = 3 };   // wave.h:12-15

// shapes the device banks recognise
enum class Shape { custom, cycle, hann, halfhann, limiter, saw, triangle, square, phasor };

template <typename T>
class Wave {
public:
    Wave() = default;
    // wave.h:23-38 (interpolation and bounds only matter to the table lookup FUNCTIONAL skips)
    Wave(std::function<T(double)> shape, Interp interp = Interp::cubic, T left = 0, T right = 1,
         bool periodic = true, Shape kind = Shape::custom)
        : kind(kind), shape_(std::move(shape)), interp_(interp), left_(left), right_(right), periodic_(periodic) {}

    T lookup(T input) const { return shape_(input); }          // wave.h:67-70 (FUNCTIONAL)
    T operator()(T phase) const { return lookup(phase); }       // 112-115
    // wave.h:117-125 sums the two tables, which FUNCTIONAL lookups never read (its result has no
    // shape and throws std::bad_function_call when called); here the sum of the shapes
    Wave<T> operator+(const Wave<T>& other) const {
        auto a = shape_, b = other.shape_;
        return Wave<T>([a, b](double p) -> T { return a(p) + b(p); }, interp_, left_, right_, periodic_);
    }

    Shape kind = Shape::custom;

private:
    std::function<T(double)> shape_;
    Interp interp_ = Interp::cubic;
    T left_ = 0, right_ = 1;
    bool periodic_ = true;
};

// wave.h:142-150.  abs() is taken as fabs (the reference's unqualified abs(double) resolves to
// fabs under the author's macOS libc++)
inline Wave<double> saw([](double phase) -> double { return 2 * phase - 1; }, Interp::linear, 0, 1, true, Shape::saw);
inline Wave<double> triangle([](double phase) -> double { return std::fabs(std::fmod(4 * phase + 3, 4.0) - 2) - 1; },
                             Interp::linear, 0, 1, true, Shape::triangle);
inline Wave<double> square([](double phase) -> double { return phase > 0.5 ? 1 : (phase < 0.5 ? -1 : 0); },
                           Interp::none, 0, 1, true, Shape::square);
inline Wave<double> phasor([](double phase) -> double { return phase; }, Interp::linear, 0, 1, true, Shape::phasor);
inline Wave<double> cycle([](double phase) -> double { return std::sin(2 * PI * phase); }, Interp::cubic, 0, 1, true,
                          Shape::cycle);
inline Wave<double> hann([](double phase) -> double { return 0.5 * (1 - std::cos(2 * PI * phase)); }, Interp::cubic,
                         0, 1, true, Shape::hann);
inline Wave<double> halfhann([](double phase) -> double { return std::sqrt(0.5 * (1 - std::cos(2 * PI * phase))); },
                             Interp::cubic, 0, 1, true, Shape::halfhann);
inline Wave<double> limiter([](double phase) -> double { return 2.0 / PI * std::atan(phase); }, Interp::linear, -100,
                            100, false, Shape::limiter);
// Bowl<float>'s form: `cycle` is a Wave<double> and does not convert, so a
// float demo supplies a Wave<float> sin(2 PI p); this is that shape
inline Wave<float> cycle_f([](double phase) -> float { return (float)std::sin(2 * PI * phase); }, Interp::cubic, 0, 1,
                           true, Shape::cycle);

}  // namespace soundmath
