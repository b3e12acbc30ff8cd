// soundmath/hz.h -- shared pieces of the drop-in headers over libhuygens_hip.so.
//
// The reference is header-only C++ in namespace soundmath (src/*.h); these headers keep
// its class names and signatures as thin, move-only wrappers over
// the C ABI in huygens_hip.h.  Errors: the C ABI returns codes; the wrappers throw
// std::runtime_error with hz_last_error() (the reference aborts through eigen_assert).
// Constants and helpers of src/includes.h:30-60 and the shapes of src/wave.h:142-150 are
// `inline` here so several translation units can link (the reference's are not).
#pragma once

#include <cmath>
#include <complex>
#include <cstddef>
#include <limits>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../huygens_hip.h"

namespace soundmath {

typedef unsigned long ulong;
typedef unsigned int uint;

inline constexpr double PI = 3.14159265359;   // includes.h:30 (truncated, kept)
inline constexpr double E = 2.718281828459045;
inline constexpr int SR = 48000;
inline constexpr double A4 = 440.0;

// includes.h:43-48
inline double relaxation(double k) {
    if (k == 0) return 0;
    return std::pow(2.0, std::log2(std::numeric_limits<double>::epsilon()) / (std::fmax(0, k) * SR));
}
inline double mtof(double midi) { return A4 * std::pow(2, (midi - 69) / 12); }   // includes.h:51-54
inline double ftom(double frequency) { return 69 + std::log2(frequency / A4) * 12; }

namespace detail {
inline void check(int code, const char* what) {
    if (code != HZ_OK) throw std::runtime_error(std::string(what) + ": " + hz_last_error());
}
}  // namespace detail

// Shapes (wave.h:142-150).  Device code cannot call a host std::function, so a shape is
// an identity the banks recognise (cycle for Additive / Sinusoids / Bowl) and a host
// callable for user code.
enum class Shape { cycle, hann, halfhann, limiter };

template <typename T>
struct Wave {
    Shape shape;
    T operator()(double p) const { return lookup(p); }
    T lookup(double p) const {
        switch (shape) {
        case Shape::cycle: return (T)std::sin(2 * PI * p);
        case Shape::hann: return (T)(0.5 * (1 - std::cos(2 * PI * p)));
        case Shape::halfhann: return (T)std::sqrt(0.5 * (1 - std::cos(2 * PI * p)));
        default: return (T)(2.0 / PI * std::atan(p));
        }
    }
};

inline Wave<double> cycle{Shape::cycle};
inline Wave<double> hann{Shape::hann};
inline Wave<double> halfhann{Shape::halfhann};
inline Wave<double> limiter{Shape::limiter};
inline Wave<float> cycle_f{Shape::cycle};   // the Wave<float> sin(2 PI p) of Bowl<float>

// pointer + length view replacing `const ArrayCT*` (oscbank.h:65)
template <typename T>
struct cspan {
    const T* data = nullptr;
    std::size_t size = 0;
    const T& operator()(std::size_t i) const { return data[i]; }
    const T& operator[](std::size_t i) const { return data[i]; }
    T sum() const {
        T s{};
        for (std::size_t i = 0; i < size; ++i) s += data[i];
        return s;
    }
};

// move-only owner of a C handle
template <typename H, int (*Destroy)(H*)>
class handle {
public:
    handle() = default;
    explicit handle(H* h) : h_(h) {}
    handle(const handle&) = delete;
    handle& operator=(const handle&) = delete;
    handle(handle&& o) noexcept : h_(o.h_) { o.h_ = nullptr; }
    handle& operator=(handle&& o) noexcept {
        std::swap(h_, o.h_);
        return *this;
    }
    ~handle() {
        if (h_) Destroy(h_);
    }
    H* get() const { return h_; }

private:
    H* h_ = nullptr;
};

}  // namespace soundmath
