// soundmath/hz.h -- shared pieces of the drop-in headers over libhuygens_hip.so.
//
// The reference is header-only C++ in namespace soundmath (src/*.h); these headers keep
// its class names and signatures as thin, move-only wrappers over
// the C ABI in huygens_hip.h.  Errors: the C ABI returns codes; the wrappers throw
// std::runtime_error with hz_last_error() (the reference aborts through eigen_assert).
// Constants and helpers (includes.h) and the shapes (wave.h) are `inline` so several translation
// units can link (the reference's are not).
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
#include "includes.h"
#include "wave.h"

namespace soundmath {

namespace detail {
inline void check(int code, const char* what) {
    if (code != HZ_OK) throw std::runtime_error(std::string(what) + ": " + hz_last_error());
}
}  // namespace detail

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
