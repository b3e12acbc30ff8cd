// soundmath/includes.h -- the constants and helpers of src/includes.h:28-80, host-only and
// `inline` (the reference defines them as non-inline globals, so it links as one translation
// unit only; demos here may span several).  The reference's unconditional PortAudio / RtMidi /
// Eigen includes (includes.h:17-26) are not needed by the HIP banks and are left out.
#pragma once

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstdlib>
#include <iostream>
#include <limits>
#include <stdexcept>
#include <string>
#include <vector>

typedef unsigned long ulong;   // includes.h:28 (global, as there)

namespace soundmath {

typedef unsigned int uint;

inline constexpr double PI = 3.14159265359;      // includes.h:30 (truncated: every phase uses it)
inline constexpr double E = 2.718281828459045;   // 31
inline constexpr int SR = 48000;                 // 32 (an int: x / SR divides in floating point)
inline constexpr int FORCE = 50000;              // 34
inline constexpr double A4 = 440.0;              // 35

inline const double epsilon = std::numeric_limits<double>::epsilon();   // 38
inline const double order = std::log2(epsilon);                        // 39

// relaxation(k): the stiffness whose smoothing settles in k seconds (includes.h:41-48)
inline double relaxation(double k) {
    if (k == 0) return 0;
    return std::pow(2.0, order / (std::fmax(0, k) * SR));
}
inline double mtof(double midi) { return A4 * std::pow(2, (midi - 69) / 12); }          // 51-54
inline double ftom(double frequency) { return 69 + std::log2(frequency / A4) * 12; }    // 56-59
inline double atodb(double amplitude) { return 20 * std::log(amplitude); }              // 61-64
inline double dbtoa(double db) { return std::pow(10, db / 20); }                        // 66-69
inline std::string notename(int midi) {                                                 // 71-75
    static const std::string notes = "C C#D D#E F F#G G#A A#B ";
    return notes.substr(2 * (midi % 12), 2) + std::to_string(midi / 12 - 1);
}
template <typename T>
int sgn(T val) {   // 77-80
    return (T(0) < val) - (val < T(0));
}

}  // namespace soundmath
