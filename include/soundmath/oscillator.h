// soundmath/oscillator.h -- Oscillator<T> (src/oscillator.h:12-71): one phase accumulator with
// smoothed frequency and phase modulation.  A single oscillator is scalar host work (a few flops
// per sample, the reference's own execution model); banks of them run on the GPU as
// Additive / Sinusoids / Oscbank.  Operation order as the reference (tick: oscillator.h:27-38).
#pragma once

#include "wave.h"

namespace soundmath {

template <typename T>
class Oscillator {
public:
    // k is the relaxation time in seconds (oscillator.h:15-24); abs() taken as fabs
    Oscillator(T f = 0, T phi = 0, T k = 2.0 / SR) {
        frequency = std::fabs(f);
        target_freq = frequency;
        phase = std::fmax(0, phi);
        target_phase = phase;
        stiffness = relaxation(k);
    }

    // once per sample (27-38)
    void tick() {
        phase += frequency / SR;
        target_phase += frequency / SR;
        frequency = target_freq * (1 - stiffness) + frequency * stiffness;
        T weight = (1 - stiffness) * cycle(2 * std::fabs(target_phase - phase) + 0.25);   // phasemod(0.5) ambiguity
        phase = weight * target_phase + (1 - weight) * phase;
        phase -= int(phase);
        target_phase -= int(target_phase);
    }

    T lookup() { return phase; }       // 40-41
    T operator()() { return phase; }   // 43-44
    void freqmod(T target) { target_freq = target; }   // 46-47
    void phasemod(T offset) {          // 49-56: target_phase kept in [0, 1)
        target_phase += offset;
        target_phase -= int(target_phase);
        target_phase += 1;
        target_phase -= int(target_phase);
    }
    void reset(T f) {                  // 58-62
        frequency = target_freq = f;
        phase = target_phase = 0;
    }

protected:
    T phase;
    T frequency;
    T target_freq;
    T target_phase;
    T stiffness;
};

}  // namespace soundmath
