// soundmath/synth.h -- Synth<T> (src/synth.h:10-21): an Oscillator read through a Wave.
// Host code like the reference (one phase and one shape call per sample); any Wave, user lambdas
// included.  Many synths summed per sample are the Sinusoids / Additive GPU banks.
#pragma once

#include "oscillator.h"
#include "wave.h"

namespace soundmath {

template <typename T>
class Synth : public Oscillator<T> {
public:
    Synth(Wave<T>* form, double f, double phi = 0, double k = 2.0 / SR) : Oscillator<T>(f, phi, k) {
        waveform = form;
    }
    T operator()() { return (*waveform)(this->lookup()); }   // synth.h:16-17

private:
    Wave<T>* waveform;
};

}  // namespace soundmath
