// soundmath/granulator.h -- drop-in Granulator<T> (src/granulator.h:12-127) over the HIP
// engine, with the Buffer<T> it reads (src/buffer.h:9-86) and the Granary<T> parameter
// source (src/granulator.h:129-192).  T = double (the engine's arithmetic).
//
// Granulator's bank (up to `polyphony` grains summed per sample) runs on the GPU.  The
// engine keeps its own device copy of the source ring: operator()() hands it the sample
// the caller last wrote at the Buffer's origin (tests/granny.cpp:36-37 writes, then reads),
// so the two rings hold the same data under the write-read-tick pattern the reference's
// demo uses.  process() is the block form of that pattern (the fast path).
//
// Deviations (documented in INTEGRATION.md): the window must be &hann (the only one the
// reference uses); tick() without a preceding operator()() counts as a read whose output
// is discarded; request() returns (unsigned)-1 like the reference when no voice is free.
#pragma once

#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <type_traits>
#include <vector>

#include "buffer.h"
#include "hz.h"

namespace soundmath {

template <typename T>
class Granulator {
    static_assert(std::is_same<T, double>::value, "the HIP Granulator computes in double");

public:
    Granulator(Wave<T>* window, Buffer<T>* source, bool realtime = true, unsigned polyphony = 512, int device = 0)
        : source_(source) {
        (void)realtime;   // unused by the reference as well (granulator.h:117)
        if (!window || window->kind != Shape::hann)
            throw std::runtime_error("Granulator: the HIP engine supports the hann window (wave.h:148)");
        hz_gran* h = nullptr;
        detail::check(hz_gran_create(polyphony, source->get_size(), device, &h), "Granulator");
        h_ = decltype(h_)(h);
    }

    // granulator.h:51-79: request a grain; returns the voice, (unsigned)-1 if none
    unsigned request(T offset, T size, T speed, T gain, T pan) {
        int v = -1;
        detail::check(hz_gran_request(h_.get(), offset, size, speed, gain, pan, read_pending_ ? 1 : 0, &v),
                      "Granulator::request");
        return (unsigned)v;
    }

    // granulator.h:81-86
    void tick() {
        if (!read_pending_) (void)(*this)();   // a read the caller skipped (see the header note)
        read_pending_ = false;
    }

    // granulator.h:88-104: the sum over active grains for the sample at the source's origin
    T operator()() {
        if (read_pending_) return last_;   // repeated read before tick(): same value
        const T x = source_->current();
        detail::check(hz_gran_sample(h_.get(), x, &last_), "Granulator::operator()");   // per-sample server
        read_pending_ = true;
        return last_;
    }

    bool idle() {   // granulator.h:106-109
        unsigned a = 0;
        detail::check(hz_gran_activity(h_.get(), &a), "Granulator::idle");
        return a == 0;
    }

    // n x { source.write(in[i]); out[i] = (*this)(); <requests at i>; source.tick(); tick(); }
    // (the source Buffer object itself is not updated by the block form)
    void process(const T* in, T* out, std::size_t n, const std::vector<hz_grain_req>& reqs = {},
                 std::vector<int>* voices = nullptr) {
        if (voices) voices->assign(reqs.size(), -1);
        detail::check(hz_gran_process(h_.get(), in, out, n, reqs.data(), (int)reqs.size(),
                                      voices ? voices->data() : nullptr),
                      "Granulator::process");
    }
    hz_gran* native() const { return h_.get(); }

private:
    Buffer<T>* source_;
    handle<hz_gran, hz_gran_destroy> h_;
    bool read_pending_ = false;
    T last_ = 0;
};

// Granary<T> (granulator.h:129-192): a host-side grain-parameter source (rand() noise and
// a metronome), kept as in the reference so a demo's control logic is unchanged.
template <typename T>
class Granary {
    static const int shape = 0, jitter = 1, speed = 2, warble = 3, size = 4, texture = 5, density = 6, spray = 7,
                     pan = 8, scatter = 9, gain = 10, wobble = 11, n_params = 12;

public:
    Granary() {
        std::memset(params_, 0, sizeof(params_));   // uninitialised in the reference
        (void)std::rand();   // Noise<T>'s constructor draws once (noise.h:11-14)
    }
    void tick() {   // Metro<T>::tick (metro.h:23-28) over Oscillator<T>::tick (oscillator.h:27-38)
        const T old = phase_;
        osc_tick();
        clicked_ = phase_ < old;
    }
    bool parameters(T* the_offset, T* the_size, T* the_speed, T* the_gain, T* the_pan) {
        if (clicked_ && (1 + noise() > 2 * params_[spray])) {
            *the_offset = noise() * params_[jitter];
            *the_size = params_[size] * std::pow(2, params_[texture] * noise());
            *the_speed = params_[speed] * std::pow(2, params_[warble] * noise());
            *the_gain = params_[gain] * std::pow(2, params_[wobble] * noise());
            *the_pan = params_[pan] + noise();
            return true;
        }
        return false;
    }
    void instruct(T param, int index) {
        params_[index] = param;
        if (index == spray || index == density) target_ = params_[density] / (1 - params_[spray] * 0.999);
    }

private:
    // Noise<T>(-1, 1) (noise.h:11-28): a fresh rand() value per call
    static T noise() { return -1 + ((T)std::rand() / RAND_MAX) * 2; }
    // Oscillator<T>(f = 0, phi = 0, k = 2/SR): smoothed frequency, phase accumulators
    void osc_tick() {
        phase_ += freq_ / SR;
        target_phase_ += freq_ / SR;
        freq_ = target_ * (1 - s_) + freq_ * s_;
        const T w = (1 - s_) * std::sin(2 * PI * (2 * std::fabs(target_phase_ - phase_) + 0.25));
        phase_ = w * target_phase_ + (1 - w) * phase_;
        phase_ -= (int)phase_;
        target_phase_ -= (int)target_phase_;
    }
    T params_[n_params];
    T phase_ = 0, target_phase_ = 0, freq_ = 0, target_ = 0;
    T s_ = (T)relaxation(2.0 / SR);
    bool clicked_ = false;
};

}  // namespace soundmath
