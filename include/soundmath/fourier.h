// soundmath/fourier.h -- drop-in Fourier (src/fourier.h:50-194), StaticSTFT
// (src/staticSTFT.h:10-177) and Cosine (src/fourier.h:197-234) over the HIP engine.
//
// Two ways to drive a Fourier, chosen by the first call:
//   per sample: write() / read() in any order and number, and the public slot operations
//     forward(i) / backward(i) / process(i) -- the reference's own state machine (O(2 laps)
//     bookkeeping per sample on the host), each slot transform and device processor on the GPU;
//   by blocks: process_block() == n x {write(x_t); read(&y_t)} on the GPU frame engine.
// A processor is the reference's int(*)(const complex<double>*, complex<double>*), run on the
// host per frame in frame order, or a built-in device processor (HZ_PROC_*).
#pragma once

#include "hz.h"

namespace soundmath {

class Fourier {
public:
    typedef int (*processor_t)(const std::complex<double>*, std::complex<double>*);

    Fourier(processor_t processor, int N, int laps, int device = 0) { init(HZ_PROC_HOST, N, laps, HZ_WIN_HALFHANN, device, processor); }
    // built-in device processor: HZ_PROC_IDENTITY, HZ_PROC_GATE_KEEP (625), HZ_PROC_HILBERT
    Fourier(int builtin, int N, int laps, int device = 0) { init(builtin, N, laps, HZ_WIN_HALFHANN, device, nullptr); }

    void write(double real, double imag = 0) { detail::check(hz_stft_write(h_.get(), real, imag), "Fourier::write"); }
    void read(double* real, double* imag) { detail::check(hz_stft_read(h_.get(), real, imag), "Fourier::read"); }
    void forward(const int i) { detail::check(hz_stft_forward(h_.get(), i), "Fourier::forward"); }
    void backward(const int i) { detail::check(hz_stft_backward(h_.get(), i), "Fourier::backward"); }
    void process(const int i) { detail::check(hz_stft_process_slot(h_.get(), i), "Fourier::process"); }
    void process_block(const double* re, const double* im, double* out_re, double* out_im, std::size_t n) {
        detail::check(hz_stft_process_block(h_.get(), re, im, out_re, out_im, n), "Fourier::process_block");
    }
    hz_stft* native() const { return h_.get(); }

protected:
    Fourier() = default;
    void init(int proc, int N, int laps, int window, int device, processor_t fn) {
        const double p0 = proc == HZ_PROC_STATIC_GATE ? 100.0 : (proc == HZ_PROC_GATE_KEEP ? 625.0 : 0.0);
        const double p1 = proc == HZ_PROC_STATIC_GATE ? 0.1 : 0.0;
        hz_stft* h = nullptr;
        detail::check(hz_stft_create(N, laps, window, proc, p0, p1, device, &h), "Fourier");
        h_ = decltype(h_)(h);
        if (fn)   // complex<double>* and double* (interleaved) are layout-compatible
            detail::check(hz_stft_set_processor(h, reinterpret_cast<hz_stft_proc>(fn)), "Fourier");
    }
    handle<hz_stft, hz_stft_destroy> h_;
};

class StaticSTFT : public Fourier {
public:
    StaticSTFT(int N, int laps, int device = 0) { init(HZ_PROC_STATIC_GATE, N, laps, HZ_WIN_HANN, device, nullptr); }
};

class Cosine {
public:
    Cosine(int N, double** in, double** out, int device = 0) {
        hz_dct* h = nullptr;
        detail::check(hz_dct_create(N, device, &h), "Cosine");
        h_ = decltype(h_)(h);
        detail::check(hz_dct_buffers(h, in, out), "Cosine");
    }
    void forward() { detail::check(hz_dct_forward(h_.get()), "Cosine::forward"); }
    void backward() { detail::check(hz_dct_backward(h_.get()), "Cosine::backward"); }
    hz_dct* native() const { return h_.get(); }

private:
    handle<hz_dct, hz_dct_destroy> h_;
};

// Freezer<N> (src/fourier.h:389-562): spectral freeze.  operator()(x) is one sample
// (a one-sample block); process() is the block form with freeze()/unfreeze() calls placed
// before given samples.  FFrame/IFrame/DFrame are internal to the engine.
template <int N>
class Freezer {
public:
    Freezer(int laps, double width, int device = 0) {
        hz_frz* h = nullptr;
        detail::check(hz_frz_create(N, laps, width, device, &h), "Freezer");
        h_ = decltype(h_)(h);
    }
    void freeze() { detail::check(hz_frz_freeze(h_.get()), "Freezer::freeze"); }
    void unfreeze() { detail::check(hz_frz_unfreeze(h_.get()), "Freezer::unfreeze"); }
    double operator()(double sample) {
        double y = 0;
        detail::check(hz_frz_process(h_.get(), &sample, &y, 1, nullptr, 0), "Freezer::operator()");
        return y;
    }
    void process(const double* in, double* out, std::size_t n, const std::vector<hz_frz_event>& events = {}) {
        detail::check(hz_frz_process(h_.get(), in, out, n, events.data(), (int)events.size()), "Freezer::process");
    }
    hz_frz* native() const { return h_.get(); }

private:
    handle<hz_frz, hz_frz_destroy> h_;
};

}  // namespace soundmath
