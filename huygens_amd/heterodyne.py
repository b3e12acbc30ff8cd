"""The heterodyne bank chain of tests/harmbank.cpp:77-101 over the HIP engine.

Heterodyne(channels, order, radii, thresh, ratio, width, stick_order, stick_rad, dry, gain)
fuses Oscbank analysis / synthesis (src/oscbank.h), Modbank, Slidebank(order, radii)
(src/slidebank.h), RMSbank(width) (src/rmsbank.h), Latchbank(thresh, ratio)
(src/latchbank.h), Stickbank(stick_order, stick_rad) (src/stickbank.h), Mixer and the
limiter: process(x) returns, per sample,
    limiter(dry x + gain mixdown(demodulators(synthesis(), smoothbank(latchbank(&rmsbank,
            slidebank(modulators(x, analysis())))))))
followed by the five ticks.  harmbank() builds the reference's instrument configuration
(transpose() and measure() of tests/harmbank.cpp:108-200).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from ._lib import check, dptr, load

SR = 48000
ANALYSIS, SYNTHESIS = 0, 1
STATE_ANALYSIS, STATE_SYNTHESIS, STATE_SLIDE, STATE_RMS, STATE_LATCH, STATE_STICK, STATE_HISTORY = range(7)


def mtof(m):   # src/includes.h: 440 * 2^((m - 69) / 12)
    return 440.0 * math.pow(2.0, (m - 69) / 12.0)


def harmbank(octaves=4, division=12, courses=1, harmonics=1, parities=2, detune=0.125, c1=24, multiplicity=4,
             wavelengths=25.0, cutoff=0.999, scale=None):
    """The tests/harmbank.cpp instrument: (channels, analysis Hz, synthesis Hz, radii).

    transpose(&analysis, 0, 0, false), transpose(&synthesis, division, 0, true) and
    measure() (tests/harmbank.cpp:116-134,176-193) with the default scale (defaultize())."""
    n = parities * division * octaves * courses * harmonics
    frequency = mtof(c1)
    scale = list(range(division * octaves)) if scale is None else list(scale)
    fa, fs, radii = np.zeros(n), np.zeros(n), np.zeros(2 * n)

    def partials(interval, spectral, reverse, out, measure=False):
        ratio = math.pow(2, interval / division)
        for i in range(division * octaves):
            for j in range(courses):
                for k in range(harmonics):
                    for l in range(parities):
                        midi = (scale[i] + detune * math.pow(2 * (j + 0.5) / courses - 1, 1)) / division
                        idx = parities * (harmonics * (courses * i + j) + k) + l
                        if measure:
                            partial = frequency * math.pow(2, midi) * (k + 1) * math.pow(-1, l)
                            out[2 * idx] = min(cutoff, math.exp((math.log(0.5) - multiplicity - 1) /
                                                                (wavelengths * SR / abs(partial))))
                        else:
                            partial = frequency * math.pow(2, midi) * (k + spectral + 1) * ratio * math.pow(-1, l)
                            out[idx] = (-1 if reverse else 1) * partial

    partials(0, 0, False, fa)
    partials(division, 0, True, fs)
    partials(0, 0, False, radii, measure=True)
    return n, fa, fs, radii


class Heterodyne:
    def __init__(self, channels, order, radii, thresh=0.0005, ratio=0.2, width=SR // 20, stick_order=1,
                 stick_rad=-0.9, dry=0.0, gain=3.0, device=0):
        lib = load()
        radii = np.ascontiguousarray(radii, dtype=np.float64)
        if radii.size != 2 * channels:
            raise ValueError("radii: 2 x channels doubles (re, im)")
        h = C.c_void_p()
        check(lib.hz_het_create(channels, order, dptr(radii), thresh, ratio, width, stick_order, stick_rad, dry,
                                gain, device, C.byref(h)))
        self._h, self._lib = h, lib
        self.channels, self.order, self.width = channels, max(1, order), width
        self.stick_order = max(1, stick_order)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_het_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def setup(self, order, radii):
        radii = np.ascontiguousarray(radii, dtype=np.float64)
        check(self._lib.hz_het_setup(self._h, order, dptr(radii)))
        self.order = max(1, order)

    def freqmod(self, bank, index, hz):
        idx = np.ascontiguousarray(np.atleast_1d(index), dtype=np.int32)
        f = np.ascontiguousarray(np.atleast_1d(hz), dtype=np.float64)
        check(self._lib.hz_het_freqmod(self._h, bank, idx.ctypes.data_as(C.POINTER(C.c_int)), dptr(f), idx.size))

    def activate(self, bank, index, on=True):
        idx = np.ascontiguousarray(np.atleast_1d(index), dtype=np.int32)
        check(self._lib.hz_het_activate(self._h, bank, idx.ctypes.data_as(C.POINTER(C.c_int)), idx.size,
                                        1 if on else 0))

    def open(self, bank, on=True):
        check(self._lib.hz_het_open(self._h, bank, 1 if on else 0))

    def process(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(x.size)
        check(self._lib.hz_het_process(self._h, dptr(x), dptr(y), x.size))
        return y

    def process_device(self, in_ptr, out_ptr, n):
        check(self._lib.hz_het_process_device(self._h, C.c_void_p(in_ptr), C.c_void_p(out_ptr), n))

    def state(self, what):
        size = {STATE_SLIDE: 2 * self.order, STATE_RMS: 1, STATE_STICK: 2 * self.stick_order,
                STATE_HISTORY: self.width}.get(what, 2)
        out = np.zeros(self.channels * size)
        check(self._lib.hz_het_state(self._h, what, dptr(out)))
        return out

    def set_stream(self, stream):
        check(self._lib.hz_het_set_stream(self._h, C.c_void_p(stream)))

    def synchronize(self):
        check(self._lib.hz_het_synchronize(self._h))

    def profile(self, enable=True):
        check(self._lib.hz_het_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        ms, launches, cs = C.c_double(), C.c_long(), C.c_long()
        check(self._lib.hz_het_profile_read(self._h, C.byref(ms), C.byref(launches), C.byref(cs)))
        return ms.value, launches.value, cs.value
