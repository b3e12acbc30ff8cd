"""ctypes binding of the heterodyne-chain restatement (oracle/hz_oracle_het.c). TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle import D, I, L, PD, VP, _bind, _p

_SIGS = {
    "orc_het_create": (VP, [I, I, PD, D, D, C.c_uint, I, D, D, D]),
    "orc_het_destroy": (None, [VP]),
    "orc_het_setup": (None, [VP, I, PD]),
    "orc_het_freqmod": (None, [VP, I, I, D]),
    "orc_het_activate": (None, [VP, I, C.POINTER(I), I, I]),
    "orc_het_sample": (D, [VP, D]),
    "orc_het_process": (None, [VP, PD, PD, L]),
    "orc_het_state": (None, [VP, I, PD]),
}


class OracleHet:
    def __init__(self, channels, order, radii, thresh=0.0005, ratio=0.2, width=2400, stick_order=1, stick_rad=-0.9,
                 dry=0.0, gain=3.0):
        self.l = _bind(_SIGS)
        radii = np.ascontiguousarray(radii, dtype=np.float64)
        self.h = self.l.orc_het_create(channels, order, _p(radii), thresh, ratio, width, stick_order, stick_rad, dry,
                                       gain)
        self.channels, self.order, self.width, self.stick_order = channels, max(1, order), width, max(1, stick_order)

    def __del__(self):
        try:
            self.l.orc_het_destroy(self.h)
        except Exception:
            pass

    def setup(self, order, radii):
        radii = np.ascontiguousarray(radii, dtype=np.float64)
        self.l.orc_het_setup(self.h, order, _p(radii))
        self.order = max(1, order)

    def freqmod(self, bank, index, hz):
        for i, f in zip(np.atleast_1d(index), np.atleast_1d(hz)):
            self.l.orc_het_freqmod(self.h, bank, int(i), float(f))

    def activate(self, bank, index, on=True):
        idx = np.ascontiguousarray(np.atleast_1d(index), dtype=np.int32)
        self.l.orc_het_activate(self.h, bank, idx.ctypes.data_as(C.POINTER(C.c_int)), idx.size, 1 if on else 0)

    def open(self, bank, on=True):
        self.activate(bank, np.arange(self.channels), on)

    def process(self, x):
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros(x.size)
        self.l.orc_het_process(self.h, _p(x), _p(y), x.size)
        return y

    def state(self, what):
        size = {2: 2 * self.order, 3: 1, 5: 2 * self.stick_order, 6: self.width}.get(what, 2)
        out = np.zeros(self.channels * size)
        self.l.orc_het_state(self.h, what, _p(out))
        return out
