"""ctypes binding of the Bowl<T> restatement (oracle/hz_oracle_bowl.c). TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle import D, I, L, PD, VP, _bind, _p

_SIGS = {
    "orc_bowl_create": (VP, [I, PD, PD, PD, I, I]),
    "orc_bowl_destroy": (None, [VP]),
    "orc_bowl_trigger": (None, [VP]),
    "orc_bowl_seek": (None, [VP, L]),
    "orc_bowl_fill": (I, [VP, C.POINTER(C.c_float), L]),
    "orc_bowl_render": (None, [VP, PD, L]),
}


class OracleBowl:
    def __init__(self, overtones, f, a, d, dtype=np.float64):
        self.l = _bind(_SIGS)
        f, a, d = (np.ascontiguousarray(v, dtype=np.float64) for v in (f, a, d))
        self._keep = (f, a, d)
        self.h = self.l.orc_bowl_create(overtones, _p(f), _p(a), _p(d), min(len(f), len(a), len(d)),
                                        1 if np.dtype(dtype) == np.float32 else 0)

    def __del__(self):
        try:
            self.l.orc_bowl_destroy(self.h)
        except Exception:
            pass

    def trigger(self):
        self.l.orc_bowl_trigger(self.h)

    def seek(self, ticks):
        """the state after trigger() and `ticks` samples (the phase counter)"""
        self.l.orc_bowl_seek(self.h, int(ticks))

    def fill(self, n):
        out = np.zeros(n, dtype=np.float32)
        self.l.orc_bowl_fill(self.h, out.ctypes.data_as(C.POINTER(C.c_float)), n)
        return out

    def render(self, n):
        out = np.zeros(n)
        self.l.orc_bowl_render(self.h, _p(out), n)
        return out
