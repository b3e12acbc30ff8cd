"""ctypes binding of the Freezer restatement (oracle/hz_oracle_frz.c). TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle import D, I, L, PD, VP, _bind, _p

_SIGS = {
    "orc_frz_create": (VP, [I, I, D]),
    "orc_frz_destroy": (None, [VP]),
    "orc_frz_geometry": (I, [VP, C.POINTER(I), C.POINTER(I)]),
    "orc_frz_freeze": (None, [VP]),
    "orc_frz_unfreeze": (None, [VP]),
    "orc_frz_frozen": (I, [VP]),
    "orc_frz_sample": (D, [VP, D]),
    "orc_frz_process": (None, [VP, PD, PD, L, C.POINTER(L), C.POINTER(I), I]),
}


def libc_srand(seed):
    """Seed the process's libc rand() (the Freezer draws its frames with it)."""
    C.CDLL(None).srand(C.c_uint(seed))


class OracleFreezer:
    def __init__(self, N, laps, width=1.0):
        self.l = _bind(_SIGS)
        self.h = self.l.orc_frz_create(N, laps, width)
        s, m = C.c_int(), C.c_int()
        self.size = self.l.orc_frz_geometry(self.h, C.byref(s), C.byref(m))
        self.stride, self.M = s.value, m.value

    def __del__(self):
        try:
            self.l.orc_frz_destroy(self.h)
        except Exception:
            pass

    def freeze(self):
        self.l.orc_frz_freeze(self.h)

    def unfreeze(self):
        self.l.orc_frz_unfreeze(self.h)

    def sample(self, x):
        return self.l.orc_frz_sample(self.h, float(x))

    def process(self, x, events=()):
        """events: iterable of (at, kind) with kind 1 freeze / 0 unfreeze, at ascending."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        ev = list(events)
        at = np.ascontiguousarray([int(e[0]) for e in ev] or [0], dtype=np.int64)
        kind = np.ascontiguousarray([int(e[1]) for e in ev] or [0], dtype=np.int32)
        y = np.zeros(x.size)
        self.l.orc_frz_process(self.h, _p(x), _p(y), x.size, at.ctypes.data_as(C.POINTER(C.c_long)),
                               kind.ctypes.data_as(C.POINTER(C.c_int)), len(ev))
        return y
