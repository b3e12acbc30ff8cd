"""ctypes binding of the Granulator restatement (oracle/hz_oracle_gran.c). TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle import D, I, L, PD, VP, _bind, _p

_SIGS = {
    "orc_gran_create": (VP, [C.c_uint, C.c_uint]),
    "orc_gran_destroy": (None, [VP]),
    "orc_gran_request": (I, [VP, D, D, D, D, D]),
    "orc_gran_write": (None, [VP, D]),
    "orc_gran_sample": (D, [VP]),
    "orc_gran_tick": (None, [VP]),
    "orc_gran_activity": (C.c_uint, [VP]),
    "orc_gran_process": (None, [VP, PD, PD, L, C.POINTER(L), PD, I, C.POINTER(I)]),
}


class OracleGranulator:
    def __init__(self, buffer_size, polyphony=512):
        self.l = _bind(_SIGS)
        self.h = self.l.orc_gran_create(polyphony, buffer_size)

    def __del__(self):
        try:
            self.l.orc_gran_destroy(self.h)
        except Exception:
            pass

    def request(self, offset, size, speed, gain, pan=0.0):
        return self.l.orc_gran_request(self.h, offset, size, speed, gain, pan)

    def write(self, x):
        self.l.orc_gran_write(self.h, x)

    def sample(self):
        return self.l.orc_gran_sample(self.h)

    def tick(self):
        self.l.orc_gran_tick(self.h)

    def activity(self):
        return self.l.orc_gran_activity(self.h)

    def process(self, x, requests=()):
        """requests: iterable of (at, offset, size, speed, gain, pan), at ascending."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        reqs = list(requests)
        at = np.ascontiguousarray([int(r[0]) for r in reqs] or [0], dtype=np.int64)
        par = np.ascontiguousarray([float(v) for r in reqs for v in r[1:6]] or [0.0], dtype=np.float64)
        voices = np.zeros(max(1, len(reqs)), dtype=np.int32)
        y = np.zeros(x.size)
        self.l.orc_gran_process(self.h, _p(x), _p(y), x.size, at.ctypes.data_as(C.POINTER(C.c_long)), _p(par),
                                len(reqs), voices.ctypes.data_as(C.POINTER(C.c_int)))
        return y, voices[:len(reqs)].copy()
