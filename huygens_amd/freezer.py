"""Freezer<N> over the HIP engine (src/fourier.h:389-562, spectral freeze).

Freezer(N, laps, width): process(x, events) runs operator()(x[i]) per sample with
freeze() / unfreeze() calls (events (at, kind), kind 1 freeze / 0 unfreeze) made before
sample `at`.  The frame choice draws libc rand() like the reference (seed with srand)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, load

FRZ_EVENT = np.dtype([("at", np.int64), ("kind", np.int32), ("pad", np.int32)])


def _events(events):
    ev = list(events or ())
    a = np.zeros(len(ev), dtype=FRZ_EVENT)
    for i, (at, kind) in enumerate(ev):
        a[i]["at"], a[i]["kind"] = int(at), int(kind)
    return a


class Freezer:
    def __init__(self, N: int, laps: int, width: float = 1.0, device: int = 0):
        lib = load()
        h = C.c_void_p()
        check(lib.hz_frz_create(N, laps, float(width), device, C.byref(h)))
        self._h, self._lib, self.N = h, lib, N

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_frz_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def freeze(self):
        check(self._lib.hz_frz_freeze(self._h))

    def unfreeze(self):
        check(self._lib.hz_frz_unfreeze(self._h))

    def process(self, x, events=()):
        x = np.ascontiguousarray(x, dtype=np.float64)
        ev = _events(events)
        y = np.zeros(x.size)
        check(self._lib.hz_frz_process(self._h, dptr(x), dptr(y), x.size,
                                       C.c_void_p(ev.ctypes.data) if ev.size else None, ev.size))
        return y

    def process_device(self, in_ptr, out_ptr, n, events=()):
        ev = _events(events)
        check(self._lib.hz_frz_process_device(self._h, C.c_void_p(in_ptr), C.c_void_p(out_ptr), n,
                                              C.c_void_p(ev.ctypes.data) if ev.size else None, ev.size))

    def info(self):
        s, m, f = C.c_int(), C.c_int(), C.c_int()
        check(self._lib.hz_frz_info(self._h, C.byref(s), C.byref(m), C.byref(f)))
        return s.value, m.value, bool(f.value)

    def set_stream(self, stream_ptr):
        check(self._lib.hz_frz_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        check(self._lib.hz_frz_synchronize(self._h))

    def profile(self, enable: bool):
        """HIP-event timing of the output kernel's launches while enabled."""
        check(self._lib.hz_frz_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        ms, n = C.c_double(), C.c_long()
        check(self._lib.hz_frz_profile_read(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value
