"""Granulator<double> over the HIP engine (src/granulator.h:12-127).

Granulator(window=&hann, source=Buffer(buffer_size), realtime, polyphony=512): the handle
owns the source ring.  process(x, requests) runs the tests/granny.cpp:34-56 loop body per
sample -- source.write(x[i]); y[i] = granny(); requests made at i; source.tick();
granny.tick() -- and returns (y, voices).  request() between calls is the reference's
request() after the last sample's read: ticked=True when its tick has not happened yet
(operator(); request(); tick()), False after it.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, load

SR = 48000

# hz_grain_req {long at; double offset, size, speed, gain, pan;}
GRAIN_REQ = np.dtype([("at", np.int64), ("offset", np.float64), ("size", np.float64), ("speed", np.float64),
                      ("gain", np.float64), ("pan", np.float64)])


def _reqs(requests):
    """requests: GRAIN_REQ array or iterable of (at, offset, size, speed, gain, pan)."""
    if requests is None:
        return np.zeros(0, dtype=GRAIN_REQ)
    if isinstance(requests, np.ndarray) and requests.dtype == GRAIN_REQ:
        return np.ascontiguousarray(requests)
    return np.array([tuple(r) for r in requests], dtype=GRAIN_REQ)


class Granulator:
    def __init__(self, buffer_size: int = 3 * SR, polyphony: int = 512, device: int = 0):
        lib = load()
        h = C.c_void_p()
        check(lib.hz_gran_create(polyphony, buffer_size, device, C.byref(h)))
        self._h, self._lib, self.polyphony = h, lib, polyphony

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_gran_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def request(self, offset, size, speed, gain, pan=0.0, ticked=False) -> int:
        v = C.c_int()
        check(self._lib.hz_gran_request(self._h, float(offset), float(size), float(speed), float(gain), float(pan),
                                        1 if ticked else 0, C.byref(v)))
        return v.value

    def sample(self, x: float) -> float:
        """`source.write(x); y = granny(); granny.tick();` (tests/granny.cpp:36-56) for one sample,
        through the per-sample server (hz_gran_sample)"""
        y = C.c_double()
        check(self._lib.hz_gran_sample(self._h, float(x), C.byref(y)))
        return y.value

    def process(self, x, requests=None):
        x = np.ascontiguousarray(x, dtype=np.float64)
        r = _reqs(requests)
        y = np.zeros(x.size)
        voices = np.zeros(max(1, r.size), dtype=np.int32)
        check(self._lib.hz_gran_process(self._h, dptr(x), dptr(y), x.size, C.c_void_p(r.ctypes.data) if r.size else None,
                                        r.size, voices.ctypes.data_as(C.POINTER(C.c_int))))
        return y, voices[:r.size].copy()

    def process_device(self, in_ptr, out_ptr, n, requests=None):
        r = _reqs(requests)
        voices = np.zeros(max(1, r.size), dtype=np.int32)
        check(self._lib.hz_gran_process_device(self._h, C.c_void_p(in_ptr), C.c_void_p(out_ptr), n,
                                               C.c_void_p(r.ctypes.data) if r.size else None, r.size,
                                               voices.ctypes.data_as(C.POINTER(C.c_int))))
        return voices[:r.size].copy()

    def activity(self) -> int:
        a = C.c_uint()
        check(self._lib.hz_gran_activity(self._h, C.byref(a)))
        return a.value

    def idle(self) -> bool:   # granulator.h:106-109
        return self.activity() == 0

    def set_stream(self, stream_ptr):
        check(self._lib.hz_gran_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        check(self._lib.hz_gran_synchronize(self._h))

    def profile(self, enable: bool):
        check(self._lib.hz_gran_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        ms, la, gs = C.c_double(), C.c_long(), C.c_long()
        check(self._lib.hz_gran_profile_read(self._h, C.byref(ms), C.byref(la), C.byref(gs)))
        return ms.value, la.value, gs.value
