"""Additive<double> and Sinusoids<double> over the HIP engine.

Mirrors soundmath::Additive<T> (src/additive.h:11-71, note API from
src/minimizer.h:111-187; physics() is out of scope) and soundmath::Sinusoids<T>
(src/sinusoids.h:10-79), waveform cycle = sin(2 PI p).  fill(n) ==
n x {out[t] = operator()(); tick();} on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, load


class Additive:
    def __init__(self, voices: int, overtones: int, decay: float, harmonicity: float = 1.0, k: float = 0.1,
                 device: int = 0, shard: tuple[int, int] | None = None):
        lib = load()
        h = C.c_void_p()
        if shard is None:
            check(lib.hz_add_create(voices, overtones, decay, harmonicity, k, device, C.byref(h)))
        else:
            check(lib.hz_add_create_shard(voices, overtones, shard[0], shard[1], decay, harmonicity, k, device,
                                          C.byref(h)))
        self._h, self._lib = h, lib

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_add_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def request(self, fundamental: float, amplitude: float = 0.0) -> int:
        v = C.c_int()
        check(self._lib.hz_add_request(self._h, fundamental, amplitude, C.byref(v)))
        return v.value

    def release(self, voice: int):
        check(self._lib.hz_add_release(self._h, voice))

    def makenote(self, pitch: float, amplitude: float) -> int:
        v = C.c_int()
        check(self._lib.hz_add_makenote(self._h, pitch, amplitude, C.byref(v)))
        return v.value

    def endnote(self, pitch: float):
        check(self._lib.hz_add_endnote(self._h, pitch))

    def fill(self, n: int) -> np.ndarray:
        out = np.zeros(n)
        if n:
            check(self._lib.hz_add_fill(self._h, dptr(out), n))
        return out

    def fill_device(self, out_ptr: int, n: int):
        check(self._lib.hz_add_fill_device(self._h, C.c_void_p(out_ptr), n))

    def set_stream(self, stream_ptr: int | None):
        check(self._lib.hz_add_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def set_target_groups(self, groups: int):
        check(self._lib.hz_add_set_target_groups(self._h, groups))

    def profile(self, enable: bool):
        check(self._lib.hz_add_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        ms, c = C.c_double(), C.c_long()
        check(self._lib.hz_add_profile_read(self._h, C.byref(ms), C.byref(c)))
        return ms.value, c.value


class Sinusoids:
    def __init__(self, fundamental: float, overtones: int, decay: float, harmonicity: float = 1.0,
                 k: float = 2.0 / 48000, device: int = 0):
        lib = load()
        h = C.c_void_p()
        check(lib.hz_sin_create(fundamental, overtones, decay, harmonicity, k, device, C.byref(h)))
        self._h, self._lib = h, lib

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_sin_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fundmod(self, target: float):
        check(self._lib.hz_sin_fundmod(self._h, target))

    def decaymod(self, target: float):
        check(self._lib.hz_sin_decaymod(self._h, target))

    def harmmod(self, target: float):
        check(self._lib.hz_sin_harmmod(self._h, target))

    def fill(self, n: int) -> np.ndarray:
        out = np.zeros(n)
        if n:
            check(self._lib.hz_sin_fill(self._h, dptr(out), n))
        return out


def lookahead_info(bank) -> tuple[int, int, int]:
    """(speculative blocks rendered, rollbacks, block length) of an Additive's per-sample service."""
    b, r, L = C.c_long(), C.c_long(), C.c_long()
    check(bank._lib.hz_add_lookahead_info(bank._h, C.byref(b), C.byref(r), C.byref(L)))
    return b.value, r.value, L.value
