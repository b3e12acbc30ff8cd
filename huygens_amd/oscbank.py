"""Oscbank<double,N> over the HIP engine.

Mirrors soundmath::Oscbank<T,N> (src/oscbank.h:15-97) and its active-set protocol
(src/multichannel.h:16-159): freqmod, activate/deactivate/open/close, operator()()
(the N phasors), mixdown(), tick(), plus the block method fill(n) ==
n x {mix[t] = mixdown(); per_band[t] = operator()(); tick();} on the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, load


class Oscbank:
    def __init__(self, N: int, k: float = 2.0 / 48000, device: int = 0, shard: tuple[int, int] | None = None):
        lib = load()
        h = C.c_void_p()
        if shard is None:
            check(lib.hz_osc_create(N, k, device, C.byref(h)))
        else:
            check(lib.hz_osc_create_shard(N, shard[0], shard[1], k, device, C.byref(h)))
        self._h, self._lib, self.N, self.shard = h, lib, N, shard
        self.local_N = N if shard is None else shard[1]

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_osc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def freqmod(self, index: int, hz: float):
        check(self._lib.hz_osc_freqmod(self._h, int(index), float(hz)))

    def activate(self, indices):
        a = np.ascontiguousarray(indices, dtype=np.int32)
        check(self._lib.hz_osc_activate(self._h, a.ctypes.data_as(C.POINTER(C.c_int)), len(a)))

    def deactivate(self, indices):
        a = np.ascontiguousarray(indices, dtype=np.int32)
        check(self._lib.hz_osc_deactivate(self._h, a.ctypes.data_as(C.POINTER(C.c_int)), len(a)))

    def open(self):
        check(self._lib.hz_osc_open(self._h))

    def close_all(self):
        """Multichannel::close() (named close_all: close() releases the handle)."""
        check(self._lib.hz_osc_close(self._h))

    def active_count(self) -> int:
        c = C.c_int()
        check(self._lib.hz_osc_active_count(self._h, C.byref(c)))
        return c.value

    def fill(self, n: int, per_band: bool = False):
        """-> mix [n] complex (and per-band phasors [n, N] complex)."""
        mix = np.zeros(2 * n)
        pb = np.zeros(2 * n * self.local_N) if per_band else None
        if n:
            check(self._lib.hz_osc_fill(self._h, dptr(mix), dptr(pb) if pb is not None else None, n))
        m = mix.view(np.complex128)
        if per_band:
            return m, pb.view(np.complex128).reshape(n, self.local_N)
        return m

    def fill_device(self, mix_ptr: int, per_band_ptr: int | None, n: int):
        check(self._lib.hz_osc_fill_device(self._h, C.c_void_p(mix_ptr), C.c_void_p(per_band_ptr or 0), n))

    def phases(self) -> np.ndarray:
        z = np.zeros(2 * self.local_N)
        check(self._lib.hz_osc_phases(self._h, dptr(z)))
        return z.view(np.complex128)

    def set_phases(self, z):
        zz = np.ascontiguousarray(np.asarray(z, dtype=np.complex128)).view(np.float64)
        check(self._lib.hz_osc_set_phases(self._h, dptr(zz)))

    def set_stream(self, stream_ptr: int | None):
        check(self._lib.hz_osc_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        check(self._lib.hz_osc_synchronize(self._h))

    def set_target_groups(self, groups: int):
        check(self._lib.hz_osc_set_target_groups(self._h, groups))

    def profile(self, enable: bool):
        check(self._lib.hz_osc_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        ms, c = C.c_double(), C.c_long()
        check(self._lib.hz_osc_profile_read(self._h, C.byref(ms), C.byref(c)))
        return ms.value, c.value

    # ---- per-sample operator API (src/oscbank.h:59-90): served from a speculative block ----
    def mixdown(self) -> complex:
        """mixdown() of the current phasors (no tick)."""
        m = np.zeros(2)
        check(self._lib.hz_osc_mixdown(self._h, dptr(m)))
        return complex(m[0], m[1])

    def tick(self):
        """tick(): one sample."""
        check(self._lib.hz_osc_fill(self._h, None, None, 1))
