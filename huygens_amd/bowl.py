"""Bowl<T> over the HIP engine (src/bowl.h:10-74): trigger(), fill(float*, bsize),
operator()()/tick() as render(n); T = double or float (dtype)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, load


class Bowl:
    def __init__(self, overtones: int, frequencies, amplitudes, decays, dtype=np.float64, device: int = 0):
        lib = load()
        f = np.ascontiguousarray(frequencies, dtype=np.float64)
        a = np.ascontiguousarray(amplitudes, dtype=np.float64)
        d = np.ascontiguousarray(decays, dtype=np.float64)
        count = min(len(f), len(a), len(d))
        h = C.c_void_p()
        is_float = 1 if np.dtype(dtype) == np.float32 else 0
        check(lib.hz_bowl_create(overtones, dptr(f), dptr(a), dptr(d), count, is_float, device, C.byref(h)))
        self._h, self._lib, self.dtype = h, lib, np.dtype(dtype)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_bowl_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def trigger(self):
        check(self._lib.hz_bowl_trigger(self._h))

    def fill(self, bsize: int) -> np.ndarray:
        """int fill(float* buffer, int bsize): float samples."""
        out = np.zeros(bsize, dtype=np.float32)
        if bsize:
            check(self._lib.hz_bowl_fill(self._h, out.ctypes.data_as(C.POINTER(C.c_float)), bsize))
        return out

    def fill_device(self, ptr: int, n: int):
        check(self._lib.hz_bowl_fill_device(self._h, C.c_void_p(ptr), n))

    def fill_delaybank(self, bank, buf_ptr: int, out_ptr: int, n: int, mix: bool = True):
        """`fill(buf, n); bank.process(buf, out, n)` on device buffers in one launch when the bank's
        taps allow it (hz_bowl_fill_delaybank), else the two block calls; both on one stream."""
        check(self._lib.hz_bowl_fill_delaybank(self._h, C.c_void_p(buf_ptr), bank._h, C.c_void_p(out_ptr), n,
                                               1 if mix else 0))

    def render(self, n: int) -> np.ndarray:
        out = np.zeros(n)
        if n:
            check(self._lib.hz_bowl_render(self._h, dptr(out), n))
        return out

    def phase(self) -> float:
        p = C.c_double()
        check(self._lib.hz_bowl_phase(self._h, C.byref(p)))
        return p.value

    def set_stream(self, stream_ptr: int | None):
        check(self._lib.hz_bowl_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def set_target_groups(self, groups: int):
        check(self._lib.hz_bowl_set_target_groups(self._h, groups))

    def profile(self, enable: bool):
        check(self._lib.hz_bowl_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        ms, c = C.c_double(), C.c_long()
        check(self._lib.hz_bowl_profile_read(self._h, C.byref(ms), C.byref(c)))
        return ms.value, c.value
