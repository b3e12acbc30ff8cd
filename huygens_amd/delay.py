"""Delay<T> and Delaybank<T,N> over the HIP engine.

Delay<T> (src/delay.h:10-108, rings of src/buffer.h:9-86): Delay(sparsity, time),
coefficients(forward, back) with (uint time, T gain) pairs, modulate_forward/back,
operator()(x)/tick() -- here process(x) over a block.  Delaybank is N independent lines
(the reference's src/delaybank.h is a stub; SURVEY.md a21 gives the definition).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, dptr, load


def _taps(pairs):
    t = np.ascontiguousarray([int(p[0]) for p in pairs], dtype=np.uint32)
    g = np.ascontiguousarray([float(p[1]) for p in pairs], dtype=np.float64)
    return t, g


class Delaybank:
    def __init__(self, lines: int, sparsity: int, time: int, dtype=np.float64, device: int = 0):
        lib = load()
        h = C.c_void_p()
        self.dtype = np.dtype(dtype)
        check(lib.hz_dly_create(lines, sparsity, time, 1 if self.dtype == np.float32 else 0, device, C.byref(h)))
        self._h, self._lib, self.lines = h, lib, lines

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hz_dly_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def coefficients(self, line: int, forward, back):
        ft, fg = _taps(forward)
        bt, bg = _taps(back)
        up = C.POINTER(C.c_uint)
        check(self._lib.hz_dly_coefficients(self._h, line, ft.ctypes.data_as(up), dptr(fg), len(ft),
                                            bt.ctypes.data_as(up), dptr(bg), len(bt)))

    def modulate_forward(self, line: int, n: int, tap):
        check(self._lib.hz_dly_modulate_forward(self._h, line, n, int(tap[0]), float(tap[1])))

    def modulate_back(self, line: int, n: int, tap):
        check(self._lib.hz_dly_modulate_back(self._h, line, n, int(tap[0]), float(tap[1])))

    def process(self, x, mix: bool = False) -> np.ndarray:
        """x: mono [n] or per-line [lines, n] (T).  Returns [lines, n], or the mixdown [n]."""
        x = np.ascontiguousarray(x, dtype=self.dtype)
        per_line = x.ndim == 2
        if per_line and x.shape[0] != self.lines:
            raise ValueError("per-line input must have one row per line")
        n = x.shape[-1]
        out = np.zeros(n if mix else (self.lines, n), dtype=self.dtype)
        if n:
            check(self._lib.hz_dly_process(self._h, C.c_void_p(x.ctypes.data), C.c_void_p(out.ctypes.data), n,
                                           1 if per_line else 0, 1 if mix else 0))
        return out

    def sample(self, x) -> np.ndarray:
        """One sample of every line, `y_k = line_k(x); tick();` (delay.h:71-97), through the
        per-sample server (hz_dly_sample): x a scalar (mono) or [lines] (T); -> [lines]."""
        xa = np.ascontiguousarray(np.atleast_1d(x), dtype=self.dtype)
        if xa.size not in (1, self.lines):
            raise ValueError("sample: one input or one per line")
        per_line = xa.size == self.lines and self.lines > 1
        out = np.zeros(self.lines, dtype=self.dtype)
        check(self._lib.hz_dly_sample(self._h, C.c_void_p(xa.ctypes.data), C.c_void_p(out.ctypes.data),
                                      1 if per_line else 0))
        return out

    def process_device(self, in_ptr: int, out_ptr: int, n: int, per_line: bool = False, mix: bool = False):
        check(self._lib.hz_dly_process_device(self._h, C.c_void_p(in_ptr), C.c_void_p(out_ptr), n,
                                              1 if per_line else 0, 1 if mix else 0))

    def tick(self, count: int = 1):
        """tick() without operator() (delay.h:92-97), count times: both rings' origins move and
        no slot is written (hz_dly_tick)."""
        check(self._lib.hz_dly_tick(self._h, int(count)))

    def origin(self) -> int:
        o = C.c_uint()
        check(self._lib.hz_dly_origin(self._h, C.byref(o)))
        return o.value

    def info(self):
        c, s = C.c_long(), C.c_uint()
        check(self._lib.hz_dly_info(self._h, C.byref(c), C.byref(s)))
        return c.value, s.value

    def set_split(self, mode: int):
        check(self._lib.hz_dly_set_split(self._h, mode))

    def set_stream(self, stream_ptr: int | None):
        check(self._lib.hz_dly_set_stream(self._h, C.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        check(self._lib.hz_dly_synchronize(self._h))

    def set_target_groups(self, groups: int):
        check(self._lib.hz_dly_set_target_groups(self._h, groups))

    def profile(self, enable: bool):
        check(self._lib.hz_dly_profile(self._h, 1 if enable else 0))

    def profile_read(self):
        ms, c = C.c_double(), C.c_long()
        check(self._lib.hz_dly_profile_read(self._h, C.byref(ms), C.byref(c)))
        return ms.value, c.value


class Delay(Delaybank):
    """Delay<T>(sparsity, time): the one-line bank."""

    def __init__(self, sparsity: int, time: int, dtype=np.float64, device: int = 0):
        super().__init__(1, sparsity, time, dtype, device)
        # operator()'s input and output as preallocated C scalars (no arrays per sample)
        ct = C.c_float if self.dtype == np.float32 else C.c_double
        self._cx, self._cy = ct(), ct()
        self._px, self._py = C.c_void_p(C.addressof(self._cx)), C.c_void_p(C.addressof(self._cy))

    def coefficients(self, forward, back):  # noqa: D102
        super().coefficients(0, forward, back)

    def modulate_forward(self, n: int, tap):  # noqa: D102
        super().modulate_forward(0, n, tap)

    def modulate_back(self, n: int, tap):  # noqa: D102
        super().modulate_back(0, n, tap)

    def process(self, x) -> np.ndarray:  # noqa: D102
        return super().process(np.asarray(x).reshape(-1))[0]

    def __call__(self, x) -> float:
        """`y = delay(x); delay.tick();` (tests/delay.cpp:22-27) through the per-sample server"""
        self._cx.value = x   # (c_float: rounded to T as the array path's cast)
        check(self._lib.hz_dly_sample(self._h, self._px, self._py, 0))
        return float(self._cy.value)
