"""ctypes binding of the Delay/Delaybank restatement (oracle/hz_oracle_dly.c). TEST INFRASTRUCTURE."""
from __future__ import annotations

import ctypes as C

import numpy as np

from oracle import D, I, L, PD, VP, _bind, _p

UP = C.POINTER(C.c_uint)
_SIGS = {
    "orc_dly_create": (VP, [I, C.c_uint, C.c_uint, I]),
    "orc_dly_destroy": (None, [VP]),
    "orc_dly_coefficients": (None, [VP, I, UP, PD, I, UP, PD, I]),
    "orc_dly_modulate_forward": (None, [VP, I, C.c_uint, C.c_uint, D]),
    "orc_dly_modulate_back": (None, [VP, I, C.c_uint, C.c_uint, D]),
    "orc_dly_process": (None, [VP, VP, VP, L, I, I]),
    "orc_dly_origin": (C.c_uint, [VP]),
    "orc_dly_tick": (None, [VP, C.c_ulong]),
}


class OracleDelaybank:
    def __init__(self, lines, sparsity, time, dtype=np.float64):
        self.l = _bind(_SIGS)
        self.dtype = np.dtype(dtype)
        self.lines = lines
        self.h = self.l.orc_dly_create(lines, sparsity, time, 1 if self.dtype == np.float32 else 0)

    def __del__(self):
        try:
            self.l.orc_dly_destroy(self.h)
        except Exception:
            pass

    def coefficients(self, line, forward, back):
        ft = np.ascontiguousarray([int(t) for t, _ in forward], dtype=np.uint32)
        fg = np.ascontiguousarray([float(g) for _, g in forward], dtype=np.float64)
        bt = np.ascontiguousarray([int(t) for t, _ in back], dtype=np.uint32)
        bg = np.ascontiguousarray([float(g) for _, g in back], dtype=np.float64)
        self.l.orc_dly_coefficients(self.h, line, ft.ctypes.data_as(UP), _p(fg), len(ft),
                                    bt.ctypes.data_as(UP), _p(bg), len(bt))

    def modulate_forward(self, line, n, tap):
        self.l.orc_dly_modulate_forward(self.h, line, n, int(tap[0]), float(tap[1]))

    def modulate_back(self, line, n, tap):
        self.l.orc_dly_modulate_back(self.h, line, n, int(tap[0]), float(tap[1]))

    def process(self, x, mix=False):
        x = np.ascontiguousarray(x, dtype=self.dtype)
        per_line = x.ndim == 2
        n = x.shape[-1]
        out = np.zeros(n if mix else (self.lines, n), dtype=self.dtype)
        self.l.orc_dly_process(self.h, C.c_void_p(x.ctypes.data), C.c_void_p(out.ctypes.data), n,
                               1 if per_line else 0, 1 if mix else 0)
        return out

    def origin(self):
        return self.l.orc_dly_origin(self.h)

    def tick(self, count=1):
        """tick() without operator() (delay.h:92-97): origins move, nothing written"""
        self.l.orc_dly_tick(self.h, count)


def taps_of(g, line):
    """(forward, back) pair lists of one line from a golden fixture."""
    fwd = [(int(t), float(v)) for t, v in zip(g["ft"][line], g["fg"][line])]
    back = [(int(t), float(v)) for t, v in zip(g["bt"][line], g["bg"][line])]
    return fwd, back


def bank_from_golden(cls, g):
    dt = np.float32 if int(g["is_float"]) else np.float64
    b = cls(int(g["lines"]), int(g["S"]), int(g["time"]), dt)
    for k in range(int(g["lines"])):
        b.coefficients(k, *taps_of(g, k))
    return b
