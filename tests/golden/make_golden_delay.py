"""Golden fixtures for Delay<T> / Delaybank<T,N> (run: python tests/golden/make_golden_delay.py).

TEST INFRASTRUCTURE.  Independent pure-Python restatement of src/buffer.h:19-67 and
src/delay.h:21-97 with explicit uint32 index arithmetic and T = float64 / float32 scalars
(numpy scalar ops keep float32 results in float32).  Cases:
  dly_impulse   Delay<double>(3, 999): the tests/delay.cpp:41 tap pattern scaled to a
                1000-sample ring, impulse in -> echo positions (int) and values;
  dly_wrap_d    Delay<double>(4, 99): delays longer than the ring (250, 130, 1000): the
                uint32 index wraps, so the slot read is NOT (o - c) mod size;
  dly_wrap_f    the same in float, plus a delay 16777217 that float rounds to 2^24;
  dly_bank_f    Delaybank<float, 6>(3, 2000), mono noise input, per-line outputs + mixdown.
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
M32 = 0xFFFFFFFF


class Line:
    def __init__(self, S, time, T):
        self.T = T
        self.size = (time + 1) & M32 or 1
        self.inp = [T(0)] * self.size
        self.out = [T(0)] * self.size
        self.origin = 0
        self.fwd = [(0, T(0))] * S
        self.back = [(0, T(0))] * S

    def coefficients(self, fwd, back):
        S = len(self.fwd)
        self.fwd = [(t, self.T(g)) for t, g in fwd[:S]] + [(0, self.T(0))] * (S - min(S, len(fwd)))
        self.back = [((t, self.T(g)) if t != 0 else (0, self.T(0))) for t, g in back[:S]]
        self.back += [(0, self.T(0))] * (S - len(self.back))

    def read(self, data, position):
        T = self.T
        center = int(position)            # (int)position, position >= 0
        before = center + 1
        disp = position - T(center)
        i1 = ((self.origin - center + self.size) & M32) % self.size
        i2 = ((self.origin - before + self.size) & M32) % self.size
        return data[i1] * (T(1) - disp) + data[i2] * disp

    def __call__(self, x):
        T = self.T
        o = self.origin
        self.inp[o] = T(x)
        self.out[o] = T(0)
        for (dt, f), (et, b) in zip(self.fwd, self.back):
            v = f * self.read(self.inp, T(dt)) - b * self.read(self.out, T(et))
            self.out[o] = self.out[o] + v
        y = self.read(self.out, T(0))
        self.origin = (self.origin + 1) % self.size
        return y


def run_line(S, time, T, fwd, back, x):
    L = Line(S, time, T)
    L.coefficients(fwd, back)
    return np.array([L(v) for v in x], dtype=T), L.origin


def main():
    out = {}
    # 1. impulse echoes
    n = 3000
    x = np.zeros(n)
    x[0] = 1.0
    fwd, back = [(0, 1.0)], [(200, 0.5), (100, 0.5)]
    y, o = run_line(3, 999, np.float64, fwd, back, x)
    out["dly_impulse"] = dict(S=3, time=999, is_float=0, lines=1, x=x, y=y[None, :], origin=o,
                              ft=np.array([[t for t, _ in fwd]], np.uint32), fg=np.array([[g for _, g in fwd]]),
                              bt=np.array([[t for t, _ in back]], np.uint32), bg=np.array([[g for _, g in back]]),
                              echoes=np.flatnonzero(y).astype(np.int64))
    # 2./3. uint wrap
    rng = np.random.default_rng(11)
    for name, T, extra in [("dly_wrap_d", np.float64, []), ("dly_wrap_f", np.float32, [(16777217, 0.125)])]:
        n = 1200
        x = rng.standard_normal(n).astype(T)
        fwd = [(0, 1.0), (250, 0.25), (7, -0.5)] + extra
        back = [(130, 0.3), (1000, 0.2), (0, 0.9), (3, 0.1)]
        S = 4
        y, o = run_line(S, 99, T, fwd, back, x)
        ft = np.zeros((1, S), np.uint32); fg = np.zeros((1, S))
        for i, (t, g) in enumerate(fwd[:S]):
            ft[0, i], fg[0, i] = t, g
        bt = np.zeros((1, S), np.uint32); bg = np.zeros((1, S))
        for i, (t, g) in enumerate(back[:S]):
            bt[0, i], bg[0, i] = t, g
        out[name] = dict(S=S, time=99, is_float=int(T == np.float32), lines=1, x=x, y=y[None, :], origin=o,
                         ft=ft, fg=fg, bt=bt, bg=bg)
    # 4. float bank, mono input, mixdown
    N, S, time, n = 6, 3, 2000, 5000
    x = (0.1 * rng.standard_normal(n)).astype(np.float32)
    ft = np.zeros((N, S), np.uint32); fg = np.zeros((N, S))
    bt = np.zeros((N, S), np.uint32); bg = np.zeros((N, S))
    ys = []
    for k in range(N):
        fwd = [(0, 1.0), (37 * k + 5, 0.5)]
        back = [(400 + 37 * k, 0.5), (900 + 53 * k, 0.45)]
        y, o = run_line(S, time, np.float32, fwd, back, x)
        ys.append(y)
        for i, (t, g) in enumerate(fwd):
            ft[k, i], fg[k, i] = t, g
        for i, (t, g) in enumerate(back):
            bt[k, i], bg[k, i] = t, g
    Y = np.stack(ys)
    mix = np.zeros(n, np.float32)
    for t in range(n):
        s = np.float32(0)
        for k in range(N):
            s = s + Y[k, t]
        mix[t] = s / np.float32(N)
    out["dly_bank_f"] = dict(S=S, time=time, is_float=1, lines=N, x=x, y=Y, mix=mix, origin=o,
                             ft=ft, fg=fg, bt=bt, bg=bg)
    for name, d in out.items():
        np.savez(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name, {k: getattr(v, "shape", v) for k, v in d.items() if k in ("y", "origin")})


if __name__ == "__main__":
    main()
