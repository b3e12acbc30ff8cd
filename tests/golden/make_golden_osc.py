"""Golden fixtures for Additive / Sinusoids (run: python tests/golden/make_golden_osc.py).

TEST INFRASTRUCTURE: written by the independent numpy restatement in spec_additive.py,
cross-checked against the closed-form phase of a settled oscillator
(phi(t) = phi0 + t f / SR: exact rotation) where the reference's dynamics reduce to it.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from spec_numpy import PI, SR  # noqa: E402
from spec_additive import additive_run, sinusoids_run  # noqa: E402

KIND = {"makenote": 0, "endnote": 1, "request": 2, "release": 3, "fundmod": 10, "decaymod": 11, "harmmod": 12}


def encode(events):
    t, k, a, b = [], [], [], []
    for (tt, kind, arg) in events:
        t.append(tt)
        k.append(KIND[kind])
        if isinstance(arg, tuple):
            a.append(float(arg[0]))
            b.append(float(arg[1]) if len(arg) > 1 else 0.0)
        else:
            a.append(float(arg))
            b.append(0.0)
    return dict(ev_t=np.array(t), ev_kind=np.array(k), ev_a=np.array(a), ev_b=np.array(b))


def main():
    out = {}
    # Additive: 4 voices x 8 overtones; a fifth note steals the nearest voice; releases
    ev = [(0, "makenote", (60, 1.0)), (0, "makenote", (67, 0.5)), (900, "makenote", (72, 0.8)),
          (1500, "endnote", (60,)), (2100, "makenote", (55, 0.7)), (2600, "makenote", (79, 0.9)),
          (3000, "release", (-1,)), (3500, "makenote", (61, 0.6))]
    n = 4096
    y = additive_run(4, 8, 0.75, 1.0, 0.1, ev, n)
    out["add_v4_o8"] = dict(V=4, O=8, decay=0.75, harm=1.0, k=0.1, n=n, y=y, **encode(ev))
    # inharmonic, slow attack
    ev = [(0, "makenote", (48, 1.0)), (10, "makenote", (52, 0.3)), (1111, "endnote", (48,))]
    y = additive_run(3, 5, 0.9, 1.3, 0.01, ev, 3000)
    out["add_v3_o5_inharm"] = dict(V=3, O=5, decay=0.9, harm=1.3, k=0.01, n=3000, y=y, **encode(ev))
    # Sinusoids: settled oscillators reduce to exact rotations -> closed-form check
    n = 4096
    y = sinusoids_run(220.0, 6, 0.7, 1.0, 2.0 / SR, [], n)
    t = np.arange(n)[:, None]
    i = np.arange(6)[None, :]
    norm = (1 - 0.7 ** 6) / (1 - 0.7)
    exact = np.sum(0.7 ** i * np.sin(2 * np.pi * (220.0 * (i + 1) / SR * t)) / norm, axis=1)
    assert np.max(np.abs(y - exact)) < 1e-9, np.max(np.abs(y - exact))
    out["sin_o6_static"] = dict(fund=220.0, O=6, decay=0.7, harm=1.0, k=2.0 / SR, n=n, y=y, **encode([]))
    ev = [(1000, "fundmod", 330.0), (2000, "decaymod", 0.5), (3000, "harmmod", 1.1)]
    y = sinusoids_run(220.0, 10, 0.8, 1.0, 2.0 / SR, ev, n)
    out["sin_o10_mods"] = dict(fund=220.0, O=10, decay=0.8, harm=1.0, k=2.0 / SR, n=n, y=y, **encode(ev))
    for name, d in out.items():
        np.savez(os.path.join(HERE, name + ".npz"), **d)
        print("wrote", name)


if __name__ == "__main__":
    main()
