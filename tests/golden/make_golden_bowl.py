"""Golden fixtures for Bowl<T> (run: python tests/golden/make_golden_bowl.py).

TEST INFRASTRUCTURE.  Independent numpy restatement of src/bowl.h:50-63:
  T = double: s(n) = sum_i a_i E^(-d_i n/SR) sin(2 PI f_i n / SR)   (vectorised, float64)
  T = float : the mixed-precision reference -- p = f*n/SR and x = -d*n/SR in float32,
              pow(E, x) and sin(2 PI p) in float64, the wave value rounded to float32, the
              running sum rounded to float32 after every mode (bowl.h:54-59).
Synthetic models in the ranges of tests/bowl.cpp:45-47 (seeded; the reference's own
303-mode data is not copied).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from spec_numpy import E, PI, SR  # noqa: E402


def bowl_model(M, seed):
    rng = np.random.default_rng(seed)
    f = np.exp(rng.uniform(np.log(20.0), np.log(16000.0), M))
    a = rng.uniform(1e-4, 5e-2, M)
    d = rng.uniform(0.05, 15.0, M)
    return f, a, d


def bowl_double(f, a, d, n, n0=0):
    t = (n0 + np.arange(n, dtype=np.float64))[:, None]
    return np.sum(a[None, :] * np.power(E, -d[None, :] * t / SR) * np.sin(2 * PI * (f[None, :] * t / SR)), axis=1)


def bowl_float(f, a, d, n, n0=0):
    f32, a32, d32 = f.astype(np.float32), a.astype(np.float32), d.astype(np.float32)
    ph = (n0 + np.arange(n)).astype(np.float32)
    sr = np.float32(SR)
    s = np.zeros(n, dtype=np.float32)
    for i in range(len(f)):
        x = (-d32[i] * ph) / sr                     # float32
        p = (f32[i] * ph) / sr                      # float32
        wv = np.sin(2 * PI * p.astype(np.float64)).astype(np.float32)
        term = np.float64(a32[i]) * np.power(E, x.astype(np.float64)) * wv.astype(np.float64)
        s = (s.astype(np.float64) + term).astype(np.float32)
    return s


def main():
    out = {}
    for name, M, seed, n in [("bowl_m32", 32, 5, 4096), ("bowl_m7", 7, 6, 3000)]:
        f, a, d = bowl_model(M, seed)
        yd = bowl_double(f, a, d, n)
        yf = bowl_float(f, a, d, n)
        out[name] = dict(M=M, f=f, a=a, d=d, n=n, y_double=yd, y_float=yf)
    for name, dd in out.items():
        np.savez(os.path.join(HERE, name + ".npz"), **dd)
        print("wrote", name)


if __name__ == "__main__":
    main()
