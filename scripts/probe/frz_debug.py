"""Freezer GPU vs oracle: first mismatching samples (diagnostic)."""
import sys
import numpy as np
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
from oracle_frz import OracleFreezer, libc_srand
from huygens_amd import Freezer

N, laps, width = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
rng = np.random.default_rng(N + laps)
t = np.arange(40000)
x = 0.3 * np.sin(2 * np.pi * 440 * t / 48000) + 0.05 * rng.standard_normal(t.size)
blocks = [(5000, [(0, 0), (3000, 1)]), (7000, [(2500, 0), (2501, 1), (6000, 1)]), (1, [(0, 0)]),
          (12000, [(4000, 1), (9000, 0)]), (15999, [])]
g, o = Freezer(N, laps, width), OracleFreezer(N, laps, width)
print("geometry", g.info(), o.stride, o.M, o.size)
ys = []
for who in (g, o):
    libc_srand(N)
    pos, out = 0, []
    for b, ev in blocks:
        out.append(who.process(x[pos:pos + b], ev))
        pos += b
    ys.append(np.concatenate(out))
d = np.abs(ys[0] - ys[1])
bad = np.flatnonzero(d > 1e-9 * np.abs(ys[1]).max())
print("peak", np.abs(ys[1]).max(), "nbad", bad.size, "first", bad[:20])
for i in bad[:8]:
    print(i, ys[0][i], ys[1][i])
