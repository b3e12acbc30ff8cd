"""Debug: where do GPU and restatement analysis phasors first differ?"""
import math
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np

from huygens_amd import Heterodyne
from oracle_het import OracleHet

N = 96
rng = np.random.default_rng(N)
radii = np.zeros(2 * N)
radii[0::2] = rng.uniform(0.95, 0.999, N)
fa = rng.uniform(40, 6000, N) * np.where(rng.random(N) < 0.5, -1, 1)
for order, width in [(4, 2400), (1, 48), (4, 48), (1, 2400)]:
    g = Heterodyne(N, order, radii, width=width)
    o = OracleHet(N, order, radii, width=width)
    for h in (g, o):
        h.freqmod(0, np.arange(N), fa)
        h.freqmod(1, np.arange(N), -2 * fa)
        h.open(0)
        h.open(1)
    x = 0.1 * np.random.default_rng(1).standard_normal(200)
    for t in range(200):
        g.process(x[t:t + 1])
        o.process(x[t:t + 1])
        a, b = g.state(0).reshape(N, 2), o.state(0).reshape(N, 2)
        bad = np.flatnonzero((a != b).any(1))
        if bad.size:
            i = bad[0]
            w = (math.cos(2 * 3.14159265359 * fa[i] / 48000), math.sin(2 * 3.14159265359 * fa[i] / 48000))
            print(f"order {order} width {width}: first diff at t={t}, channels {bad[:8]}, ch {i}: gpu {a[i].tolist()} "
                  f"orc {b[i].tolist()} w(py) {w}")
            break
    else:
        print(f"order {order} width {width}: analysis equal for 200 samples")
    for what in range(7):
        a, b = g.state(what), o.state(what)
        print("  state", what, "equal" if np.array_equal(a, b) else f"diff {np.max(np.abs(a - b)):.3e}")
