"""(diagnostics) block calls on another handle while the per-sample server is resident: wall
time per call, with the server launched with a 20 ms idle exit (HZ_RT_IDLE_US)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["HZ_RT_IDLE_US"] = "20000"
from huygens_amd import Filterbank, rt_info  # noqa: E402
from golden.spec_numpy import resonant_coefficients, white_noise_f32  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
g, g2 = Filterbank(2, N), Filterbank(2, N)
fwd, back = resonant_coefficients(N, 0.99, 1.0)
for fb in (g, g2):
    for n in range(N):
        fb.coefficients(n, fwd[n], back[n])
    fb.boost(np.ones(N))
    fb.open()
x = white_noise_f32(4096, seed=2)
g2.process(x)
times, res = [], []
for i in range(30):
    g(0.1)
    g.tick()
    r0 = rt_info(0)
    t0 = time.perf_counter()
    g2.process(x)
    times.append(time.perf_counter() - t0)
    res.append(rt_info(0)[2])
print("N", N, "block call ms:", " ".join(f"{1e3 * t:.3f}" for t in times))
print("resident after:", res, "info", rt_info(0))
