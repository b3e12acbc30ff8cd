"""Per-sample operator()+tick() rate of the Filterbank drop-in (C1: 128 bands, C2: 4096)
through the C ABI (ctypes), i.e. the path a demo's process() callback takes per sample."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from huygens_amd import Filterbank  # noqa: E402
from golden.spec_numpy import resonant_coefficients  # noqa: E402

for N in (128, 4096):
    fwd, back = resonant_coefficients(N, 0.999, 1.0)
    fb = Filterbank(2, N, 0.1, 1.0, device=0)
    for n in range(N):
        fb.coefficients(n, fwd[n], back[n])
    fb.boost(np.ones(N))
    fb.open()
    x = np.random.default_rng(1).uniform(-1, 1, 3000)
    for i in range(200):
        fb(x[i]); fb.tick()
    t0 = time.perf_counter()
    for i in range(200, 3000):
        fb(x[i]); fb.tick()
    dt = time.perf_counter() - t0
    print(f"N={N}: {2800 / dt:.0f} samples/s per-sample ({1e6 * dt / 2800:.1f} us/sample)", flush=True)
    fb.close()
