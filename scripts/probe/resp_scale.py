"""Probe: the stationary engine's kernels against the call length (grid size), to tell per-workgroup
latency from throughput limits.  Run under rocprofv3 --kernel-trace; summarise with
scripts/kstats_grid.py.  C2 bank (4096 bands, O = 2), calls of n samples once stationary."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from golden.spec_numpy import resonant_coefficients  # noqa: E402
from huygens_amd import Filterbank  # noqa: E402
from huygens_amd._lib import HZ_FB_PATH_RESPONSE  # noqa: E402

import torch  # noqa: E402

N = 4096
fwd, back = resonant_coefficients(N, 0.999, 1.0)
g = Filterbank(2, N, 0.1, 1.0)
for n in range(N):
    g.coefficients(n, fwd[n], back[n])
g.boost(np.ones(N))
g.open()
rng = np.random.default_rng(0)
x = torch.tensor(rng.uniform(-1, 1, 480000), dtype=torch.float64, device="cuda")
y = torch.empty_like(x)
for _ in range(10):
    g.process_device(x.data_ptr(), y.data_ptr(), 480000)
assert g.last_path() == HZ_FB_PATH_RESPONSE, g.last_path()
for n in [int(v) for v in (sys.argv[1:] or ["32768", "65536", "131072", "262144", "480000"])]:
    for _ in range(20):
        g.process_device(x.data_ptr(), y.data_ptr(), n)
    g.synchronize()
    torch.cuda.synchronize()
    print("n", n, "path", g.last_path(), flush=True)
