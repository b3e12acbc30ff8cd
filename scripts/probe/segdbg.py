import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from huygens_amd import Filterbank
R = 0.9999
rng = np.random.default_rng(31)
x = rng.uniform(-1, 1, 200_000).astype(np.float32).astype(np.float64)[:4096]
np.save(os.path.join(ROOT, "gpurun_out", "segdbg_x.npy"), x)
g = Filterbank(2, 1, 1.0, 1.0)
g.coefficients(0, [1.0, 0.0, 0.0], [2 * R, R * R])
g.boost(np.ones(1))
g.open()
g.set_path(1)
y = g.process(x)
np.save(os.path.join(ROOT, "gpurun_out", "segdbg_y.npy"), y)
