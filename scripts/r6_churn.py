"""Round 6: setter churn on the C2 bank -- 1024-sample streamed calls with mix() on 9 random bands
every 4800 samples -- for rocprofv3 kernel traces (which launches a churned block costs)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from huygens_amd import Filterbank  # noqa: E402

N, S, B = 4096, 480000, 1024
fwd, back = bench.c2_coefficients()
fb = Filterbank(2, N, 0.1, 1.0)
for n in range(N):
    fb.coefficients(n, fwd[n], back[n])
fb.boost(np.ones(N))
fb.open()
fb.set_stream(torch.cuda.current_stream().cuda_stream)
x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, S)).cuda()
y = torch.empty_like(x)
for _ in range(3):
    fb.process_device(x.data_ptr(), y.data_ptr(), S)
rng = np.random.default_rng(17)
nb = S // B
for label, churn in (("converged", False), ("churn", True)):
    for i in range(64):
        fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(nb):
        if churn and (i * B) // 4800 != ((i - 1) * B) // 4800:
            for b, v in zip(rng.choice(N, 9, replace=False), rng.uniform(0.5, 1.5, 9)):
                fb.mix(int(b), float(v))
        fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
    torch.cuda.synchronize()
    print(label, "us per block %.2f" % (1e6 * (time.perf_counter() - t0) / nb), "last path", fb.last_path(), flush=True)
