"""C2 streaming diagnostic: 469 process() calls of 1024 samples, timed; run under rocprofv3."""
import sys
import time
import numpy as np
sys.path.insert(0, ".")
import torch
import bench
from huygens_amd import Filterbank

dev = torch.device("cuda", 0)
fwd, back = bench.c2_coefficients()
fb = Filterbank(2, bench.N_BANDS, 0.1, 1.0, device=0)
for n in range(bench.N_BANDS):
    fb.coefficients(n, fwd[n], back[n])
fb.boost(np.ones(bench.N_BANDS))
fb.open()
fb.set_stream(torch.cuda.current_stream(dev).cuda_stream)
x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, 480000)).to(dev)
y = torch.empty_like(x)
B = 1024
fb.process_device(x.data_ptr(), y.data_ptr(), 480000)   # converge + warm
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(469):
        fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"rep {rep}: {dt * 1e6 / 469:.1f} us per 1024-sample block, {4096 * B * 469 / dt:.3e} band-samples/s")
