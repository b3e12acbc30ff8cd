"""Timing probe for the heterodyne chain kernel: channel-samples/s at a few bank sizes."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np
import torch

from huygens_amd import Heterodyne

for N, n in [(96, 48000), (16384, 16384), (131072, 16384), (262144, 8192)]:
    rng = np.random.default_rng(0)
    radii = np.zeros(2 * N)
    radii[0::2] = rng.uniform(0.95, 0.999, N)
    g = Heterodyne(N, 4, radii, width=2400, gain=3.0 / max(1, N // 96))
    fa = rng.uniform(40, 8000, N)
    g.freqmod(0, np.arange(N), fa)
    g.freqmod(1, np.arange(N), -2 * fa)
    g.open(0)
    g.open(1)
    x = torch.from_numpy(0.2 * rng.standard_normal(n)).cuda()
    y = torch.empty_like(x)
    g.set_stream(torch.cuda.current_stream().cuda_stream)
    g.process_device(x.data_ptr(), y.data_ptr(), n)   # warm
    torch.cuda.synchronize()
    g.profile(True)
    t = time.perf_counter()
    g.process_device(x.data_ptr(), y.data_ptr(), n)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    ms, launches, cs = g.profile_read()
    print(f"N={N} n={n}: chain {ms:.2f} ms over {launches} launches, wall {wall*1e3:.2f} ms, "
          f"{cs / (ms * 1e-3):.3e} channel-samples/s, ring {16 * cs / (ms * 1e-3) / 1e9:.0f} GB/s", flush=True)
    g.close()
