"""Streaming diagnostic: per-call time of 1024-sample process_device() calls for a tiny bank (host
and launch overhead) and for the C2 bank, plus the raw cost of an empty ctypes call."""
import ctypes
import sys
import time
import numpy as np
sys.path.insert(0, ".")
import torch
import bench
from huygens_amd import Filterbank

dev = torch.device("cuda", 0)
x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, 480000)).to(dev)
y = torch.empty_like(x)
B = 1024
for N in (16, 256, 4096):
    fwd, back = bench.c2_coefficients(N)
    fb = Filterbank(2, N, 0.1, 1.0, device=0)
    for n in range(N):
        fb.coefficients(n, fwd[n], back[n])
    fb.boost(np.ones(N))
    fb.open()
    fb.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    fb.process_device(x.data_ptr(), y.data_ptr(), 480000)   # converge
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(469):
            fb.process_device(x.data_ptr() + 8 * B * i, y.data_ptr() + 8 * B * i, B)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"N={N:5d} rep {rep}: {(t2 - t0) * 1e6 / 469:6.1f} us per block (host issue {(t1 - t0) * 1e6 / 469:6.1f} us), "
              f"path {fb.last_path()}")
    fb.close()
libc = ctypes.CDLL(None)
t0 = time.perf_counter()
for i in range(100000):
    libc.abs(1)
print(f"empty ctypes call: {(time.perf_counter() - t0) * 1e6 / 100000:.2f} us")
