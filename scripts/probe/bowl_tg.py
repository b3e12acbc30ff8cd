"""Streamed Bowl<float>(2048) fill(1024) x 469: time per block vs target_groups (mode groups
per short call: fewer groups = more modes per wave and fewer slab rows to reduce)."""
import sys, time
import numpy as np
import torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from huygens_amd import Bowl
from bench_rows import c5_model

M, B, NB = 2048, 1024, 469
dev = torch.device("cuda", 0)
f, a, d = c5_model(M)
buf = torch.empty(NB * B, dtype=torch.float32, device=dev)
for tg in (256, 128, 64, 32, 16, 256):
    bowl = Bowl(M, f, a, d, np.float32)
    bowl.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    bowl.set_target_groups(tg)
    for i in range(NB):
        bowl.fill_device(buf.data_ptr() + 4 * B * i, B)
    torch.cuda.synchronize(dev)
    bowl.trigger()
    t0 = time.perf_counter()
    for r in range(3):
        bowl.trigger()
        for i in range(NB):
            bowl.fill_device(buf.data_ptr() + 4 * B * i, B)
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / 3
    print(f"target_groups {tg}: {1e6 * dt / NB:.2f} us per block", flush=True)
