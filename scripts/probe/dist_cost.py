"""General-engine step time with and without a distortion functor (C2 bank, 10 s call)."""
import time, sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from huygens_amd import Filterbank
from huygens_amd._lib import HZ_FB_PATH_GENERAL, HZ_DIST_SOFTCLIP, HZ_DIST_SATURATE, HZ_DIST_LIMITER, HZ_DIST_NONE
import bench

fwd, back = bench.c2_coefficients()
S = 480000
x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, S)).cuda()
y = torch.empty_like(x)
for dist, par in ((HZ_DIST_NONE, 0.0), (HZ_DIST_SOFTCLIP, 0.5), (HZ_DIST_SATURATE, 0.0), (HZ_DIST_LIMITER, 0.0)):
    fb = Filterbank(2, 4096, 0.1, 1.0)
    for n in range(4096):
        fb.coefficients(n, fwd[n], back[n])
    fb.boost(np.ones(4096))
    fb.open()
    fb.set_path(HZ_FB_PATH_GENERAL)
    if dist != HZ_DIST_NONE:
        fb.distortion(dist, par)
    for _ in range(3):
        fb.process_device(x.data_ptr(), y.data_ptr(), S)
    fb.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        fb.process_device(x.data_ptr(), y.data_ptr(), S)
    fb.synchronize()
    print("dist %d: %.3f ms per 10 s step" % (dist, (time.perf_counter() - t0) / 10 * 1e3), flush=True)
