"""Round 6: the high-Q C2 variant (R = 0.9999, horizon 507,904) on 480,000-sample calls -- ms per
call and the three launches' event times -- for A/B of the long-horizon MAC (HZ_MACC_BINS)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from huygens_amd import Filterbank  # noqa: E402
from huygens_amd._lib import HZ_FB_PATH_RESPONSE  # noqa: E402

S, N = 480000, 4096
fq, bq = bench.c2_coefficients(R=0.9999)
hq = Filterbank(2, N, 0.1, 1.0)
for n in range(N):
    hq.coefficients(n, fq[n], bq[n])
hq.boost(np.ones(N))
hq.open()
st = torch.cuda.current_stream()
hq.set_stream(st.cuda_stream)
x = torch.from_numpy(np.random.default_rng(1).uniform(-1, 1, S)).cuda()
y = torch.empty_like(x)
for _ in range(6):
    hq.process_device(x.data_ptr(), y.data_ptr(), S)
    if hq.last_path() == HZ_FB_PATH_RESPONSE:
        break
for _ in range(3):
    hq.process_device(x.data_ptr(), y.data_ptr(), S)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    hq.process_device(x.data_ptr(), y.data_ptr(), S)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
hq.profile(True)
for _ in range(5):
    hq.process_device(x.data_ptr(), y.data_ptr(), S)
torch.cuda.synchronize()
f, m, i, nl = hq.profile_read()
print(json.dumps({"tag": sys.argv[1] if len(sys.argv) > 1 else "", "ms_per_call": 1e3 * dt, "path": hq.last_path(),
                  "modal": hq.modal_info(), "fwd_ms": f / nl, "mac_ms": m / nl, "inv_ms": i / nl}))
