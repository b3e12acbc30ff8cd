#!/bin/bash
# (diagnostic) the setter launch twice in a row (HZ_SETTER_TWICE=1): cold against warm span
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/twice
mkdir -p $D
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/twice/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/twice/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
rm -f $D/t.bin
HZ_SETTER_TWICE=1 HZ_STREAM_TRACE=$D/t.bin timeout -k 10 120 $D/churn $D > /dev/null || exit 1
python3 - <<'PY'
import numpy as np
raw = open("gpurun_out/r6/twice/t.bin", "rb").read()
rec = 8 + 1024 * 8
n = len(raw) // rec
prev = None
first, second = [], []
for i in range(n):
    k, wg = np.frombuffer(raw, dtype=np.int32, count=2, offset=i * rec)
    st = np.frombuffer(raw, dtype=np.uint64, count=1024, offset=i * rec + 8).astype(np.int64)
    span = (st[512:512 + wg].max() - st[:wg].min()) / 100.0
    if k == 2:
        (second if prev == 2 else first).append(span)
    prev = int(k)
print("setter launch span: first (cold) %.2f us, second (warm) %.2f us, n=%d" % (np.mean(first), np.mean(second), len(second)))
PY
