#!/bin/bash
# (A/B) the setter launch whole against split in two (HZ_SETTER_SPLIT=1: taps + upkeep without LDS,
# then the column workgroups), alternating, with the launch trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/split
mkdir -p $D
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/split/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/split/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
HZ_SETTER_SPLIT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_fb_churn_gpu.py 2>&1 | tail -2
for sp in 0 1 0 1; do
  echo "split $sp: $(HZ_SETTER_SPLIT=$sp timeout -k 10 120 $D/churn $D)"
done
for sp in 0 1; do
  rm -f $D/t$sp.bin
  HZ_SETTER_SPLIT=$sp HZ_STREAM_TRACE=$D/t$sp.bin timeout -k 10 120 $D/churn $D > /dev/null && echo "trace split $sp" && OUTWG=64 python3 scripts/stream_trace.py $D/t$sp.bin | grep -E "span|upkeep|taps|columns"
done
