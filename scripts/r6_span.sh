#!/bin/bash
# (diagnostic) setter launch time against the spread of the setters' bands (HZ_CHURN_SPAN)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/span
mkdir -p $D
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/span/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/span/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for sp in 16 4096; do for sk in 6 5; do
  HZ_CHURN_SPAN=$sp HZ_SETTER_SKIP=$sk timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D/p${sp}_$sk -o trace -- $D/churn $D > $D/p${sp}_$sk.log 2>&1 || exit 1
  echo "span $sp skip $sk: $(python3 scripts/churn_trace.py $D/p${sp}_$sk/trace_kernel_trace.csv | grep setter_kernel)"
done; done
