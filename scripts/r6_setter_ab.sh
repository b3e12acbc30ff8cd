#!/bin/bash
# (diagnostic) the setter launch with roles skipped: HZ_SETTER_SKIP = 1 columns, 2 taps, 4 upkeep
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/setter_ab
mkdir -p $D
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/setter_ab/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/setter_ab/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for sk in ${SKIPS:-0 1 2 4 3 5 6 7}; do
  HZ_SETTER_SKIP=$sk timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $D/p$sk -o trace -- $D/churn $D > $D/p$sk.log 2>&1 || exit 1
  echo "skip $sk: $(tail -1 $D/p$sk.log | cut -c1-80)"
  python3 scripts/churn_trace.py $D/p$sk/trace_kernel_trace.csv | grep -E "setter|span"
done
