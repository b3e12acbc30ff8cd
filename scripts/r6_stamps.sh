#!/bin/bash
# (diagnostic) per-phase times of the setter launch's column workgroups (HZ_SETTER_STAMPS)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/stamps
mkdir -p $D
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/stamps/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/stamps/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
rm -f $D/trace*.bin; for sk in 0; do HZ_SETTER_SKIP=$sk HZ_STREAM_TRACE=$D/trace$sk.bin timeout -k 10 120 $D/churn $D && echo "skip $sk" && OUTWG=64 python3 scripts/stream_trace.py $D/trace$sk.bin; done
