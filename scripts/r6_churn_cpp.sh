#!/bin/bash
# Round 6: the C++ churn driver (tests/cpp/churn.cpp) alone, with host-time counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/churn_cpp
mkdir -p $D
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/churn_cpp/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/churn_cpp/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
timeout -k 10 120 $D/churn $D
