#!/bin/bash
# Round 6: setter churn after the fused setter launch -- parity tests, the C++ churn driver, its kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/churn2
mkdir -p $D
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_fb_churn_gpu.py \
    tests/test_fb_stream_gpu.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/churn2/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/churn2/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
timeout -k 10 120 $D/churn $D && timeout -k 10 120 $D/churn $D &&
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o trace -- $D/churn $D > $D/prof.log 2>&1
tail -1 $D/prof.log
