#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/many
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_rt_server_gpu.py tests/test_filterbank_rt_gpu.py -x -v -s --timeout 300 \
   --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "sample_many|interleaved|PASSED|FAILED|^E " "$OUT/pytest.log" | head -40; echo "rc=$rc"; exit $rc
