#!/bin/bash
# Round 5: the GPU suite (or a -k selection: SEL=...), one process, per-test time limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/${TAG:-tests}
mkdir -p "$OUT"
date
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=15 -k "$SEL" > "$OUT/pytest.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=25 > "$OUT/pytest.log" 2>&1
fi
rc=$?; grep -E "PASSED|FAILED|ERROR" "$OUT/pytest.log" | grep -E "FAILED|ERROR" | head -20; tail -30 "$OUT/pytest.log"; echo "pytest rc=$rc"
exit $rc
