#!/bin/bash
# Stationary-engine iteration loop on the GPU box: its parity tests, a short C2 bench, kernel stats.
#   TAG=name [TESTS="tests/a.py tests/b.py"] [BENCH_ARGS=...] bash scripts/c2_check.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c2}
mkdir -p "$OUT"
TESTS=${TESTS-"tests/test_filterbank_resp_gpu.py tests/test_c2_pinned_gpu.py"}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
  [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-traffic --no-per-sample --side-steps 50 --stream-blocks 469 \
    ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; tail -c 3000 "$OUT/bench.log"; echo; echo "bench rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-traffic --no-per-sample --side-steps 0 \
    --stream-blocks 0 ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cut -d, -f1-4 "$f" | head -14
exit 0
