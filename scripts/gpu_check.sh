#!/bin/bash
# GPU session used through gpurun: tests -> smoke -> bench -> rocprofv3 stats.
# Stops at the first crash/timeout (exit >= 124 or signals); ordinary pytest
# failures (exit 1) are logged and the measurement still runs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1) return 1;; *) return 0;; esac; }

echo "== pytest -m gpu" ; date
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
if fatal $rc; then echo "stop: pytest crashed ($rc)"; exit $rc; fi

echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; cat "$OUT/smoke.log" | tail -3; echo "smoke rc=$rc"
if fatal $rc; then exit $rc; fi

echo "== bench"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; tail -3 "$OUT/bench.log"; echo "bench rc=$rc"
if fatal $rc; then exit $rc; fi

if [ -n "${PROFILE-1}" ]; then
  echo "== rocprofv3 kernel trace"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
      python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 > "$OUT/prof.log" 2>&1
  rc=$?; tail -3 "$OUT/prof.log"; echo "rocprof rc=$rc"
  find "$OUT/prof" -name "*stats*" | head
fi
exit 0
