#!/bin/bash
# C2 with the stationary engine: bench (default engine choice) + rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c2resp}
mkdir -p "$OUT"
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1
rc=$?; tail -2 "$OUT/bench.log"; echo "bench rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
    python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-traffic --stream-blocks 0 --side-steps 0 > "$OUT/prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-4,7 "$f" | head -14
exit $rc
