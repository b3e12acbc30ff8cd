#!/bin/bash
# Round 5 (session 2): secondary rows with PMC evidence (traffic + executed flops per dominant
# kernel) and their kernel-trace summaries, overall and per launch size.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/${TAG:-rows2}/rows
mkdir -p "$OUT"
for w in ${ROWS:-c3 c4 c5 c6 c7 c8 c9}; do
  echo "== row $w"; date
  timeout -k 10 600 python -u bench.py --workload $w --steps ${STEPS:-20} --warmup 2 > "$OUT/bench_$w.json" \
     2> "$OUT/bench_$w.err" || { tail -20 "$OUT/bench_$w.err"; exit 1; }
  tail -c 400 "$OUT/bench_$w.json"; echo
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$w" -o $w -- \
    python3 bench.py --workload $w --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-traffic \
    > "$OUT/prof_$w.log" 2>&1 || exit 1
  python3 scripts/kstats_grid.py "$OUT/prof_$w" "$OUT/${w}_kernel_stats_by_grid.csv" || exit 1
done
echo done; date
