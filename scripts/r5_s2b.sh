#!/bin/bash
# Round 5 (session 2): the default C2 bench line + its kernel-trace stats, then secondary rows
# (ROWS) with PMC evidence and per-launch-size kernel-trace summaries.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/${TAG:-s2b}
mkdir -p "$OUT"
if [ -z "$SKIP_C2" ]; then
  echo "== bench c2"; date
  timeout -k 10 600 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -20 "$OUT/bench_c2.err"; exit 1; }
  tail -c 300 "$OUT/bench_c2.json"; echo
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- \
    python3 bench.py --no-traffic --no-cpu-baseline --no-per-sample > "$OUT/prof_c2.log" 2>&1 || exit 1
fi
TAG=${TAG:-s2b} ROWS="$ROWS" bash scripts/r5_rows2.sh
