#!/bin/bash
# SQ counter passes on the C2 bench (rocprofv3 --pmc, kernel-trace only, one group per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sq}
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; tail -2 "$OUT/p$i.log"
  case $rc in 0) ;; *) echo "stop"; exit $rc;; esac
done
python3 - "$OUT" <<'PY'
import csv, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(list)
for root, _, files in os.walk(out):
    for f in files:
        if f.endswith("counter_collection.csv"):
            for r in csv.DictReader(open(os.path.join(root, f))):
                agg[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:60s} {c:28s} n={len(v):3d} max={max(v):.4e}")
PY
exit 0
