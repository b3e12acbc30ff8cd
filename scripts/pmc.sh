#!/bin/bash
# PMC passes (rocprofv3 --pmc, kernel-trace only; one counter group per pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
CMD="python3 bench.py --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --stream-blocks 0 ${BENCH_ARGS:-}"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --stats -d "$OUT/p$i" -o pmc --output-format csv -- $CMD > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"; tail -2 "$OUT/p$i.log"
  case $rc in 0|1) ;; *) echo "stop"; exit $rc;; esac
done
exit 0
