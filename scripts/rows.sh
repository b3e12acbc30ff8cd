#!/bin/bash
# Secondary-row measurements (bench.py --workload c3/c4/c5) + rocprofv3 kernel stats each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rows}
mkdir -p "$OUT"
for w in ${ROWS:-c3 c4 c5}; do
  echo "== bench $w"; date
  timeout -k 10 400 python bench.py --workload $w --steps ${STEPS:-5} --warmup 1 > "$OUT/bench_$w.log" 2>&1
  rc=$?; tail -2 "$OUT/bench_$w.log"; echo "rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o trace --output-format csv -- \
      python3 bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-traffic > "$OUT/prof_$w.log" 2>&1
  rc=$?; echo "rocprof rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
