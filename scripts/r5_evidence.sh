#!/bin/bash
# Round 5 evidence: the default bench line (N = 1, traffic / flops PMC, CPU baseline, per-sample) and
# its kernel-trace stats; the secondary rows (each with PMC evidence) and their stats; the N = 2
# launcher rehearsal.  Stops at the first failed step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/${TAG:-ev}
mkdir -p "$OUT/rows" "$OUT/rehearse"
if [ -z "$SKIP_C2" ]; then
  echo "== bench c2"; date
  timeout -k 10 600 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail -20 "$OUT/bench_c2.err"; exit 1; }
  tail -c 300 "$OUT/bench_c2.json"; echo
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- \
    python3 bench.py --no-traffic --no-cpu-baseline --no-per-sample > "$OUT/prof_c2.log" 2>&1 || exit 1
fi
for w in ${ROWS:-c3 c4 c5 c6 c7 c8 c9}; do
  echo "== row $w"; date
  timeout -k 10 600 python -u bench.py --workload $w --steps ${STEPS:-20} --warmup 2 > "$OUT/rows/bench_$w.json" \
     2> "$OUT/rows/bench_$w.err" || { tail -20 "$OUT/rows/bench_$w.err"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rows/prof_$w" -o $w -- \
    python3 bench.py --workload $w --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-traffic \
    > "$OUT/rows/prof_$w.log" 2>&1 || exit 1
done
if [ -z "$SKIP_REH" ]; then
  echo "== rehearsal --gpus 2"; date
  HZ_BENCH_REHEARSAL=1 timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 --no-per-sample \
     --side-steps 10 --stream-blocks 64 > "$OUT/rehearse/c2_n2.json" 2> "$OUT/rehearse/c2_n2.err" || exit 1
  for w in c3 c4; do
    HZ_BENCH_REHEARSAL=1 timeout -k 10 600 python -u bench.py --gpus 2 --workload $w --steps 10 --warmup 2 \
       --no-cpu-baseline --no-traffic > "$OUT/rehearse/${w}_n2.json" 2> "$OUT/rehearse/${w}_n2.err" || exit 1
  done
fi
echo done; date
