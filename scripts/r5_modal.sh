#!/bin/bash
# Round 5: modal band states -- tests, then bench A/B (modal on / matrix-core pass), then rocprof stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/modal
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "modal or resp or c2_pinned or fullsize or high_q or highq or stream" > "$OUT/pytest.log" 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -5; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for i in 1 2; do
  timeout -k 10 200 python -u bench.py $Q --modal 1 > "$OUT/bench_modal_$i.json" || exit 3
  timeout -k 10 200 python -u bench.py $Q --modal 0 > "$OUT/bench_mfma_$i.json" || exit 3
done
for f in "$OUT"/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['step']['components_ms_per_call'])"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o modal -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" $Q --steps 100 > "$GRAFT_REPO_ROOT/$OUT/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$OUT/prof.err"
echo "rocprof rc=$?"
find "$GRAFT_REPO_ROOT/$OUT/prof" -name "*kernel_stats.csv" | head -3
