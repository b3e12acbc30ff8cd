#!/bin/bash
# Round 5 final evidence: the GPU suite, smoke, the C2 bench line (PMC traffic + flops, CPU
# baseline) and its rocprofv3 kernel-trace summary (overall and per grid)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/final
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$OUT/pytest_gpu.log" | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 2; }
tail -2 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err" || { tail "$OUT/bench_c2.err"; exit 3; }
python -c "import json; d=json.loads(open('$OUT/bench_c2.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['frac'], r['step']['components_ms_per_call'], r['step']['traffic_per_kernel'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o c2 -- \
  python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-traffic --no-per-sample --side-steps 0 --stream-blocks 0 \
  > "$OUT/prof.log" 2>&1 || exit 4
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/fb_c2_kernel_stats.csv" \;
python3 scripts/kstats_grid.py "$OUT/prof" "$OUT/fb_c2_kernel_stats_by_grid.csv" || true
head -5 "$OUT/fb_c2_kernel_stats.csv" | cut -c1-200
exit 0
