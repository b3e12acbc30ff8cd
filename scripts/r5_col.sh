#!/bin/bash
# Round 5: column-split stationary path -- parity, then A/B timing against the three-kernel path,
# then a kernel-trace profile of the default bench
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/${TAG:-col}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_filterbank_resp_gpu.py tests/test_c2_pinned_gpu.py tests/test_fb_stream_gpu.py \
   -x -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; echo "pytest rc=$rc"; [ $rc = 0 ] || { grep -E "^E " "$OUT/pytest.log" | head -20; exit $rc; }
for k in 1 0 1 0; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-traffic --no-per-sample --no-cpu-baseline \
     --stream-blocks 0 --side-steps 0 --resp-engine $k > "$OUT/bench_e$k.json" 2> "$OUT/bench_e$k.err" || exit $?
  python3 -c "import json;d=json.loads(open('$OUT/bench_e$k.json').read().strip().splitlines()[-1]);r=d['roofline'];print('engine $k', 'ms/step %.5f'%d['ms_per_step'], 'comp', r['step']['components_ms_per_call'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv -- \
   python3 bench.py --steps 50 --warmup 5 --no-traffic --no-per-sample --no-cpu-baseline --stream-blocks 0 --side-steps 0 \
   > "$OUT/prof.log" 2>&1 || exit $?
f=$(find "$OUT/prof" -name "*kernel_stats.csv" | head -1); cp "$f" "$OUT/kernel_stats.csv"; head -12 "$OUT/kernel_stats.csv" | cut -c1-200
