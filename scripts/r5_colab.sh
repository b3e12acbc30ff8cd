#!/bin/bash
# Round 5: column-split path A/B (engine 1 vs 0) + phase stamps from the diagnostic library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/${TAG:-colab}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_filterbank_resp_gpu.py tests/test_c2_pinned_gpu.py -x -q --timeout 300 \
     --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc = 0 ] || { grep -E "^E " "$OUT/pytest.log" | head -20; exit $rc; }
fi
for k in 1 0 1 0; do
  timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-traffic --no-per-sample --no-cpu-baseline \
     --stream-blocks 0 --side-steps 0 --resp-engine $k > "$OUT/bench_e$k.json" 2> "$OUT/bench_e$k.err" || exit $?
  python3 -c "import json;d=json.loads(open('$OUT/bench_e$k.json').read().strip().splitlines()[-1]);r=d['roofline'];print('engine $k', 'ms/step %.5f'%d['ms_per_step'], 'comp', r['step']['components_ms_per_call'])"
done
HZ_LIB_PATH=$PWD/huygens_amd/lib/diag/libhuygens_hip.so timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-traffic \
   --no-per-sample --no-cpu-baseline --stream-blocks 0 --side-steps 0 > "$OUT/diag.json" 2> "$OUT/diag.err" || exit $?
grep -h "stamps\]" "$OUT/diag.err" | head -5
