#!/bin/bash
# stationary engine: chunk / time segments of the zero-start band-state pass (HZ_FB_END_L / _M)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-endab}
mkdir -p "$OUT"
for cfg in "0 0" "32 2" "32 4" "64 2" "128 2"; do
  set -- $cfg
  HZ_FB_END_L=$1 HZ_FB_END_M=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic \
      --stream-blocks 0 --side-steps 0 > "$OUT/ab_$1_$2.log" 2>&1 || { tail -5 "$OUT/ab_$1_$2.log"; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/ab_$1_$2.log').read().strip().splitlines()[-1]); print('L=$1 M=$2: %.4f ms/step' % d['ms_per_step'], d['roofline']['components_ms_per_launch'])"
done
HZ_FB_END_L=32 HZ_FB_END_M=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filterbank_resp_gpu.py -m gpu > "$OUT/pytest_32_2.log" 2>&1; tail -1 "$OUT/pytest_32_2.log"
