#!/bin/bash
# C9 coefficient streams: tv parity tests, then the row with the bounded-range trig (default) and libm (A/B)
set -o pipefail
OUT=gpurun_out/r4/c9
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_filterbank_tv_gpu.py \
  tests/test_c1_resynthesis.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload c9 --steps 10 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/fast$i.log 2>&1 || exit 1
  HZ_FB_TV_LIBM=1 timeout -k 10 300 python bench.py --workload c9 --steps 10 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/libm$i.log 2>&1 || exit 1
done
for f in fast1 libm1 fast2 libm2; do python3 -c "
import json,sys
l=json.loads(open('$OUT/$f.log').read().strip().splitlines()[-1]); print('$f', round(l['ms_per_step'],3), round(l['roofline']['frac'],4))"; done
