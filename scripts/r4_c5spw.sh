#!/bin/bash
# C5 fused block: samples per workgroup 4 (default) vs 2 and 8, alternating, after the chain tests
set -o pipefail
OUT=gpurun_out/r4/c5spw
mkdir -p $OUT
for v in 2 8; do
  HZ_CHAIN_SPW=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_chain_gpu.py \
    > $OUT/pytest_$v.log 2>&1 || { tail -20 $OUT/pytest_$v.log; exit 1; }
  tail -1 $OUT/pytest_$v.log
done
for i in 1 2; do for v in 4 2 8; do
  HZ_CHAIN_SPW=$v timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 1 --no-cpu-baseline --no-traffic > $OUT/b_${v}_$i.log 2>&1 || exit 1
  python3 -c "
import json
l=json.loads(open('$OUT/b_${v}_$i.log').read().strip().splitlines()[-1]); b=l['block']; print('spw $v run $i', round(b['us_per_block'],3), round(b['kernel_us_per_block'],3))"
done; done
