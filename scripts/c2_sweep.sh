#!/bin/bash
# C2 engine time per setting of one environment knob: VAR=HZ_FB_GEMM_OCC VALS="3 4 6"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/sweep; mkdir -p $OUT
for v in ${VALS}; do
  env $VAR=$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/b_$v 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('$OUT/b_$v') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$VAR=$v: C2 ms/step %.4f kernel_ms %.4f comps %s' % (d['ms_per_step'], r['kernel_avg_ms'], r['components_ms_per_launch']))"
done
