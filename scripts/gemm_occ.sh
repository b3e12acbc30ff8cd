#!/bin/bash
# C2 engine time vs GEMM slice count (HZ_FB_GEMM_OCC workgroups per CU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/gocc; mkdir -p $OUT
for o in ${OCCS:-3 4 5 6}; do
  HZ_FB_GEMM_OCC=$o timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/b$o 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('$OUT/b$o') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('occ $o: C2 ms/step %.4f kernel_ms %.4f comps %s' % (d['ms_per_step'], r['kernel_avg_ms'], r['components_ms_per_launch']))"
done
