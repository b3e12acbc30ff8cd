#!/bin/bash
# Per-wave phase timestamps of the C2 state kernel (diagnostics build variant, HZ_FB_LTI_ABL=16),
# then C2 timings per phase order (HZ_FB_LTI_ORDER)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/stamps; mkdir -p $OUT
for o in ${ORDERS:-0 1}; do
  HZ_FB_LTI_ORDER=$o HZ_FB_LTI_ABL=16 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/log$o 2>&1 || exit $?
  echo "order $o"; grep stamps $OUT/log$o | tail -16
  HZ_FB_LTI_ORDER=$o timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/bench$o 2>&1 || exit $?
  python3 -c "
import json; l=[x for x in open('$OUT/bench$o') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('order $o: C2 ms/step %.4f kernel_ms %.4f comps %s' % (d['ms_per_step'], r['kernel_avg_ms'], r['components_ms_per_launch']))"
done
