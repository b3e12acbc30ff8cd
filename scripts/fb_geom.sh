#!/bin/bash
# C2 kernel geometry sweep: bench.py with each (waves, bands per wave).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${TAG:-geom}
mkdir -p "$OUT"
for g in ${GEOMS:-"16 1" "8 1" "4 1" "4 2" "4 4"}; do
  set -- $g
  timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-traffic --stream-blocks 0 \
      --waves $1 --bands-per-wave $2 > "$OUT/geom_$1_$2.log" 2>&1
  rc=$?
  python3 -c "
import json,sys
for l in open('$OUT/geom_$1_$2.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$1x$2', round(d['ms_per_step'],3), 'ms', '%.3e'%d['value'], 'frac', round(r['frac'],3), 'mix', round(r['kernel_avg_ms'],3), 'red', round(r['reduce_ms_per_launch'],3))
"
  [ $rc -ne 0 ] && { tail -5 "$OUT/geom_$1_$2.log"; exit $rc; }
done
exit 0
