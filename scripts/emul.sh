#!/bin/bash
# per-GPU shard step of an N-GPU C2 job, measured on one GPU (bench.py --emulate-world N)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-emul}; mkdir -p $OUT
for w in ${WORLDS:-1 2 4 8}; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --stream-blocks 0 --emulate-world $w > $OUT/ew$w.log 2>&1
  rc=$?; python3 -c "
import json
l=[x for x in open('$OUT/ew$w.log') if x.startswith('{')]
d=json.loads(l[-1]); r=d['roofline']
print('world $w: shard %d bands, ms/step %.4f comps %s' % (d['config']['bands_per_gpu'], d['ms_per_step'], {k: round(v,4) for k,v in r['components_ms_per_launch'].items()}))
"; case $rc in 0) ;; *) echo rc=$rc; exit $rc;; esac
done
