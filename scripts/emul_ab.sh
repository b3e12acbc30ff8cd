#!/bin/bash
# emulated-world shard steps for several env settings: WORLDS, then settings as arguments
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-emul_ab}; mkdir -p $OUT
for setting in "$@"; do
  [ "$setting" = "-" ] && setting=""
  for w in ${WORLDS:-8}; do
    env $setting timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --stream-blocks 0 --emulate-world $w > $OUT/ew.log 2>&1
    rc=$?; python3 -c "
import json
l=[x for x in open('$OUT/ew.log') if x.startswith('{')]
d=json.loads(l[-1]); r=d['roofline']
print('[$setting] world $w: ms/step %.4f comps %s' % (d['ms_per_step'], {k: round(v,4) for k,v in r['components_ms_per_launch'].items()}))
"; case $rc in 0) ;; *) echo rc=$rc; exit $rc;; esac
  done
done
