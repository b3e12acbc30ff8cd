#!/bin/bash
# A/B of env settings on the C2 bench: parity of the LTI tests once, then one bench line per
# setting ("VAR=val VAR2=val" strings as arguments; "-" = defaults).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
if [ -z "$NOTEST" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_filterbank_lti_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
fi
i=0
for setting in "$@"; do
  i=$((i+1))
  [ "$setting" = "-" ] && setting=""
  env $setting timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --stream-blocks 0 ${BENCH_ARGS:-} > "$OUT/bench_$i.log" 2>&1
  rc=$?; python3 -c "
import json
l=[x for x in open('$OUT/bench_$i.log') if x.startswith('{')]
d=json.loads(l[-1]); r=d['roofline']
print('[$setting] ms/step %.4f value %.3e comps %s' % (d['ms_per_step'], d['value'], {k: round(v,4) for k,v in r['components_ms_per_launch'].items()}))
" ; case $rc in 0) ;; *) echo "rc=$rc"; exit $rc;; esac
done
