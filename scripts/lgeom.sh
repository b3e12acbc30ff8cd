#!/bin/bash
# LTI chunk-length comparison on the C2 bench: parity of the LTI tests, then bench per L.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lgeom}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_filterbank_lti_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
for L in ${LS:-32 64}; do
  HZ_FB_LTI_L=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --stream-blocks 0 > "$OUT/bench_L$L.log" 2>&1
  rc=$?; echo "L=$L rc=$rc"; python3 -c "
import json,sys
l=[x for x in open('$OUT/bench_L$L.log') if x.startswith('{')]
d=json.loads(l[-1]); r=d['roofline']
print('ms/step %.4f value %.3e comps %s' % (d['ms_per_step'], d['value'], r['components_ms_per_launch']))
" ; case $rc in 0) ;; *) exit $rc;; esac
done
