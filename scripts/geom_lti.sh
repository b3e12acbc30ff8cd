#!/bin/bash
# LTI engine geometry sweep on the C2 bench (+ the LTI parity tests first).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_filterbank_lti_gpu.py > gpurun_out/lti_tests.log 2>&1
rc=$?; tail -3 gpurun_out/lti_tests.log; [ $rc -le 1 ] || exit $rc
for g in ${GEOMS:-16,1,16 32,1,16 16,2,8}; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --stream-blocks 0 --lti $g > gpurun_out/g_$g.log 2>&1 || exit 3
  python3 -c "
import json
for l in open('gpurun_out/g_$g.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('$g', round(d['ms_per_step'],3), 'mix', round(r['kernel_avg_ms'],3), 'red', round(r['reduce_ms_per_launch'],3))
"
done
exit 0
