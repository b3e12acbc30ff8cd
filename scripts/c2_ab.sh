#!/bin/bash
# C2 A/B: LTI parity tests on the in-tree library, then default C2 bench lines (no traffic /
# cpu passes) for it and for huygens_amd/lib/ab/lib_base.so (HZ_LIB_PATH), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${TAG:-c2ab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_filterbank_lti_gpu.py ${TESTS:-} > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for v in new base; do
    L=""; [ $v = base ] && L="HZ_LIB_PATH=$PWD/huygens_amd/lib/ab/lib_base.so"
    env $L timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/$v$i.log 2>&1 || exit 1
    python3 -c "
import json; l=[x for x in open('$OUT/$v$i.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$v$i C2 ms/step %.4f value %.3e kernel_ms %.4f comps %s' % (d['ms_per_step'], d['value'], r['kernel_avg_ms'], {k: round(v,4) for k,v in r['components_ms_per_launch'].items()}))"
  done
done
