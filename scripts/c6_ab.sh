#!/bin/bash
# C6 A/B: granulator parity tests on the in-tree library, then C6 bench lines for it and for
# huygens_amd/lib/ab/lib_base.so (HZ_LIB_PATH), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${TAG:-c6ab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_granulator_gpu.py > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in new base; do
    L=""; [ $v = base ] && L="HZ_LIB_PATH=$PWD/huygens_amd/lib/ab/lib_base.so"
    env $L timeout -k 10 200 python bench.py --workload c6 --steps 100 --warmup 10 --no-cpu-baseline --no-traffic > $OUT/$v$i.log 2>&1 || exit 1
    python3 -c "
import json; l=[x for x in open('$OUT/$v$i.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('$v$i C6 ms/step %.4f value %.3e kernel_ms %.4f' % (d['ms_per_step'], d['value'], r['kernel_ms_per_step']))"
  done
done
