#!/bin/bash
# C3 iteration loop: additive parity tests, then the C3 bench line and rocprof kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c3q}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_additive_gpu.py ${TESTS:-} > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload c3 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/bench.log; exit $rc; }
python3 -c "
import json; l=[x for x in open('$OUT/bench.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('C3 ms/step %.4f value %.3e kernel_ms %.4f frac %.3f ref-eq %s' % (d['ms_per_step'], d['value'], r['kernel_avg_ms'], r['frac'], r.get('reference_equivalent')))"
