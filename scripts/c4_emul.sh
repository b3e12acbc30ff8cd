#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/c4_emul; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_stft_gpu.py tests/test_cpp_gpu.py -m gpu > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; echo "pytest rc=$rc"; case $rc in 0|1) ;; *) exit $rc;; esac
for w in 1 2 4 8; do
  timeout -k 10 200 python bench.py --workload c4 --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --emulate-world $w > $OUT/ew$w.log 2>&1
  rc=$?; python3 -c "
import json
l=[x for x in open('$OUT/ew$w.log') if x.startswith('{')]
d=json.loads(l[-1]); r=d['roofline']
print('c4 world $w: ms/step %.4f frames/s %.3e kernel_ms %.4f ola_ms %.4f' % (d['ms_per_step'], d['value'], r['kernel_ms_per_step'], r['ola_ms_per_step']))
"; case $rc in 0) ;; *) echo rc=$rc; exit $rc;; esac
done
