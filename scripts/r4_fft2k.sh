#!/bin/bash
# hz_fft2k.h wave-local passes: stationary / streaming parity, then the C2 bench (kernel stats)
set -o pipefail
OUT=gpurun_out/r4/fft2k
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filterbank_resp_gpu.py \
  tests/test_c2_pinned_gpu.py tests/test_fb_stream_gpu.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline --no-per-sample > $OUT/b$i.json 2> $OUT/b$i.err || exit 1
  python3 -c "
import json
l=json.loads(open('$OUT/b$i.json').read().strip().splitlines()[-1]); print('run $i', round(l['ms_per_step'],5), round(l['roofline']['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o c2 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-traffic --no-cpu-baseline --no-per-sample > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
