#!/bin/bash
# Round 6: the general engine with softclip (compacted tail): parity, then the C2 bank's 10 s calls
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/soft
mkdir -p $D
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_filterbank_gpu.py tests/test_rt_server_gpu.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py --dist softclip --steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-per-sample --no-general-side --side-steps 0 --stream-blocks 0 > $D/soft$r.json 2> $D/soft$r.err || { tail -5 $D/soft$r.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$D/soft$r.json') if l.startswith('{')][-1])
print('softclip C2 ms/step %.4f' % d['ms_per_step'], d['roofline'].get('kernel'))"
done
