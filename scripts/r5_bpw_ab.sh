#!/bin/bash
# C2 LDS MAC: 4 blocks per wave (HZ_MAC_BPW=4, 16 per workgroup) against 8 (default); parity with 4
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/bpw
mkdir -p "$OUT"
HZ_MAC_BPW=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_filterbank_resp_gpu.py tests/test_c2_pinned_gpu.py tests/test_fb_modal_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for r in 1 2 3; do
  for v in 8 4; do
    export HZ_MAC_BPW=$v
    timeout -k 10 200 python -u bench.py $Q > "$OUT/c2_$v.$r.json" 2> "$OUT/c2_$v.$r.err" || { tail -5 "$OUT/c2_$v.$r.err"; exit 3; }
    python -c "import json; d=json.loads(open('$OUT/c2_$v.$r.json').read().strip().splitlines()[-1]); print('c2 bpw $v', round(d['ms_per_step']*1e3,2), d['roofline']['step']['components_ms_per_call'])"
  done
done
