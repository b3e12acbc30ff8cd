#!/bin/bash
# C2: 16-byte input loads in the forward and output stores in the inverse (this tree) against
# 8-byte ones (huygens_amd/lib/ab_old, the previous commit's build);
# stationary-engine parity first, then alternating bench runs on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/vec
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_filterbank_resp_gpu.py tests/test_c2_pinned_gpu.py tests/test_fb_modal_gpu.py tests/test_fb_stream_gpu.py \
  tests/test_fb_highq_gpu.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for r in 1 2 3; do
  for v in new old; do
    if [ $v = old ]; then export HZ_LIB_PATH=$PWD/huygens_amd/lib/ab_old/libhuygens_hip.so; else unset HZ_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py $Q > "$OUT/c2_$v.$r.json" 2> "$OUT/c2_$v.$r.err" || { tail -5 "$OUT/c2_$v.$r.err"; exit 3; }
    python -c "import json; d=json.loads(open('$OUT/c2_$v.$r.json').read().strip().splitlines()[-1]); print('c2 $v', round(d['ms_per_step']*1e3,2), d['roofline']['step']['components_ms_per_call'])"
  done
done
HZ_LIB_PATH=$PWD/huygens_amd/lib/diag/libhuygens_hip.so timeout -k 10 200 python -u bench.py $Q --steps 40 > "$OUT/diag.json" 2> "$OUT/diag.err"; grep -a stamps "$OUT/diag.err"; exit 0
