#!/bin/bash
# A/B of the stationary engine's end-state placement (HZ_FB_RESP_STATE 0 / 1 / 2) on C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-respab}
mkdir -p "$OUT"
for m in ${MODES:-0 1 2}; do
  HZ_FB_RESP_STATE=$m timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic \
      --stream-blocks 0 --side-steps 0 > "$OUT/ab_$m.log" 2>&1 || exit $?
  python -c "import json,sys; d=json.loads(open('$OUT/ab_$m.log').read().strip().splitlines()[-1]); print('state mode $m: %.4f ms/step' % d['ms_per_step'], d['roofline']['components_ms_per_launch'])"
done
for m in ${PROF_MODES:-1}; do
  HZ_FB_RESP_STATE=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$m" -o trace --output-format csv -- \
      python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-traffic --stream-blocks 0 --side-steps 0 > "$OUT/prof_$m.log" 2>&1 || exit $?
done
