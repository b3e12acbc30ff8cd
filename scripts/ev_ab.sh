#!/bin/bash
# timed C2 steps vs step / warmup counts (same box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${TAG:-evab}; mkdir -p $OUT
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-traffic --stream-blocks 0"
for sw in "20 3" "50 50" "200 20" "200 200" "1000 100" "20 500" "2000 200"; do
  set -- $sw
  $B --steps $1 --warmup $2 > $OUT/s$1_w$2.log 2>&1 || exit 1
  echo "steps $1 warmup $2 $(grep -h -o '"ms_per_step": [0-9.]*' $OUT/s$1_w$2.log)"
done
