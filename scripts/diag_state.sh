#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/diag_state; mkdir -p $OUT
HZ_FB_LTI_DIAG_STATE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- \
   python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/log 2>&1
echo rc=$?; cat $OUT/prof/*kernel_stats.csv | cut -c1-200
