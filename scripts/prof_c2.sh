#!/bin/bash
# rocprofv3 kernel stats of a short C2 bench (extra env passed through)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof_c2}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- \
   python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 ${BENCH_ARGS:-} > $OUT/log 2>&1
echo rc=$?; cut -d, -f1-4 $OUT/prof/*kernel_stats.csv | cut -c1-160
