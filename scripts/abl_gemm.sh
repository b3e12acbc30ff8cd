#!/bin/bash
# GEMM ablation (diagnostics): HZ_FB_GEMM_ABL=1 no GS loads, 2 no K loads, 3 neither
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/ablg; mkdir -p $OUT
for v in ${ABLS:-0 1 2 3}; do
  HZ_FB_GEMM_ABL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o trace --output-format csv -- \
     python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/log$v 2>&1 || exit $?
  echo "ABL=$v"; grep -h "fb_lti_gemm" $OUT/p$v/*kernel_stats.csv | cut -d, -f1,3,4 | sed "s/.*fb_lti_gemm/fb_lti_gemm/" | cut -c1-120
done
