#!/bin/bash
# State-kernel ablation (diagnostics): rocprof kernel times with the E chains and/or the scan
# compiled out (HZ_FB_LTI_ABL=1: no E, 2: no scan, 3: neither; results are wrong by design).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/abl; mkdir -p $OUT
for v in ${ABLS:-0 1 2 3}; do
  HZ_FB_LTI_ABL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p$v -o trace --output-format csv -- \
     python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/log$v 2>&1 || exit $?
  echo "ABL=$v"; grep -h "fb_lti_kernel<2, 1*[26][48]*, 2" $OUT/p$v/*kernel_stats.csv | cut -d, -f1,3,4 | sed "s/.*fb_lti_kernel/fb_lti_kernel/" | cut -c1-120
done
