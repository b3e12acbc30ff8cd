#!/bin/bash
# LTI kernel ablation timings (experiments only): libraries built with -DHZ_LTI_ABLATE=A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for A in ${ABL:-0 1 2 4 7}; do
  for g in ${GEOMS:-16,1,16}; do
    HZ_LIB_PATH=$PWD/huygens_amd/lib/abl/libhuygens_hip_$A.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --stream-blocks 0 --lti $g > gpurun_out/abl_$A_$g.log 2>&1 || exit 3
    python3 -c "
import json
for l in open('gpurun_out/abl_$A_$g.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('abl $A geom $g', round(d['ms_per_step'],3), 'mix', round(r['kernel_avg_ms'],3), 'red', round(r['reduce_ms_per_launch'],3))
"
  done
done
exit 0
