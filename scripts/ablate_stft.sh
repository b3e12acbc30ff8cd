#!/bin/bash
# STFT frame-kernel ablation timings (experiments only): libraries built with -DHZ_STFT_ABLATE=A.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for A in ${ABL:-0 1 2 4 8 16}; do
  HZ_LIB_PATH=$PWD/huygens_amd/lib/ablS/libhuygens_hip_s$A.so timeout -k 10 120 python bench.py --workload c4 --steps 5 \
      --warmup 1 --no-cpu-baseline --no-traffic > gpurun_out/ablS_$A.log 2>&1 || exit 3
  python3 -c "
import json
for l in open('gpurun_out/ablS_$A.log'):
    if l.startswith('{'):
        d=json.loads(l); r=d['roofline']; print('abl $A step', round(d['ms_per_step'],4), 'frame', round(r['kernel_ms_per_step'],4))
"
done
exit 0
