#!/bin/bash
# (diagnostic) kernel-argument placement: HIP_FORCE_DEV_KERNARG=0 / 1 on the churn driver (with the
# launch trace) and on the C2 bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/kernarg
mkdir -p $D
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, ".")
import bench
f, b = bench.c2_coefficients()
np.concatenate([np.asarray(f)[:, :3], np.asarray(b)[:, :2]], axis=1).astype(np.float64).tofile("gpurun_out/r6/kernarg/coef.bin")
np.random.default_rng(1).uniform(-1, 1, 480000).tofile("gpurun_out/r6/kernarg/x.bin")
PY
/opt/rocm/bin/hipcc -std=c++17 -O2 -I include tests/cpp/churn.cpp -o $D/churn -L huygens_amd/lib -lhuygens_hip -Wl,-rpath,$PWD/huygens_amd/lib || exit 1
for kv in 0 1; do
  echo "HIP_FORCE_DEV_KERNARG=$kv"
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 120 $D/churn $D || exit 1
  rm -f $D/t$kv.bin
  HIP_FORCE_DEV_KERNARG=$kv HZ_STREAM_TRACE=$D/t$kv.bin timeout -k 10 120 $D/churn $D > /dev/null && python3 scripts/stream_trace.py $D/t$kv.bin | grep -E "span|column marks|setter columns"
  HIP_FORCE_DEV_KERNARG=$kv timeout -k 10 200 python3 -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-traffic --no-per-sample --no-general-side --side-steps 0 --stream-blocks 200 > $D/bench$kv.json 2> $D/bench$kv.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('$D/bench$kv.json') if l.startswith('{')][-1])
print('C2 ms/step %.4f' % d['ms_per_step'], 'kernels', {k: round(v*1e3,2) for k,v in d['roofline']['kernels_ms_per_call'].items()}, 'streaming us/block', d.get('streaming',{}).get('us_per_block'))
"
done
