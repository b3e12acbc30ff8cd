#!/bin/bash
# Per-rank C2 step of an N-GPU job on one MI355X (bench.py --emulate-world P: rank 0's shard of a
# time-split stationary job; the other shards' handles only feed the whole bank's response).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-emul}; mkdir -p $OUT
for P in ${WORLDS:-1 2 4 8}; do
  timeout -k 10 200 python bench.py --emulate-world $P --steps 100 --warmup 10 --no-cpu-baseline --no-traffic \
      --no-per-sample --side-steps 0 --stream-blocks 0 > $OUT/p$P.log 2>&1 || { echo "P=$P failed"; tail -5 $OUT/p$P.log; exit 1; }
  python3 - $OUT/p$P.log $P <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]
P = int(sys.argv[2])
print(f"P={P}: per-rank step {d['ms_per_step']:.4f} ms, whole-job {P * 4096 * 480000 / (d['ms_per_step'] / 1e3):.3e} "
      f"band-samples/s, dominant {d['roofline']['kernel_avg_ms']:.4f} ms, comps {d['roofline']['step']['components_ms_per_call']}")
PY
done
