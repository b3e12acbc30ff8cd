#!/bin/bash
# C2 per-rank step of the time-partitioned (weak-scaling) multi-GPU bench, emulated on one GPU
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-emulweak}
mkdir -p "$OUT"
for P in ${WORLDS:-1 2 4 8}; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-traffic --stream-blocks 0 \
      --side-steps 0 --emulate-world $P > "$OUT/emul_$P.log" 2>&1 || { tail -5 "$OUT/emul_$P.log"; exit 1; }
  python - "$OUT/emul_$P.log" $P <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("P=%s ms/step %.4f value %.3e scaling %s per-gpu %s roofline frac %.3f comps %s" % (sys.argv[2], d["ms_per_step"], d["value"], d["scaling"], d["config"]["samples_per_gpu"], d["roofline"]["frac"], d["roofline"]["components_ms_per_launch"]))
PY
done
