#!/bin/bash
# Round 6: per-rank C2 step of the N > 1 value path (time split of the fixed 10 s call), emulated
# on one MI355X: rank r of P alone (bench.py --emulate-world P --emulate-rank r), P = 1, 2, 4, 8,
# the first and the last rank (the last holds the exceptional Nyquist band); then a one-GPU
# rehearsal of bench.py --gpus 2 (two ranks on cuda:0, gloo through host copies).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r6/emul
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="--steps 200 --warmup 20 --no-cpu-baseline --no-traffic --no-per-sample --stream-blocks 0 --side-steps ${SIDE:-50}"
for P in 1 2 4 8; do
  for R in 0 $((P - 1)); do
    [ "$P" = 1 ] && [ "$R" = 0 ] && [ -f $OUT/p1_r0.json ] && continue
    timeout -k 10 240 python3 -u bench.py $COMMON --emulate-world $P --emulate-rank $R > $OUT/p${P}_r${R}.json 2> $OUT/p${P}_r${R}.err || exit $?
    python3 - "$OUT/p${P}_r${R}.json" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print(sys.argv[1], "ms/step %.4f" % d["ms_per_step"], "value %.3e" % d["value"],
      "kernels", {k: round(v * 1e3, 2) for k, v in (r.get("kernels_ms_per_call") or {}).items()},
      "samples_per_gpu", d["config"]["samples_per_gpu"],
      "side", {k: round(v["ms_per_step"], 4) for k, v in (d.get("side") or {}).items() if isinstance(v, dict) and "ms_per_step" in v})
PY
  done
done
if [ -n "$REHEARSE" ]; then
  HZ_BENCH_REHEARSAL=1 timeout -k 10 300 python3 -u bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline --no-traffic \
     --stream-blocks 32 --side-steps 20 > $OUT/rehearse_n2.json 2> $OUT/rehearse_n2.err || exit $?
  tail -c 1500 $OUT/rehearse_n2.json
fi
