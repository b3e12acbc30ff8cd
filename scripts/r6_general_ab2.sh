#!/bin/bash
# Round 6: general engine mix pass, recompute (MODE_MIXR, default) against the fix-up form
# (HZ_FB_FIXUP=1), alternating on one box, no functor and &softclip, 16-wave groups.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r6/general_ab2
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="--steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-per-sample --stream-blocks 0 --side-steps 0 --no-general-side"
for rep in 1 2; do
for mode in "--general" "--dist softclip"; do
  for fix in ${FIXES:-0 1}; do
    tag="$(echo $mode | tr -d ' -')_fix${fix}_$rep"
    HZ_FB_FIXUP=$fix timeout -k 10 120 python3 -u bench.py $COMMON $mode > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; exit 1; }
    python3 - $OUT/$tag.json $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("%-28s ms/call %.4f  mix kernel %.4f ms  frac18 %.3f" % (sys.argv[2], d["ms_per_step"], r["kernel_avg_ms"],
      18 * 4096 * 480000 / (r["kernel_avg_ms"] / 1e3) / 1e12 / 78.6))
PY
  done
done
done
