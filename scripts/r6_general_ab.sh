#!/bin/bash
# Round 6: the general engine (fb_mix_kernel) on the C2 bank -- no functor (--general) and the
# reference demos' &softclip (--dist softclip) -- across workgroup geometries (waves x bands per
# wave, hz_fb_tune), 480,000-sample calls.  Prints ms per call and the mix kernel's event time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r6/general_ab
mkdir -p $OUT
export TMPDIR=/tmp
COMMON="--steps 20 --warmup 3 --no-cpu-baseline --no-traffic --no-per-sample --stream-blocks 0 --side-steps 0 --no-general-side"
for mode in "--general" "--dist softclip"; do
  for geom in "16 1" "8 1" "8 2" "4 1" "4 2" "4 4"; do
    set -- $geom
    tag="$(echo $mode | tr -d ' -')_w$1_nb$2"
    timeout -k 10 120 python3 -u bench.py $COMMON $mode --waves $1 --bands-per-wave $2 > $OUT/$tag.json 2> $OUT/$tag.err || { echo "$tag failed"; tail -3 $OUT/$tag.err; continue; }
    python3 - $OUT/$tag.json $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r = d["roofline"]
print("%-28s ms/call %.4f  mix kernel %.4f ms  frac18 %.3f  path %s" % (sys.argv[2], d["ms_per_step"], r["kernel_avg_ms"],
      18 * 4096 * 480000 / (r["kernel_avg_ms"] / 1e3) / 1e12 / 78.6, d["engine"]))
PY
  done
done
