#!/bin/bash
# Round 5: modal phases' cost (HZ_MODAL_DIAG: 1 no phase 1, 2 no phase 2, 3 no exceptional partials;
# timing only -- the states are wrong in the diagnostic runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r5/modal_diag
mkdir -p "$OUT"
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for d in 0 1 2 3 0; do
  HZ_MODAL_DIAG=$d timeout -k 10 200 python -u bench.py $Q > "$OUT/d$d.json" || exit 3
  python -c "import json; d=json.load(open('$OUT/d$d.json')); print('diag $d', d['ms_per_step'], d['roofline']['step']['components_ms_per_call'])"
done
