#!/bin/bash
# Round 5: modal phase granularity (HZ_MODAL_R1PER residues per phase-1 workgroup, HZ_MODAL_K1PER
# columns per phase-2 workgroup), alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r5/modal_per
mkdir -p "$OUT"
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for r in 1 2; do
  for cfg in "1 1" "4 1" "16 1" "1 4" "4 4" "16 4"; do
    set -- $cfg
    HZ_MODAL_R1PER=$1 HZ_MODAL_K1PER=$2 timeout -k 10 200 python -u bench.py $Q > "$OUT/p$1_$2.$r.json" || exit 3
    python -c "import json; d=json.load(open('$OUT/p$1_$2.$r.json')); print('r1per $1 k1per $2', d['ms_per_step'], d['roofline']['step']['components_ms_per_call'])"
  done
done
