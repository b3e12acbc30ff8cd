#!/bin/bash
# Round 5: where modal phase 2 runs (HZ_MODAL_P2: inv = after the inverse transforms, inv_first =
# before them, mac = beside the MAC), alternating, plus the matrix-core pass
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r5/modal_p2
mkdir -p "$OUT"
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for r in 1 2; do
  for p in inv inv_first mac; do
    HZ_MODAL_P2=$p timeout -k 10 200 python -u bench.py $Q > "$OUT/$p.$r.json" || exit 3
    python -c "import json; d=json.load(open('$OUT/$p.$r.json')); print('$p', d['ms_per_step'], d['roofline']['step']['components_ms_per_call'])"
  done
done
timeout -k 10 200 python -u bench.py $Q --modal 0 > "$OUT/mfma.json" || exit 3
python -c "import json; d=json.load(open('$OUT/mfma.json')); print('mfma', d['ms_per_step'], d['roofline']['step']['components_ms_per_call'])"
