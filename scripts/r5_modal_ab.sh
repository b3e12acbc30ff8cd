#!/bin/bash
# Round 5: modal tests, then the modal step against the matrix-core pass, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r5/modal_ab
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "modal or c2_pinned or resp" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for r in 1 2; do
  for m in 1 0; do
    timeout -k 10 200 python -u bench.py $Q --modal $m > "$OUT/m$m.$r.json" || exit 3
    python -c "import json; d=json.load(open('$OUT/m$m.$r.json')); print('modal $m', d['ms_per_step'], d['roofline']['step']['components_ms_per_call'])"
  done
done
