#!/bin/bash
# Round 5 (session 2): the GPU suite, then A/B runs (alternating) of
#   C2: modal phase 1 in the forward launch (default) vs in the MAC launch (HZ_MODAL_P1=mac)
#   C4: segment overlap-add (default) vs the flat one (HZ_STFT_OLA_FLAT=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/${TAG:-s2a}
mkdir -p "$OUT"
if [ -z "$SKIP_TESTS" ]; then
  date
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=15 \
    > "$OUT/pytest.log" 2>&1
  rc=$?; grep -E "FAILED|ERROR" "$OUT/pytest.log" | head -20; tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
  [ $rc -eq 0 ] || exit $rc
fi
Q="--no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 0"
for r in 1 2; do
  for v in fwd mac; do
    if [ $v = mac ]; then E="HZ_MODAL_P1=mac"; else E="HZ_MODAL_P1=fwd"; fi
    env $E timeout -k 10 200 python -u bench.py $Q > "$OUT/c2_$v.$r.json" || exit 3
    python -c "import json; d=json.load(open('$OUT/c2_$v.$r.json')); print('c2 p1=$v', d['ms_per_step'], d['roofline']['step']['components_ms_per_call'])"
  done
done
for r in 1 2; do
  for v in seg flat; do
    if [ $v = flat ]; then E="HZ_STFT_OLA_FLAT=1"; else E="HZ_STFT_OLA_SEG=1"; fi
    env $E timeout -k 10 200 python -u bench.py --workload c4 --steps 20 --warmup 2 --no-cpu-baseline --no-traffic \
      > "$OUT/c4_$v.$r.json" || exit 4
    python -c "import json; d=json.load(open('$OUT/c4_$v.$r.json')); r=d['roofline']; print('c4 ola=$v', d['ms_per_step'], r['kernel_ms_per_step'], r['ola_ms_per_step'])"
  done
done
date
