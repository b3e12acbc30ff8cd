#!/bin/bash
# A/B of environment settings on the short C2 bench: VARIANTS="A=1 B=2;A=3" bash scripts/ab_env.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
IFS=';' read -ra VS <<< "$VARIANTS"
i=0
for v in "${VS[@]}"; do
  for rep in 1 2; do
    env $v timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-traffic --no-per-sample --side-steps 0 \
        --stream-blocks 0 ${BENCH_ARGS:-} > "$OUT/v$i.$rep.log" 2>&1 || { echo "variant [$v] failed"; tail -5 "$OUT/v$i.$rep.log"; exit 1; }
    ms=$(python3 -c "import json,sys; l=[x for x in open('$OUT/v$i.$rep.log') if x.startswith('{')][-1]; d=json.loads(l); print(d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['step']['components_ms_per_call'])")
    echo "[$v] rep $rep: ms_per_step, state ms, comps = $ms"
  done
  i=$((i+1))
done
