#!/bin/bash
# rocprofv3 kernel stats of the short C2 bench per environment variant:
#   VARIANTS="A=1;A=2" bash scripts/prof_env.sh   -> gpurun_out/$TAG/p<i>/..._kernel_stats.csv
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-profenv}
mkdir -p "$OUT"
IFS=';' read -ra VS <<< "$VARIANTS"
i=0
for v in "${VS[@]}"; do
  env $v timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$OUT/p$i" -o trace --output-format csv -- \
      python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-traffic --no-per-sample --side-steps 0 \
      --stream-blocks 0 ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1 || { echo "variant [$v] failed"; tail -3 "$OUT/p$i.log"; exit 1; }
  f=$(find "$OUT/p$i" -name "*kernel_stats.csv" | head -1)
  echo "== [$v]"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Calls"]) >= 10:
        print(f'{float(r["AverageNs"])/1e3:9.2f} us  x{r["Calls"]:>4}  {r["Name"][:110]}')
PY
  i=$((i+1))
done
