#!/bin/bash
# stationary engine: output blocks per MAC thread (HZ_FB_RESP_MAC_R 4 / 8 / 16)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-macab}
mkdir -p "$OUT"
for r in 8 4 16; do
  HZ_FB_RESP_MAC_R=$r timeout -k 10 200 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filterbank_resp_gpu.py -m gpu -k "c2_recipe or lazy" > "$OUT/pytest_$r.log" 2>&1 || { tail -20 "$OUT/pytest_$r.log"; exit 1; }
  HZ_FB_RESP_MAC_R=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$r" -o trace --output-format csv -- \
      python3 bench.py --steps 50 --warmup 4 --no-cpu-baseline --no-traffic --stream-blocks 0 --side-steps 0 > "$OUT/prof_$r.log" 2>&1 || exit $?
  python3 - "$OUT/prof_$r/trace_kernel_stats.csv" $r <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'resp_mac' in r['Name']:
        print('R', sys.argv[2], r['Name'][:40].ljust(42), r['Calls'].rjust(4), '%8.1f' % (float(r['AverageNs']) / 1e3))
PY
done
