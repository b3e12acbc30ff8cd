#!/bin/bash
# stationary engine: radix-8 (512 threads) vs radix-4 (1024 threads) FFT workgroups
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-radix}
mkdir -p "$OUT"
HZ_FB_RESP_RADIX=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filterbank_resp_gpu.py -m gpu > "$OUT/pytest4.log" 2>&1 || { tail -20 "$OUT/pytest4.log"; exit 1; }
tail -1 "$OUT/pytest4.log"
for r in 8 4; do
  HZ_FB_RESP_RADIX=$r timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$r" -o trace --output-format csv -- \
      python3 bench.py --steps 50 --warmup 4 --no-cpu-baseline --no-traffic --stream-blocks 0 --side-steps 0 > "$OUT/prof_$r.log" 2>&1 || exit $?
  python3 - "$OUT/prof_$r/trace_kernel_stats.csv" $r <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'resp_fwd' in r['Name'] or 'resp_inv' in r['Name']:
        print('radix', sys.argv[2], r['Name'][:40].ljust(42), r['Calls'].rjust(4), '%8.1f' % (float(r['AverageNs']) / 1e3))
PY
done
