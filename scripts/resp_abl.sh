#!/bin/bash
# stationary engine: kernel times with / without the FFT passes (HZ_FB_RESP_ABL=1, wrong results)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-respabl}
mkdir -p "$OUT"
for a in 0 1; do
  HZ_FB_RESP_ABL=$a timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$a" -o trace --output-format csv -- \
      python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --no-traffic --stream-blocks 0 --side-steps 0 > "$OUT/prof_$a.log" 2>&1 || exit $?
  python3 - "$OUT/prof_$a/trace_kernel_stats.csv" $a <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'resp_' in r['Name'] or '128, 1' in r['Name']:
        print('abl', sys.argv[2], r['Name'][:50].ljust(52), r['Calls'].rjust(4), '%8.1f' % (float(r['AverageNs']) / 1e3))
PY
done
