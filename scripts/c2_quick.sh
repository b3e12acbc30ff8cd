#!/bin/bash
# C2 iteration loop: LTI parity tests, then a C2 bench line and rocprof kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c2q}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_filterbank_lti_gpu.py ${TESTS:-} > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/bench.log 2>&1
rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/bench.log; exit $rc; }
python3 -c "
import json; l=[x for x in open('$OUT/bench.log') if x.startswith('{')][-1]; d=json.loads(l); r=d['roofline']
print('C2 ms/step %.4f value %.3e kernel_ms %.4f comps %s' % (d['ms_per_step'], d['value'], r['kernel_avg_ms'], r['components_ms_per_launch']))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- \
   python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/prof.log 2>&1
rc=$?; echo rocprof rc=$rc
python3 - <<PY
import csv, glob
for f in glob.glob("$OUT/prof/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if "fb_lti" in n or "sum_kernel" in n or "xrows" in n:
            print("  %-40s %6s calls %8.1f us" % (n[n.find("fb_"):n.find("(", n.find("fb_"))], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
