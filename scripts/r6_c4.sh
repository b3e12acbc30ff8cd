#!/bin/bash
# Round 6: C4 (StaticSTFT 4096 x 4 laps) -- parity and the row line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/c4
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_stft_gpu.py "tests/test_fullsize_gpu.py::test_c4_full_length" > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for r in 1 2; do
timeout -k 10 300 python3 -u bench.py --workload c4 --steps 20 --warmup 3 ${EXTRA} > $D/bench_c4_$r.json 2> $D/bench_c4_$r.err || { tail -20 $D/bench_c4_$r.err; exit 1; }
python3 - $D/bench_c4_$r.json <<'PY'
import json, sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
r=d["roofline"]
print("C4 ms/step %.4f value %.3e" % (d["ms_per_step"], d["value"]), "frac", r.get("frac"), "kernel ms", r.get("kernel_avg_ms"), r.get("kernel"))
PY
EXTRA="--no-cpu-baseline --no-traffic"
done
