#!/bin/bash
# Round 6: Additive (C3) with one group per call -- parity tests and the C3 row with PMC evidence
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/c3
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_additive_gpu.py \
   "tests/test_fullsize_gpu.py::test_c3_full_length" tests/test_cpp_gpu.py > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python3 -u bench.py --workload c3 --steps 20 --warmup 3 > $D/bench_c3.json 2> $D/bench_c3.err || { tail -20 $D/bench_c3.err; exit 1; }
python3 - <<'PY'
import json
d=json.loads([l for l in open("gpurun_out/r6/c3/bench_c3.json") if l.startswith("{")][-1])
r=d["roofline"]
print("C3 ms/step %.4f value %.3e" % (d["ms_per_step"], d["value"]), "frac", r.get("frac"), "traffic", r.get("traffic"))
ev=r.get("pmc_evidence") or {}
print({k: ev.get(k) for k in ("traffic_bytes","algorithmic_bytes","traffic_over_algorithmic","seconds","fracs","binding_pipe")})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c3 -- python3 bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline --no-traffic > $D/prof.log 2>&1 || exit 1
head -5 $D/prof/c3_kernel_stats.csv | cut -c1-150
