#!/bin/bash
# stationary engine: GPU tests, then C2 emulated shard steps (time-sharded at P > 1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-respchk}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_filterbank_resp_gpu.py -m gpu > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc = 0 ] || exit $rc
for P in ${WORLDS:-1 2 4 8}; do
  timeout -k 10 200 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-traffic --stream-blocks 0 \
      --side-steps 0 --emulate-world $P > "$OUT/emul_$P.log" 2>&1
  rc=$?; [ $rc = 0 ] || { tail -5 "$OUT/emul_$P.log"; exit $rc; }
  python - "$OUT/emul_$P.log" $P <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("P=%s ms/step %.4f engine %s comps %s" % (sys.argv[2], d["ms_per_step"], d.get("engine"), r["components_ms_per_launch"]))
PY
done
