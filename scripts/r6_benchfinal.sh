#!/bin/bash
# Round 6: smoke, the default bench line, its rocprofv3 kernel-trace summary
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/final
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -2 $D/smoke.log
timeout -k 10 500 python -u bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
tail -c 600 $D/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o c2 -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic > $D/prof.log 2>&1 || { tail -20 $D/prof.log; exit 1; }
ls $D/prof
