# default bench line (N = 1) + its rocprof kernel stats
set -o pipefail
OUT=gpurun_out/r4/bench
mkdir -p $OUT
timeout -k 10 900 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 600 $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o c2 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-traffic --no-cpu-baseline --no-per-sample > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
