set -o pipefail
mkdir -p gpurun_out/r4/split
cd /tmp && export TMPDIR=/tmp
HZ_FB_SPLIT=16 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/split/trace16 -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-per-sample --stream-blocks 0 --side-steps 0 \
  > $GRAFT_REPO_ROOT/gpurun_out/r4/split/trace16.log 2>&1
