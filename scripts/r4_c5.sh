# C5: the fused Bowl -> Delaybank block (parity + row bench + kernel stats)
set -o pipefail
mkdir -p gpurun_out/r4/c5
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_chain_gpu.py tests/test_bowl_gpu.py tests/test_delay_gpu.py > gpurun_out/r4/c5/pytest.log 2>&1 || { tail -30 gpurun_out/r4/c5/pytest.log; exit 1; }
tail -2 gpurun_out/r4/c5/pytest.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-traffic > gpurun_out/r4/c5/bench_c5.json 2> gpurun_out/r4/c5/bench_c5.err || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/r4/c5/bench_c5.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], json.dumps(d['block']))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r4/c5/prof -o c5 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 3 --warmup 1 --no-traffic --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r4/c5/prof.log 2>&1
