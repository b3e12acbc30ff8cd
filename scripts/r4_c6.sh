set -o pipefail
OUT=gpurun_out/r4/c6
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_granulator_gpu.py tests/test_rt_server_gpu.py -k "gran or Gran" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --workload c6 --steps 10 --warmup 2 --no-traffic > $OUT/bench_c6.json 2> $OUT/bench_c6.err || exit 1
HZ_GRAN_LIBCOS=1 timeout -k 10 300 python -u bench.py --workload c6 --steps 10 --warmup 2 --no-traffic --no-cpu-baseline > $OUT/bench_c6_libcos.json 2>> $OUT/bench_c6.err || exit 1
for f in bench_c6 bench_c6_libcos; do python -c "
import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', d['value'], d['ms_per_step'], r['frac'])"; done
