set -o pipefail
mkdir -p gpurun_out/r4/e2e
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_fb_stream_gpu.py tests/test_bench_contract_gpu.py > gpurun_out/r4/e2e/pytest.log 2>&1 || { tail -30 gpurun_out/r4/e2e/pytest.log; exit 1; }
tail -1 gpurun_out/r4/e2e/pytest.log
timeout -k 10 300 python -u bench.py --steps 50 --no-cpu-baseline --no-traffic --no-per-sample --side-steps 0 > gpurun_out/r4/e2e/bench.json 2> gpurun_out/r4/e2e/bench.err || exit 1
python -c "
import json;d=json.loads(open('gpurun_out/r4/e2e/bench.json').read().strip().splitlines()[-1]);s=d['streaming'];print(s['us_per_block'], s['end_to_end_host_buffers'])"
