# round 4: streaming engine, per-sample server, speculative blocks -- tests, bench streaming, rocprof
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fb_stream_gpu.py \
  tests/test_rt_server_gpu.py tests/test_lookahead_gpu.py tests/test_filterbank_rt_gpu.py \
  > gpurun_out/r4/pytest_new.log 2>&1 ; echo "pytest rc=$?" >> gpurun_out/r4/pytest_new.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-traffic --no-cpu-baseline --side-steps 0 \
  > gpurun_out/r4/bench_stream.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_stream2 -o s --output-format csv -- \
  python3 bench.py --steps 3 --warmup 2 --no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 469 \
  > gpurun_out/r4/prof_stream2.log 2>&1
