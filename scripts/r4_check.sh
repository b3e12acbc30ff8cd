# round-4 check: Filterbank GPU tests, a short bench, rocprof kernel stats of the streaming blocks
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_fb_stream_gpu.py tests/test_filterbank_resp_gpu.py tests/test_c2_pinned_gpu.py tests/test_filterbank_gpu.py \
  tests/test_filterbank_lti_gpu.py tests/test_filterbank_rt_gpu.py tests/test_bench_contract_gpu.py tests/test_cpp_gpu.py \
  > gpurun_out/r4/pytest_fb.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-traffic --no-cpu-baseline > gpurun_out/r4/bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd - && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4/prof_stream -o s --output-format csv -- \
  python3 bench.py --steps 3 --warmup 2 --no-traffic --no-cpu-baseline --no-per-sample --side-steps 0 --stream-blocks 469 \
  > gpurun_out/r4/prof_stream.log 2>&1
