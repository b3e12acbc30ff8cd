set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_rt_server_gpu.py tests/test_lookahead_gpu.py tests/test_filterbank_rt_gpu.py tests/test_cpp_gpu.py \
  > gpurun_out/r4/pytest_rt.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r4/pytest_rt.log
