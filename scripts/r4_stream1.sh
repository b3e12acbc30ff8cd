set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_fb_stream_gpu.py > gpurun_out/r4_stream1.log 2>&1
