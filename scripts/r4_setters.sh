#!/bin/bash
# per-sample setter path: parity tests, then the per-sample latency around setters
set -o pipefail
mkdir -p gpurun_out/r4/setters
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_filterbank_rt_gpu.py tests/test_rt_server_gpu.py tests/test_filterbank_lti_gpu.py tests/test_filterbank_gpu.py \
  tests/test_cpp_gpu.py > gpurun_out/r4/setters/pytest.log 2>&1 && \
timeout -k 10 200 python3 scripts/probe/rt_midi_lat.py gpurun_out/r4/setters/midi 500 > gpurun_out/r4/setters/midi.log 2>&1
rc=$?
tail -3 gpurun_out/r4/setters/pytest.log; cat gpurun_out/r4/setters/midi.log
exit $rc
