#!/bin/bash
# per-sample server with the device request line: every per-sample test, then the rt_midi latency
# probe with the device line (default) and the pinned host line (HZ_RT_HOST_MAILBOX=1), alternating
set -o pipefail
OUT=gpurun_out/r4/mailbox
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_rt_server_gpu.py \
  tests/test_filterbank_rt_gpu.py tests/test_delay_gpu.py tests/test_granulator_gpu.py tests/test_cpp_gpu.py \
  tests/test_lookahead_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  timeout -k 10 100 python3 scripts/probe/rt_midi_lat.py $OUT/dev$i 500 > $OUT/dev$i.log 2>&1 || exit 1
  HZ_RT_HOST_MAILBOX=1 timeout -k 10 100 python3 scripts/probe/rt_midi_lat.py $OUT/host$i 500 > $OUT/host$i.log 2>&1 || exit 1
done
for f in dev1 host1 dev2 host2; do echo "$f: $(grep -E '^all|^first' $OUT/$f.log | tr '\n' ' ')"; done
