#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
F=tests/test_filterbank_resp_gpu.py
for prev in test_time_range_shards test_c2_full_size_against_lti test_shards_sum; do
  n=0
  for i in 1 2 3 4 5 6; do
    timeout -k 10 120 python -u -m pytest -q --timeout 60 --timeout-method thread -p no:cacheprovider "$F::$prev" "$F::test_stream_and_per_sample_after_stationary" > /tmp/o.log 2>&1 || n=$((n+1))
  done
  echo "$prev then the stream test: $n failing runs of 6"
done
