#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
n=0
for i in 1 2 3 4 5 6 7 8 9 10; do
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_filterbank_resp_gpu.py > /tmp/f.log 2>&1 || { n=$((n+1)); grep -E "^E  |FAILED" /tmp/f.log | head -3; }
done
echo "$n failing file runs of 10"
