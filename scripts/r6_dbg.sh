#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for i in 1 2 3 4 5 6 7 8; do
HZ_TEST_STATE_FIRST=1 timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_filterbank_resp_gpu.py > /tmp/f.log 2>&1 || { grep -E "^E  |FAILED" /tmp/f.log | head -4; }
done
echo done
