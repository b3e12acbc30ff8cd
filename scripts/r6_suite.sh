#!/bin/bash
# Round 6: the whole GPU suite on the final library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/final
mkdir -p $D
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest_gpu.log 2>&1
rc=$?
tail -5 $D/pytest_gpu.log
exit $rc
