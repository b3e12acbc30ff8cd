#!/bin/bash
# (A/B) the long-horizon MAC's blocks per thread (HZ_MACC_BPW = 8, 4, 2), alternating, then the high-Q tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/hqab
mkdir -p $D
for b in 1 4 2 1 4 2; do
  echo "SPLIT $b: $(HZ_MACC_SPLIT=$b timeout -k 10 200 python3 -u scripts/r6_hq.py 2>/dev/null | tail -1)"
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_fb_highq_gpu.py "tests/test_fullsize_gpu.py::test_c2_high_q_stationary_and_blocks" tests/test_fb_modal_gpu.py > $D/pytest.log 2>&1; tail -1 $D/pytest.log
