#!/bin/bash
# Round-end C2 evidence: the GPU suite, smoke, the default bench line (PMC traffic + flops, CPU
# legs), then a clean rocprofv3 kernel trace of the timed steps only (no side figures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
TAG=${TAG:-final} PYTEST_TIMEOUT=600 PYTEST_ARGS="--timeout 300 --timeout-method thread" PROFILE= \
    bash scripts/gpu_check.sh || exit $?
OUT=gpurun_out/${TAG:-final}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_clean" -o trace --output-format csv -- \
    python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-traffic --no-per-sample --side-steps 0 \
    --stream-blocks 0 > "$OUT/prof_clean.log" 2>&1
rc=$?; echo "clean rocprof rc=$rc"
exit $rc
