#!/bin/bash
# STFT frame-kernel check: GPU parity tests, bench c4, and a rocprofv3 kernel-stats pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-stft}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_stft_gpu.py tests/test_cpp_gpu.py \
    > "$OUT/pytest_stft.log" 2>&1 || { tail -20 "$OUT/pytest_stft.log"; exit 1; }
tail -2 "$OUT/pytest_stft.log"
timeout -k 10 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline ${C4_ARGS:-} \
    > "$OUT/bench_c4.log" 2>&1 || { tail -5 "$OUT/bench_c4.log"; exit 1; }
tail -1 "$OUT/bench_c4.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c4" -o trace --output-format csv -- \
    python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof_c4.log" 2>&1 || exit 1
grep -h "stft" $(find "$OUT/prof_c4" -name "*kernel_stats.csv") | cut -c1-160
exit 0
