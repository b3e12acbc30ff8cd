#!/bin/bash
# Round 5, first GPU pass: the advisor regression tests, a bench.py --gpus 2 rehearsal through the
# built-in launcher (no manual torchrun), a one-GPU bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/r5/first
mkdir -p "$OUT"
echo "== new tests"; date
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
   tests/test_fb_stream_gpu.py tests/test_rt_server_gpu.py -k "shrinks or mix_mid or beyond_server or exact_config or small_bank" \
   > "$OUT/pytest_new.log" 2>&1
rc=$?; tail -12 "$OUT/pytest_new.log"; echo "pytest rc=$rc"
[ $rc = 0 ] || [ $rc = 1 ] || exit $rc
echo "== rehearsal bench.py --gpus 2"; date
HZ_BENCH_REHEARSAL=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --no-traffic \
   --no-cpu-baseline --no-per-sample --side-steps 5 --stream-blocks 16 > "$OUT/rehearse_c2_n2.json" 2> "$OUT/rehearse_c2_n2.err"
rc=$?; cut -c1-800 "$OUT/rehearse_c2_n2.json"; echo "rehearsal rc=$rc"; [ $rc = 0 ] || { tail -30 "$OUT/rehearse_c2_n2.err"; exit $rc; }
echo "== bench N=1"; date
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-traffic --no-per-sample --no-cpu-baseline \
   > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err"
rc=$?; cut -c1-600 "$OUT/bench_n1.json"; echo "bench rc=$rc"
exit $rc
