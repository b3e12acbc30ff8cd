# C4: one frame per workgroup (stft_half4096_kernel, HZ_STFT_FRAME=half) against the pair kernel
# (HZ_STFT_FRAME=pair): STFT parity suites for both, then alternating bench runs on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r5/half
mkdir -p $OUT
HZ_STFT_FRAME=half timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stft_gpu.py tests/test_stft_slots_gpu.py tests/test_fullsize_gpu.py -k "stft or c4 or STFT" > $OUT/pytest_half.log 2>&1 || { tail -30 $OUT/pytest_half.log; exit 1; }
tail -2 $OUT/pytest_half.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stft_gpu.py tests/test_stft_slots_gpu.py tests/test_fullsize_gpu.py -k "stft or c4 or STFT" > $OUT/pytest_pair.log 2>&1 || { tail -30 $OUT/pytest_pair.log; exit 1; }
tail -2 $OUT/pytest_pair.log
for i in 1 2 3; do
  for v in half pair; do
    export HZ_STFT_FRAME=$v
    timeout -k 10 300 python -u bench.py --workload c4 --steps 40 --warmup 3 --no-traffic --no-cpu-baseline > $OUT/b_${v}_$i.json 2>$OUT/b_${v}_$i.err || { tail -5 $OUT/b_${v}_$i.err; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/b_${v}_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v $i step', round(d['ms_per_step']*1e3,2), 'frame', round(r['kernel_ms_per_step']*1e3,2), 'ola', round(r['ola_ms_per_step']*1e3,2), 'frac', round(r['frac'],3))"
  done
done
