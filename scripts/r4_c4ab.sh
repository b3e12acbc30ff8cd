# same-box A/B of the pair4096 kernel's radix-8 form (twiddle once vs stage-wise), alternating
set -o pipefail
OUT=gpurun_out/r4/c4ab
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stft_gpu.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
HZ_STFT_TWIDDLE_ONCE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stft_gpu.py >> $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
grep passed $OUT/pytest.log
for i in 1 2 3; do
  for v in once stage; do
    if [ $v = once ]; then export HZ_STFT_TWIDDLE_ONCE=1; else unset HZ_STFT_TWIDDLE_ONCE; fi
    timeout -k 10 300 python -u bench.py --workload c4 --steps 40 --warmup 3 --no-traffic --no-cpu-baseline > $OUT/b_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('$OUT/b_${v}_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v $i', r['kernel_ms_per_step'], r['frac'])"
  done
done
