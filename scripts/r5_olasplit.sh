# C4 overlap-add: one workgroup per segment (default) against two (HZ_STFT_OLA_SPLIT=2):
# STFT parity with the split, then alternating bench runs on one box
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r5/olasplit
mkdir -p $OUT
HZ_STFT_OLA_SPLIT=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stft_gpu.py tests/test_stft_slots_gpu.py tests/test_fullsize_gpu.py -k "stft or c4 or STFT" > $OUT/pytest_split4.log 2>&1 || { tail -30 $OUT/pytest_split4.log; exit 1; }
tail -1 $OUT/pytest_split4.log
for i in 1 2 3; do
  for v in 1 2 4; do
    export HZ_STFT_OLA_SPLIT=$v
    timeout -k 10 300 python -u bench.py --workload c4 --steps 40 --warmup 3 --no-traffic --no-cpu-baseline > $OUT/b_${v}_$i.json 2>$OUT/b_${v}_$i.err || { tail -5 $OUT/b_${v}_$i.err; exit 1; }
    python -c "import json;d=json.loads(open('$OUT/b_${v}_$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('split $v $i step', round(d['ms_per_step']*1e3,2), 'frame', round(r['kernel_ms_per_step']*1e3,2), 'ola', round(r['ola_ms_per_step']*1e3,2))"
  done
done
