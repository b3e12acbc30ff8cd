# same-box A/B: band-state workgroups dispatched before / after the inverse transforms
set -o pipefail
OUT=gpurun_out/r4/statefirst
mkdir -p $OUT
for i in 1 2 3; do
  for v in after first; do
    if [ $v = first ]; then export HZ_FB_STATE_FIRST=1; else unset HZ_FB_STATE_FIRST; fi
    timeout -k 10 240 python -u bench.py --steps 200 --no-cpu-baseline --no-traffic --no-per-sample --stream-blocks 0 --side-steps 0 \
      > $OUT/b_${v}_$i.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads(open('$OUT/b_${v}_$i.json').read().strip().splitlines()[-1]);print('$v $i', d['ms_per_step'], d['roofline']['kernel_avg_ms'])"
  done
done
HZ_FB_STATE_FIRST=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_c2_pinned_gpu.py tests/test_filterbank_resp_gpu.py > $OUT/pytest.log 2>&1; tail -1 $OUT/pytest.log
