set -o pipefail
mkdir -p gpurun_out/r4/pipe
for m in 0 1 2; do
  if [ $m = 1 ]; then export HZ_FB_PIPE_HACK=1; fi
  if [ $m = 2 ]; then export HZ_FB_PIPE_HACK2=1; fi
  timeout -k 10 240 python -u bench.py --steps 200 --no-cpu-baseline --no-traffic --no-per-sample --stream-blocks 0 --side-steps 0 \
    > gpurun_out/r4/pipe/bench_$m.json 2> gpurun_out/r4/pipe/bench_$m.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r4/pipe/bench_$m.json').read().strip().splitlines()[-1]);print('hack $m', d['ms_per_step'])"
done
