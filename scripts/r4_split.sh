# split-chip stationary step: the band-state pass and the transforms on complementary CU masks
set -o pipefail
mkdir -p gpurun_out/r4/split
run() {  # split mode tag
  HZ_FB_SPLIT=$1 HZ_FB_SPLIT_MODE=$2 timeout -k 10 240 python -u bench.py --steps 200 --no-cpu-baseline --no-traffic --no-per-sample \
    --stream-blocks 0 --side-steps 0 > gpurun_out/r4/split/bench_$3.json 2> gpurun_out/r4/split/bench_$3.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/r4/split/bench_$3.json').read().strip().splitlines()[-1]);print('split $1 mode $2', d['ms_per_step'], d['value'])"
}
for s in 8 16 24; do run $s 5 s${s}m5; run $s 6 s${s}m6; run $s 2 s${s}m2; done
