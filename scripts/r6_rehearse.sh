#!/bin/bash
# Round 6 end: one-GPU rehearsal of bench.py --gpus 2 (both ranks on cuda:0, collectives over gloo
# through host copies) on the final engines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/r6/rehearse
mkdir -p $OUT
export TMPDIR=/tmp
HZ_BENCH_REHEARSAL=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline --no-traffic \
   --stream-blocks 32 --side-steps 20 > $OUT/c2_n2.json 2> $OUT/c2_n2.err || { tail -20 $OUT/c2_n2.err; exit 1; }
python3 -c "
import json
d=json.loads([l for l in open('$OUT/c2_n2.json') if l.startswith('{')][-1])
print('n_gpus', d['n_gpus'], 'ms/step %.4f' % d['ms_per_step'], 'value %.3e' % d['value'], d.get('scaling'))"
