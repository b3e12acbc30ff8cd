#!/bin/bash
# Round 6: C3 (Additive, 256 overtones x voices over the ranks) per-rank step emulated on one MI355X
# (rank 0's overtone shard of P, no reduce), P = 1, 2, 4, 8 -- VERDICT r5 item 1
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/r6/c3emul
mkdir -p $OUT
export TMPDIR=/tmp
for P in 1 2 4 8; do
  timeout -k 10 240 python3 -u bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic \
      --emulate-world $P > $OUT/c3_p$P.json 2> $OUT/c3_p$P.err || exit $?
  python3 -c "
import json,sys
d=json.loads([l for l in open('$OUT/c3_p$P.json') if l.startswith('{')][-1])
print('P=$P', 'ms/step %.4f' % d['ms_per_step'], 'value %.3e' % d['value'], 'emulated', d.get('emulated_world'))
"
done
