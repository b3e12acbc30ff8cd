#!/bin/bash
# (A/B) Additive groups per call: HZ_ADD_GROUPS = 1 (every task in every workgroup), 4, 19 (one task per wave)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
D=gpurun_out/r6/c3ab
mkdir -p $D
export TMPDIR=/tmp
for g in 19 1 4 2 19 1; do
  HZ_ADD_GROUPS=$g timeout -k 10 200 python3 -u bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline --no-traffic > $D/g$g.json 2> $D/g$g.err || { tail -5 $D/g$g.err; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('$D/g$g.json') if l.startswith('{')][-1])
print('groups $g: C3 ms/step %.4f' % d['ms_per_step'])"
done
