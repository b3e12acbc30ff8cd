#!/bin/bash
# Rehearsal of bench.py's N > 1 paths on a one-GPU box (C2, C3, C4 at world 2): 2 ranks on cuda:0,
# the collectives over gloo through host copies (HZ_BENCH_REHEARSAL=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp HZ_BENCH_REHEARSAL=1
OUT=gpurun_out/r4/rehearse
mkdir -p "$OUT"
port=29531
for w in c2 c3 c4; do
  extra="--no-traffic --no-cpu-baseline"
  [ $w = c2 ] && extra="$extra --side-steps 5 --stream-blocks 16"
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port $port bench.py --gpus 2 --workload $w --steps 10 --warmup 5 $extra > "$OUT/$w-n2.log" 2>&1
  rc=$?; echo "rc=$rc ($w)"; grep -h '^{' "$OUT/$w-n2.log" | cut -c1-600
  [ $rc = 0 ] || { tail -30 "$OUT/$w-n2.log"; exit $rc; }
  port=$((port + 1))
done
