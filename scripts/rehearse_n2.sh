#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: 2 ranks on cuda:0 over gloo (host copies)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp HZ_BENCH_REHEARSAL=1
OUT=gpurun_out/${TAG:-rehearse}
mkdir -p "$OUT"
for extra in "" "--gather"; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NPROC:-2} --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus ${NPROC:-2} --steps 20 --warmup 20 --side-steps 5 --stream-blocks 16 \
      --no-traffic $extra > "$OUT/n2$extra.log" 2>&1
  rc=$?; echo "rc=$rc ($extra)"; grep -h '^{' "$OUT/n2$extra.log" | cut -c1-700
  [ $rc = 0 ] || { tail -30 "$OUT/n2$extra.log"; exit $rc; }
done
