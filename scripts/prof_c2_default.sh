#!/bin/bash
# rocprofv3 kernel stats of the default C2 bench (200 timed steps, 20 warmup)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof_c2d}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o trace --output-format csv -- \
   python3 bench.py --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/log 2>&1 || exit 1
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"
G2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_LDS"
TAG=sq_c3 BENCH_ARGS="--workload c3" bash scripts/sq.sh "$G1" "$G2" > gpurun_out/sq_c3.txt 2>&1 && \
TAG=sq_c4 BENCH_ARGS="--workload c4" bash scripts/sq.sh "$G1" "$G2" > gpurun_out/sq_c4.txt 2>&1
