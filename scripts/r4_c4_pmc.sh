# C4 frame kernel counters: wave-cycle breakdown, LDS conflicts, instruction mix (separate passes)
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/r4/c4pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$i -o c4 -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 3 --warmup 1 --no-traffic --no-cpu-baseline > $OUT/p$i.log 2>&1 || exit 1
  i=$((i+1))
done
