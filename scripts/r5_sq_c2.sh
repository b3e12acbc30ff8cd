# SQ / TCC counters of the C2 step's three kernels (per-wave instruction mix, waits)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_ANY"
G2="TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
TAG=${TAG:-sq_c2} bash scripts/sq.sh "$G1" "$G2" > gpurun_out/${TAG:-sq_c2}.txt 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/${TAG:-sq_c2} resp_ > gpurun_out/${TAG:-sq_c2}_summary.txt
cat gpurun_out/${TAG:-sq_c2}_summary.txt
