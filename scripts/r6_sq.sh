#!/bin/bash
# Round 6: SQ / TCC counters of the FINAL kernels -- the C2 stationary step (resp_fwd_kernel,
# resp_mac_kernel_lds<24,8>, resp_inv_kernel<0>) and the general engine on &softclip calls
# (fb_mix_kernel<2,SOFTCLIP,...>) -- one rocprofv3 --pmc pass per counter group.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_ANY"
G2="TCC_HIT_sum TCC_MISS_sum SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM"
G3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
COMMON="--no-per-sample --side-steps 0 --no-general-side"
TAG=r6/sq_c2 BENCH_ARGS="$COMMON" bash scripts/sq.sh "$G1" "$G2" "$G3" > gpurun_out/r6/sq_c2.txt 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/r6/sq_c2 resp_ > gpurun_out/r6/sq_c2_summary.txt
TAG=r6/sq_soft BENCH_ARGS="$COMMON --dist softclip" bash scripts/sq.sh "$G1" "$G2" "$G3" > gpurun_out/r6/sq_soft.txt 2>&1 || exit 1
python3 scripts/pmc_summary.py gpurun_out/r6/sq_soft fb_ > gpurun_out/r6/sq_soft_summary.txt
cat gpurun_out/r6/sq_c2_summary.txt gpurun_out/r6/sq_soft_summary.txt | head -120
