#!/bin/bash
# C4 evidence: kernel trace (overlap-add cold vs warm via HZ_STFT_OLA_REPEAT=2) and SQ/TCC
# counter passes on the pair and overlap-add kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-c4prof}
mkdir -p "$OUT"
B="python3 bench.py --workload c4 --steps 20 --warmup 2 --no-cpu-baseline --no-traffic"
HZ_STFT_OLA_REPEAT=2 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- \
    $B > "$OUT/kt.log" 2>&1 || { echo "kt failed"; tail -5 "$OUT/kt.log"; exit 1; }
find "$OUT/kt" -name "*kernel_stats.csv" -exec cat {} \;
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_ANY"
G2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR"
i=0
for grp in "$G1" "$G2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace -d "$OUT/p$i" -o pmc --output-format csv -- \
      python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-traffic > "$OUT/p$i.log" 2>&1
  rc=$?; echo "pass $i rc=$rc"
  case $rc in 0) ;; *) tail -3 "$OUT/p$i.log"; exit $rc;; esac
done
python3 scripts/pmc_summary.py "$OUT" stft_ | tee "$OUT/pmc_summary.txt"
exit 0
