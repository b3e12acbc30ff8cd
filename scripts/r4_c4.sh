# C4: the specialised 4096-point pair kernel (parity, A/B against the generic pair kernel, stats)
set -o pipefail
OUT=gpurun_out/r4/c4
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_stft_gpu.py tests/test_stft_slots_gpu.py tests/test_freezer_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
HZ_STFT_GENERIC_PAIR=1 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-traffic --no-cpu-baseline > $OUT/bench_c4_generic.json 2>> $OUT/bench_c4.err || exit 1
for f in bench_c4 bench_c4_generic; do python -c "
import json;d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', d['ms_per_step'], r['frac'], r['kernel_ms_per_step'], r.get('traffic'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o c4 -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 10 --warmup 2 --no-traffic --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"
i=1
for P in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $GRAFT_REPO_ROOT/$OUT/p$i -o c4 -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 3 --warmup 1 --no-traffic --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/p$i.log 2>&1 || exit 1
  i=$((i+1))
done
