#!/bin/bash
# Executed floating-point work per row (rocprofv3 --pmc, kernel-trace only): one F64 and one
# F32 counter pass per row; per kernel: dispatches, FMA/MUL/ADD/TRANS wave-instructions and
# MFMA mops, summed over the run.  flops = 64 lanes x (2 FMA + MUL + ADD) + 512 x MFMA_MOPS_F64
# (+ 256 x MFMA_MOPS_F32 is not used here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-flops}; mkdir -p $OUT
for w in ${ROWS:-c2 c3 c4 c5 c6 c7 c8 c9}; do
  for prec in F64 F32; do
    C="SQ_INSTS_VALU_FMA_$prec SQ_INSTS_VALU_MUL_$prec SQ_INSTS_VALU_ADD_$prec SQ_INSTS_VALU_TRANS_$prec SQ_INSTS_VALU_MFMA_MOPS_$prec SQ_WAVES"
    timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d $OUT/${w}_$prec -o pmc --output-format csv -- \
      python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --stream-blocks 0 > $OUT/${w}_$prec.log 2>&1
    rc=$?; echo "$w $prec rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python3 - $OUT <<'PY'
import csv, os, re, sys, collections
out = sys.argv[1]
for row in sorted(d for d in os.listdir(out) if os.path.isdir(os.path.join(out, d))):
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
    for root, _, files in os.walk(os.path.join(out, row)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    m = re.search(r"(\w+)(<[^()]*>)?\(", r["Kernel_Name"])
                    k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:60]
                    agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
    print("==", row)
    for k, c in sorted(agg.items()):
        p = row.split("_")[1]
        fl = 64 * (2 * c.get(f"SQ_INSTS_VALU_FMA_{p}", 0) + c.get(f"SQ_INSTS_VALU_MUL_{p}", 0) + c.get(f"SQ_INSTS_VALU_ADD_{p}", 0))
        fl += (512 if p == "F64" else 256) * c.get(f"SQ_INSTS_VALU_MFMA_MOPS_{p}", 0)
        print(f"  {k:60s} disp {len(disp[k]):4d} flops {fl:.4e} trans {64*c.get(f'SQ_INSTS_VALU_TRANS_{p}',0):.4e}")
PY
