"""Summarise the churn pass of a kernel trace (scripts/r6_churn2.sh): span per block, per-kernel
durations, the gaps between kernel pairs, the one-time per-band response kernels."""
import collections
import csv
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "stream_block_kernel<6, true>" in r["Kernel_Name"]]
seg = rows[idx[0] - 1:idx[-1] + 1]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
print(f"churn pass: span {(t1 - t0) / 1e3:.1f} us over {len(idx)} DUAL blocks = {(t1 - t0) / 1e3 / len(idx):.2f} us per block")
dur = collections.defaultdict(list)
for r in seg:
    dur[r["Kernel_Name"][:70]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in dur.items():
    print(f"  {k:70s} n={len(v):4d} mean {np.mean(v):7.2f} median {np.median(v):7.2f} us")
gaps = collections.defaultdict(list)
for p, q in zip(seg, seg[1:]):
    gaps[(p["Kernel_Name"][:36], q["Kernel_Name"][:36])].append(
        (int(q["Start_Timestamp"]) - int(p["End_Timestamp"])) / 1e3)
for k, v in gaps.items():
    print(f"  gap {k[0]} -> {k[1]}: n={len(v)} mean {np.mean(v):.2f} us")
for r in rows:
    if any(s in r["Kernel_Name"] for s in ("rbasis", "rspec", "rband")):
        print("  one-time", r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, "us")
