"""Kernel-trace summary per kernel AND launch size from rocprofv3 *_kernel_trace.csv files.
usage: python scripts/kstats_grid.py <dir> <out.csv>
A row whose kernel runs at several launch sizes per step (C3: 24,000- and 456,000-sample Additive
launches) gets one line per size, so each average is a single bench-sized launch's duration."""
import csv
import glob
import os
import statistics
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    groups = {}
    for r in rows:
        grid = r.get("Grid_Size") or "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        groups.setdefault((r["Kernel_Name"], grid), []).append(dur)
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Grid", "Calls", "TotalDurationNs", "AverageNs", "MedianNs", "MinNs", "MaxNs"])
        for (name, grid), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, grid, len(v), sum(v), sum(v) / len(v), statistics.median(v), min(v), max(v)])


if __name__ == "__main__":
    main()
