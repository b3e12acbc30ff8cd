"""Mean PMC counter values per kernel from rocprofv3 --pmc csv output (counter_collection.csv).
usage: python scripts/pmc_summary.py <dir> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys


def main():
    files = glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True)
    pats = sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if pats and not any(p in name for p in pats):
                    continue
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, cs in acc.items():
        print(name[:100])
        for c, v in sorted(cs.items()):
            print(f"    {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
