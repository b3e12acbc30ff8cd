"""Per-kernel duration summary from a rocprofv3 rocpd database (or kernel_stats.csv).
usage: python scripts/kstats.py <run_results.db | dir> [--grid] [name-substring ...]
(--grid: one line per kernel and grid size)"""
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    if os.path.isdir(path):
        dbs = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
        path = dbs[0]
    c = sqlite3.connect(path)
    args = sys.argv[2:]
    grid = "--grid" in args
    pats = [a for a in args if a != "--grid"]
    key = "name, grid_x, grid_y" if grid else "name"
    sel = key if grid else "name, 0, 0"
    rows = c.execute(f"select {sel}, count(*), avg(end - start), min(end - start), sum(end - start) from kernels "
                     f"group by {key} order by name, sum(end - start) desc").fetchall()
    rows.sort(key=lambda r: -r[6] if not grid else 0)
    print(f"{'calls':>6} {'avg_us':>9} {'min_us':>9} {'total_ms':>9} {'grid':>12}  kernel")
    for name, gx, gy, n, avg, mn, tot in rows:
        if pats and not any(p in name for p in pats):
            continue
        gs = f"{gx}x{gy}" if grid else ""
        print(f"{n:6d} {avg / 1e3:9.2f} {mn / 1e3:9.2f} {tot / 1e6:9.3f} {gs:>12}  {name[:100]}")


if __name__ == "__main__":
    main()
