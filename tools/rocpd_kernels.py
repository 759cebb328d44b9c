"""Summarise a rocprofv3 SQLite (rocpd) kernel trace: per (kernel, grid) count and mean us.

    python tools/rocpd_kernels.py gpurun_out/x/run_results.db [regex]
"""
import collections
import re
import sqlite3
import sys


def main():
    db = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, lds_size from kernels order by start").fetchall()
    agg = collections.defaultdict(list)
    for n, d, gx, gy, gz, lds in rows:
        if pat and not pat.search(n):
            continue
        agg[(n[:110], gx, gy, gz, lds)].append(d / 1e3)
    tot = sum(sum(v) for v in agg.values())
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{sum(v):10.1f} us {len(v):5d} x {sum(v)/len(v):9.1f} us  grid={k[1:4]} lds={k[4]}  {k[0]}")
    print(f"total {tot:.1f} us")


if __name__ == "__main__":
    main()
