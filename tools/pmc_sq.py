"""Summarise tools/pmc_sq.sh passes: per-launch means and per-wave ratios per (kernel, grid).
    python tools/pmc_sq.py gpurun_out/<tag>"""
import csv
import glob
import os
import sys
from collections import defaultdict

d = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(sys.argv[1], "sq*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        d[(r["Kernel_Name"].split("(")[0][-80:] + r["Kernel_Name"][r["Kernel_Name"].find("<"):r["Kernel_Name"].find(">") + 1],
           int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, g), c in d.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = m.get("SQ_WAVES", 0) or 1
    print(f"== {k} grid={g}")
    for n in sorted(m):
        print(f"   {n:28s} {m[n]:16.1f}   per wave {m[n] / w:12.1f}")
    if "SQ_WAVE_CYCLES" in m:
        wc = m["SQ_WAVE_CYCLES"]
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
            if n in m:
                print(f"   {n} / WAVE_CYCLES = {m[n] / wc:.3f}")
