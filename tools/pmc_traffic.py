"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch HBM traffic.

    python tools/pmc_traffic.py <dir with pmc_FETCH_SIZE/ and pmc_WRITE_SIZE/> <out.json> <bench-tag> \
        [<config> <per-GPU batch> <frames>]          (default C3 8 861)

The workload is recorded in the summary: bench.py only takes `traffic` from a summary
of the same config, batch and frames as the line it prints.

Units and corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
counters are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B per
lane) coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores.
Every kernel here reads and writes 16 B per lane on its streaming paths.
`traffic_bytes_per_launch` is the mean over all launches of the kernel in the profiled
run (hop-64 and hop-256 launches of the LVC block alike), the same averaging bench.py
uses for `achieved`.  bench.py reads the result as `roofline.traffic`.  `lib_sha16` names the
library the passes ran (run this where they ran): bench.py flags a summary of another build.
"""
import csv
import hashlib
import json
import os
import sys
from collections import defaultdict


def load(path):
    d = defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            d[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return d


def main():
    src, out, tag = sys.argv[1], sys.argv[2], sys.argv[3]
    config, batch, frames = (sys.argv[4], int(sys.argv[5]), int(sys.argv[6])) if len(sys.argv) > 6 else ("C3", 8, 861)
    fetch = load(os.path.join(src, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write = load(os.path.join(src, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    per_grid, tot = [], defaultdict(lambda: [0.0, 0])
    for key in sorted(fetch):
        name, grid = key
        f = sum(fetch[key]) / len(fetch[key]) * 1024 * 2.0      # KiB -> B, gfx950 x2
        w = sum(write.get(key, [0.0])) / max(len(write.get(key, [])), 1) * 1024
        per_grid.append({"kernel": name, "grid": grid, "launches": len(fetch[key]),
                         "fetch_bytes_corrected": f, "write_bytes": w, "traffic_bytes": f + w})
        t = tot[name]
        t[0] += (f + w) * len(fetch[key])
        t[1] += len(fetch[key])
    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "prodiff_amd", "libprodiff_hip.so")
    lib = os.environ.get("PRODIFF_HIP_LIB", lib)
    try:
        sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    except OSError:
        sha = None
    res = {"bench_tag": tag, "lib_sha16": sha, "config": config, "batch": batch, "frames": frames, "units": "bytes per launch (FETCH_SIZE KiB x1024 x2 + WRITE_SIZE KiB x1024)",
           "per_grid": per_grid,
           "kernels": {k: {"traffic_bytes_per_launch": v[0] / v[1], "launches": v[1]} for k, v in tot.items()}}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, v in res["kernels"].items():
        print(f"{v['traffic_bytes_per_launch'] / 1e6:10.1f} MB/launch  {k[:90]}")


if __name__ == "__main__":
    main()
