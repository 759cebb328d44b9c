"""Per-kernel MFMA / VALU utilisation from tools/pmc_sq.sh passes -> JSON.

    python tools/sq_summary.py gpurun_out/<tag> [--config C3] [--top 6] [-o profiles/rNN_c3_sq.json]

Counters (rocprofv3, gfx950; MI355X_MICROARCH.md "rocprofv3 PMC slots" and the cycle-constant
table): SQ_VALU_MFMA_BUSY_CYCLES counts matrix-pipe cycles summed over SIMDs (32 per
32x32x16 bf16 MFMA); SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed
over waves; GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Per launch:
  cycles       = GRBM_GUI_ACTIVE / 8                 (the launch's span in shader cycles)
  mfma_busy    = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles)
  valu_busy    = 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x cycles)
  wait_any     = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (parked on s_waitcnt / s_barrier)
  wait_inst    = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (issue stalls: dependencies, busy pipes)
  active       = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
Kernels are keyed by name and template arguments; launches of every grid size are summed.
GRBM_GUI_ACTIVE includes the dispatch ramp, so on launches of a few tens of microseconds the
fractions read low by a few percent.
"""
import argparse
import csv
import glob
import hashlib
import json
import os
from collections import defaultdict

SIMDS = 1024


def short(name):
    base = name.replace("(anonymous namespace)::", "").replace("pd::", "").replace("void ", "")
    return base.split("(")[0].strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--config", default=None)
    ap.add_argument("--top", type=int, default=8)
    ap.add_argument("-o", default=None)
    a = ap.parse_args()
    # (kernel, dispatch) -> counter -> value; durations from the first pass
    per = defaultdict(dict)
    dur = {}
    for f in sorted(glob.glob(os.path.join(a.dir, "sq*", "run_counter_collection.csv"))):
        p = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            key = (p, k, r["Dispatch_Id"])
            per[key][r["Counter_Name"]] = per[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            per[key]["_dur_ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            per[key]["_vgpr"] = int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"])
            per[key]["_lds"] = int(r["LDS_Block_Size"])
    tot = defaultdict(lambda: defaultdict(float))
    n = defaultdict(lambda: defaultdict(int))
    meta = {}
    for (p, k, _), c in per.items():
        for cn, v in c.items():
            if cn.startswith("_"):
                continue
            tot[k][cn] += v
            n[k][cn] += 1
        tot[k]["_dur_ns@" + p] += c["_dur_ns"]
        n[k]["_dur_ns@" + p] += 1
        meta[k] = (c["_vgpr"], c["_lds"])
    rows = []
    for k, t in tot.items():
        m = {cn: t[cn] / n[k][cn] for cn in t}           # per-launch means
        durs = [m[x] for x in m if x.startswith("_dur_ns@")]
        launches = max(n[k][x] for x in n[k] if x.startswith("_dur_ns@"))
        avg_us = min(durs) / 1e3 if durs else None
        cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        waves = m.get("SQ_WAVES", 0.0) or 1.0
        row = dict(kernel=k, launches_profiled=launches, avg_us_profiled=round(avg_us, 2) if avg_us else None,
                   vgpr=meta[k][0], lds_bytes=meta[k][1], waves_per_launch=round(waves))
        if cyc:
            row["cycles_per_launch"] = round(cyc)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                row["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * cyc), 4)
            if "SQ_ACTIVE_INST_VALU" in m:
                row["valu_busy"] = round(4 * m["SQ_ACTIVE_INST_VALU"] / (SIMDS * cyc), 4)
        if wc:
            for cn, lab in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst"),
                            ("SQ_ACTIVE_INST_ANY", "active"), ("SQ_ACTIVE_INST_VALU", "active_valu")):
                if cn in m:
                    row[lab] = round(m[cn] / wc, 4)
            row["wave_cycles"] = round(4 * wc / waves)
        for cn in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                   "SQ_LDS_BANK_CONFLICT"):
            if cn in m:
                row[cn.replace("SQ_", "").lower() + "_per_wave"] = round(m[cn] / waves, 1)
        row["_total_us"] = (avg_us or 0) * launches
        rows.append(row)
    rows.sort(key=lambda r: -r["_total_us"])
    rows = rows[:a.top]
    for r in rows:
        r.pop("_total_us")
    lib = os.environ.get("PRODIFF_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                          "prodiff_amd", "libprodiff_hip.so"))
    try:
        sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16]
    except OSError:
        sha = None
    out = dict(config=a.config, lib_sha16=sha, source=a.dir, definitions=__doc__.split("\n\n")[1].strip(), kernels=rows)
    s = json.dumps(out, indent=1)
    if a.o:
        open(a.o, "w").write(s + "\n")
    for r in rows:
        print(f"{r['kernel'][:70]:70s} {r.get('avg_us_profiled')!s:>9} us  mfma {r.get('mfma_busy', 0):.3f}  "
              f"valu {r.get('valu_busy', 0):.3f}  wait {r.get('wait_any', 0):.2f}/{r.get('wait_inst', 0):.2f}  "
              f"vgpr {r['vgpr']} lds {r['lds_bytes']}")


if __name__ == "__main__":
    main()
