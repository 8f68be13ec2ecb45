"""Summarise scripts/pmc_k10_pair.sh: per config, the median over the
gf_matmul_v16 dispatches of every counter (PMC passes) and of the kernel
duration (trace), plus derived ratios (SQ cycle counters are quad-cycles
summed over all waves; GRBM_GUI_ACTIVE summed over the 8 XCDs)."""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
CFG = {1: "RS(6,3) x 1024", 2: "RS(10,4) x 256", 3: "RS(10,4) x 1024"}
out = {}
for i, name in CFG.items():
    vals, meta = {}, {}
    for f in glob.glob(os.path.join(d, f"p{i}_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "gf_matmul_v16" not in r["Kernel_Name"]:
                continue
            vals.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            meta = {"kernel": r["Kernel_Name"], "vgpr": int(r["VGPR_Count"]), "lds": int(r["LDS_Block_Size"]),
                    "wg": int(r["Workgroup_Size"]), "grid": int(r["Grid_Size"])}
    med = {c: statistics.median(v.values()) for c, v in vals.items()}
    durs = []
    for f in glob.glob(os.path.join(d, f"t{i}", "run_kernel_trace.csv")):
        for r in csv.DictReader(open(f)):
            if "gf_matmul_v16" in r["Kernel_Name"]:
                durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    res = dict(meta)
    res["dur_ms_median"] = round(statistics.median(durs), 4) if durs else None
    res["counters"] = {k: round(v, 1) for k, v in sorted(med.items())}
    wc = med.get("SQ_WAVE_CYCLES")
    if wc:
        res["frac_of_wave_cycles"] = {k: round(med[k] / wc, 3) for k in
                                      ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU",
                                       "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_BUSY_CYCLES") if k in med}
    if "GRBM_GUI_ACTIVE" in med and res["dur_ms_median"]:
        res["clock_GHz_est"] = round(med["GRBM_GUI_ACTIVE"] / 8 / (res["dur_ms_median"] * 1e-3) / 1e9, 3)
    if "FETCH_SIZE" in med:
        res["hbm_bytes"] = round(med["FETCH_SIZE"] * 1024 * 2 + med.get("WRITE_SIZE", 0) * 1024)
    out[name] = res
print(json.dumps(out, indent=1))
