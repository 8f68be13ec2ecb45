"""Summarise scripts/pmc_layout.sh: per (config, layout), the median over the
gf_matmul_v16 dispatches of every counter and of the kernel duration, and the
stall counters as fractions of the per-instance cycles (TCP: 256 instances,
TCC: 16 per XCD x 8; GRBM_GUI_ACTIVE summed over the 8 XCDs)."""
import csv
import glob
import json
import os
import re
import statistics
import sys

d = sys.argv[1]
out = {}
tags = sorted({re.sub(r"^(t|p)_", "", re.sub(r"_\d+$", "", os.path.basename(x)))
               for x in glob.glob(os.path.join(d, "[tp]_*")) if os.path.isdir(x)})
for tag in tags:
    vals = {}
    for f in glob.glob(os.path.join(d, f"p_{tag}_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "gf_matmul_v16" in r["Kernel_Name"]:
                vals.setdefault(r["Counter_Name"], {}).setdefault(r["Dispatch_Id"], 0.0)
                vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    med = {c: statistics.median(v.values()) for c, v in vals.items()}
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
            for f in glob.glob(os.path.join(d, f"t_{tag}", "run_kernel_trace.csv"))
            for r in csv.DictReader(open(f)) if "gf_matmul_v16" in r["Kernel_Name"]]
    res = {"dur_ms_median": round(statistics.median(durs), 4) if durs else None,
           "counters": {k: round(v, 1) for k, v in sorted(med.items())}}
    cyc = med.get("GRBM_GUI_ACTIVE", 0) / 8
    if cyc:
        res["per_instance_cycle"] = {k: round(v / (256 if k.startswith("TCP") else 128) / cyc, 4)
                                     for k, v in sorted(med.items()) if k.startswith(("TCP", "TCC"))}
    out[tag] = res
print(json.dumps(out, indent=1))
