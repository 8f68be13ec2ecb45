"""Average every PMC counter per kernel name over the counter_collection CSVs
under a directory (rocprofv3 --pmc output).  usage: summarize_pmc.py DIR"""
import collections
import csv
import glob
import os
import sys

acc = collections.defaultdict(list)
for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            short = name[:name.rfind("(")] if name.endswith(")") else name  # drop the argument list
            i = min([short.find(t) for t in ("gf_", "checksum") if t in short] or [0])
            short = short[i:][:100]  # kernel template name, namespaces of its arguments kept
            acc[(short, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:100s} {c:24s} n={len(v):3d} mean={sum(v) / len(v):.4g}")
