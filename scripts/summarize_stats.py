"""Shortens rocprofv3 kernel_stats.csv names for committing under profiles/."""
import csv
import re
import sys


def short(name: str) -> str:
    if "gf_matmul" in name:
        return re.sub(r"\(hec::MatmulArgs\)", "", name)
    if name.startswith("void at::native") or name.startswith("at::"):
        m = re.match(r"void (at::native::[\w:]*?(\w+_kernel\w*))", name)
        return ("torch:" + m.group(2)) if m else "torch:" + name[:60]
    return name[:80]


src, dst = sys.argv[1], sys.argv[2]
with open(src) as f, open(dst, "w", newline="") as g:
    r = csv.DictReader(f)
    w = csv.DictWriter(g, fieldnames=r.fieldnames)
    w.writeheader()
    for row in r:
        row["Name"] = short(row["Name"])
        w.writerow(row)
