"""Turns rocprofv3 --pmc CSVs (FETCH_SIZE pass + WRITE_SIZE pass) into
profiles/pmc_traffic.json: HBM bytes per launch of the engine kernel.

Corrections per /opt/skills/guides/MI355X_MICROARCH.md §HBM:
  * FETCH_SIZE / WRITE_SIZE are in KiB (x1024);
  * on gfx950 FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane)
    coalesced streaming read -> x2 (our loads are global_load_dwordx4);
  * WRITE_SIZE reads exactly for 16-B-per-lane streaming stores.
usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR K M CELL STRIPES OUT.json
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, name_re="gf_matmul_v16"):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if name_re in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                    rows.append(float(r["Counter_Value"]))
    return rows


def main():
    fdir, wdir, k, m, cell, stripes, out = sys.argv[1:8]
    k, m, cell, stripes = int(k), int(m), int(cell), int(stripes)
    f = per_dispatch(fdir, "FETCH_SIZE")
    w = per_dispatch(wdir, "WRITE_SIZE")
    if not f or not w:
        raise SystemExit(f"no counter rows (fetch {len(f)}, write {len(w)})")
    fetch = 2.0 * 1024 * sum(f) / len(f)
    write = 1024.0 * sum(w) / len(w)
    algo_read, algo_write = k * cell * stripes, m * cell * stripes
    res = {
        "config": {"k": k, "m": m, "cell": cell, "stripes": stripes},
        "kernel": "gf_matmul_v16",
        "dispatches": {"fetch": len(f), "write": len(w)},
        "fetch_bytes_per_launch": fetch,
        "write_bytes_per_launch": write,
        "hbm_bytes_per_launch": fetch + write,
        "algorithmic_bytes_per_launch": algo_read + algo_write,
        "traffic_over_algorithmic": (fetch + write) / (algo_read + algo_write),
        "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on 16B/lane streaming reads); WRITE_SIZE KiB x1024",
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
