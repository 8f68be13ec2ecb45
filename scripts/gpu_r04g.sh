#!/bin/bash
# round-4 lease g: the fused kernels of the product library after the
# addressing fix (scalar wave index, saddr loads, no spills): crc63 under the
# kernel trace, twice
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04g; mkdir -p $o
B="--crc --corrupt none --steps 10 --warmup 3 --extra-configs 0 --cpu-seconds 0 --host-path 0 --verify sample"
for rep in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/crc63.$rep -o run --output-format csv -- \
    python3 -u bench.py $B > $o/crc63.$rep.log 2>&1 || { tail -20 $o/crc63.$rep.log; exit 2; }
  python3 - $o/crc63.$rep $o/crc63.$rep.log <<'PY'
import csv, glob, json, sys
d, log = sys.argv[1:]
for p in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "gf_fused_crc" in r["Name"] or "checksum" in r["Name"]:
            print(round(float(r["AverageNs"]) / 1e6, 4), "ms x", r["Calls"], r["Name"][:110])
c = json.loads([l for l in open(log) if l.startswith("{")][-1]).get("crc32c", {})
print({k: v for k, v in c.items() if "frac" in k or k.endswith("_ms") or k == "decode_verify_kernel"})
PY
done
