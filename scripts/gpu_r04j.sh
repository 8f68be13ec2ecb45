#!/bin/bash
# round-4 lease j: same-box A/B of this tree's product library against the
# round-3 final build (35c31d3, lib/libhdfs_ec_amd_r03x.so via HEC_LIB_PATH):
# the mixed-pattern decode RS(10,4) x 256 and the RS(6,3) bench line, three
# alternations
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04j; mkdir -p $o
OLD=@hdfs-native_amd/lib/libhdfs_ec_amd_r03x.so
M="--k 10 --m 4 --stripes 256 --decode-mode mixed --steps 20 --warmup 5 --extra-configs 0 --cpu-seconds 0 --host-path 0 --verify sample"
H="--steps 20 --warmup 5 --extra-configs 0 --cpu-seconds 0 --host-path 0 --verify sample"
for rep in 1 2 3; do
  bash scripts/ab_tune.sh $o/mx$rep - "$M" new= r03x=$OLD > $o/mx$rep.txt 2>&1 || { tail $o/mx$rep.txt; exit 1; }
  bash scripts/ab_tune.sh $o/hl$rep - "$H" new= r03x=$OLD > $o/hl$rep.txt 2>&1 || { tail $o/hl$rep.txt; exit 1; }
done
for f in $o/mx*/*.json $o/hl*/*.json; do python3 - $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; dm = r.get("decode_mixed", {})
print("/".join(sys.argv[1].split("/")[-2:]), "value", d["value"], "line frac", r["frac"], "kernel ms", r["avg_launch_ms"],
      "| mixed ms", dm.get("avg_launch_ms"), "frac", dm.get("frac"))
PY
done
