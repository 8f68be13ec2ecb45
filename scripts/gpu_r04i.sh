#!/bin/bash
# round-4 lease i: mixed-pattern decode RS(10,4) x 256, blocks per CU (tune
# key 3; default 8 with one resident: each block restages the resident plans)
# and the tile-order group (key 8), two alternations, live decode roofline
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04i; mkdir -p $o
B="--k 10 --m 4 --stripes 256 --decode-mode mixed --steps 20 --warmup 5 --extra-configs 0 --cpu-seconds 0 --host-path 0 --verify sample"
for rep in 1 2; do
  bash scripts/ab_tune.sh $o/r$rep - "$B" prod= bpc8=3=8 bpc1=3=1 bpc2=3=2 bpc4=3=4 grp2=8=2 grp16=8=16 > $o/r$rep.txt 2>&1 || { tail $o/r$rep.txt; exit 1; }
  for f in $o/r$rep/*.json; do python3 - $f <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
dm = d["roofline"].get("decode_mixed", {})
print(sys.argv[1].split("/")[-1], "value", d["value"], "decode", d.get("decode_GiBps"), "mixed kernel ms", dm.get("avg_launch_ms"), "frac", dm.get("frac"))
PY
  done
done
