#!/bin/bash
# Same-box sweep (GPU box): RS(10,4), the BASELINE's 2048 stripes on ONE GPU
# (--global-stripes 2048 at N = 1), across the tile-order group (key 8),
# blocks per CU (key 3) and chunks per lane (key 1), alternating rounds.
# Writes one bench line per run; first failure ends the script.
set -o pipefail
out=${1:-gpurun_out/k10s}
mkdir -p $out
C="--cpu-seconds 0 --host-path 0 --k 10 --m 4 --global-stripes 2048 --steps 10 --warmup 3"
for r in 1 2; do
  for t in "" "8=1" "8=2" "8=8" "8=16" "3=4" "3=16" "1=1" "1=4"; do
    tag="t${t:-def}_r$r"
    timeout -k 10 200 python3 -u bench.py $C ${t:+--tune $t} > $out/$tag.log 2>&1 || exit 1
    echo "$tag $(grep '^{' $out/$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["frac"])')"
  done
done
echo ok
