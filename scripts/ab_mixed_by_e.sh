#!/bin/bash
# Same-box A/B (GPU box): mixed-pattern decode as one launch for the batch's
# largest erasure count (default, tune key 20 = 0) vs one launch per erasure
# count over a stripe map (key 20 = 3).  Alternating runs.
set -o pipefail
out=${1:-gpurun_out/abe}
mkdir -p $out
C="--cpu-seconds 0 --host-path 0 --decode-mode mixed"
for r in 1 2 3; do
  for cfg in "--k 10 --m 4 --stripes 512" "--k 10 --m 4 --stripes 256" "" "--k 3 --m 2"; do
    for t in "" "20=3"; do
      tag=$(echo "k${cfg// /_}_t${t:-def}_r$r" | tr -d '-')
      timeout -k 10 120 python3 -u bench.py $C $cfg ${t:+--tune $t} > $out/$tag.log 2>&1 || exit 1
    done
  done
done
echo ok
