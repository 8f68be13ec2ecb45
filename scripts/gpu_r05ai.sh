#!/bin/bash
# round 5: fused encode + CRC on the queue at 4 slabs (measurement)
set -o pipefail
out=gpurun_out/r05ai
mkdir -p $out
export TMPDIR=/tmp
PROBE_ENC4=1 timeout -k 10 600 python3 -u scripts/probe_fused_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
