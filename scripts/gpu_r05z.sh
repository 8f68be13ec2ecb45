#!/bin/bash
# round 5: fused encode + CRC with the work queue (tune key 28) A/B, then
# the profile part B of the final tree
set -o pipefail
out=gpurun_out/r05z
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u scripts/probe_fused_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
