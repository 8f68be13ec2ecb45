#!/bin/bash
# round 5: register kernel on the queue at 1 vs 2 blocks per CU
set -o pipefail
out=gpurun_out/r05ak
mkdir -p $out
export TMPDIR=/tmp
PROBE_GROUP=1 timeout -k 10 600 python3 -u scripts/probe_matmul_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
