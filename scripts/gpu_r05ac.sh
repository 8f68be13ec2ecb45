#!/bin/bash
# round 5: 64 KiB cells -- LDS-DMA kernel vs the register kernel on the queue
set -o pipefail
out=gpurun_out/r05ad
mkdir -p $out
export TMPDIR=/tmp
PROBE_C64K=1 PROBE_CELLS=4096:262144,8192:131072,16384:65536,131072:8192,262144:4096 timeout -k 10 600 python3 -u scripts/probe_matmul_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
