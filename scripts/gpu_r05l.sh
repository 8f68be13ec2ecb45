#!/bin/bash
# round 5: kernel-trace the CRC probe (product DMA kernel vs the probe's own)
set -o pipefail
out=gpurun_out/r05m
mkdir -p $out
export TMPDIR=/tmp
PROBE_SETS=2 PROBE_LAYOUT=split timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o crc -- ./scripts/probe_crc_dma > $out/probe_split.txt 2>&1 || exit 2
cat $out/probe_split.txt
find $out/prof -name "*kernel_stats.csv" -exec cat {} \;
