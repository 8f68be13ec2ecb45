#!/bin/bash
# Measurement (GPU box): XCD-contiguous block -> tile mapping (tune key 16)
# vs round-robin, interleaved via probe_rows.py.  Usage: probe_xcd.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out}
mkdir -p "$out"
P="timeout -k 10 300 python3 -u scripts/probe_rows.py"
PROBE_K=6 PROBE_S=1024 PROBE_R=3 PROBE_ROUNDS=6 PROBE_SHAPES="0:0:0,0:0:0:16=1,0:0:0:16=1:8=8,0:0:0:8=8" \
    $P > "$out/probe_xcd_k6.log" 2>&1 || exit 1
PROBE_K=10 PROBE_S=512 PROBE_R=4 PROBE_SHAPES="0:0:0,0:0:0:16=1" $P > "$out/probe_xcd_k10.log" 2>&1 || exit 2
PROBE_K=6 PROBE_S=16384 PROBE_R=3 PROBE_CELL=65536 PROBE_SHAPES="0:0:0,0:0:0:16=1,4:256:1:5=1,4:256:1:5=1:16=1" \
    $P > "$out/probe_xcd_k6_64k.log" 2>&1 || exit 3
echo probe ok
