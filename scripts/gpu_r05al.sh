#!/bin/bash
# round 5: non-temporal sum stores (tune key 30) for the CRC-only and the
# fused encode + CRC kernels
set -o pipefail
out=gpurun_out/r05al
mkdir -p $out
export TMPDIR=/tmp
PROBE_CRC_AB=1 PROBE_LAYOUTS=split,stripe PROBE_SETS=2 PROBE_ROUNDS=5 timeout -k 10 400 python3 -u scripts/probe_layout.py > $out/crc_ab.txt 2>&1 || exit 2
cat $out/crc_ab.txt
PROBE_NT=1 timeout -k 10 400 python3 -u scripts/probe_fused_wq.py > $out/fused_nt.txt 2>&1 || exit 3
cat $out/fused_nt.txt
