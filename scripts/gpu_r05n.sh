#!/bin/bash
# round 5: same-process A/B of the CRC32C kernels (LDS-DMA default vs the
# register-staged one, measurement build), bench layout + stripe layout
set -o pipefail
out=gpurun_out/r05n
mkdir -p $out
export TMPDIR=/tmp
PROBE_CRC_AB=1 PROBE_LAYOUTS=split,stripe,shard PROBE_SETS=2 PROBE_ROUNDS=5 timeout -k 10 400 python3 -u scripts/probe_layout.py > $out/crc_ab.txt 2>&1 || exit 2
cat $out/crc_ab.txt
