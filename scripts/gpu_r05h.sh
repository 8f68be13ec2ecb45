#!/bin/bash
# round 5: the LDS-DMA CRC32C kernel -- CRC / checksum / verify parity (product
# and measurement builds), then the CRC probe on the bench layout
set -o pipefail
out=gpurun_out/r05k
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_experimental.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "crc32c or checksum_verify or decode_verify_vs or crc_schemes" > $out/tests.txt 2>&1
rc=$?
tail -5 $out/tests.txt
[ $rc -eq 0 ] || exit 1
PROBE_SETS=2 PROBE_LAYOUT=split timeout -k 10 300 ./scripts/probe_crc_dma > $out/probe_split.txt 2>&1 || exit 2
cat $out/probe_split.txt
