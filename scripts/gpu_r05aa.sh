#!/bin/bash
# round 5: CRC32C checksum kernel on the work queue (tune key 29) -- parity
# of the variants, then the same-buffer A/B on the bench layouts
set -o pipefail
out=gpurun_out/r05ao
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "crc_runs" > $out/tests.txt 2>&1
rc=$?
tail -3 $out/tests.txt
[ $rc -eq 0 ] || exit 1
PROBE_CRC_AB=1 PROBE_LAYOUTS=split,stripe PROBE_SETS=2 PROBE_ROUNDS=5 timeout -k 10 500 python3 -u scripts/probe_layout.py > $out/crc_ab.txt 2>&1 || exit 2
cat $out/crc_ab.txt
