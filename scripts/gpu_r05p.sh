#!/bin/bash
# round 5: mixed-decode work queue (tune key 26) -- parity, then the
# same-process A/B against the fixed tile order
set -o pipefail
out=gpurun_out/r05s
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_experimental.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 300 --timeout-method thread -k "work_queue or mixed or decode_verify or verified" > $out/tests.txt 2>&1
rc=$?
tail -5 $out/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python3 -u scripts/probe_mixed_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
