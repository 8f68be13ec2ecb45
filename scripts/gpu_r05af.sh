#!/bin/bash
# round 5: plan-specialised decode + verify on the work queue (tune key 28 = 1)
set -o pipefail
out=gpurun_out/r05af
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "jit_verify_shapes or encode_crc_work_queue" > $out/tests.txt 2>&1
rc=$?
tail -3 $out/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python3 -u scripts/probe_fused_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
