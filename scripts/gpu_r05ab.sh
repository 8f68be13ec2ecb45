#!/bin/bash
# round 5: RS(10,4) register kernel shapes on the work queue
set -o pipefail
out=gpurun_out/r05ah
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "matmul_work_queue" > $out/tests.txt 2>&1
rc=$?
tail -3 $out/tests.txt
[ $rc -eq 0 ] || exit 1
PROBE_K10=1 timeout -k 10 600 python3 -u scripts/probe_matmul_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
