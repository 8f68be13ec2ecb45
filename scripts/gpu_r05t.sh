#!/bin/bash
# round 5: register kernel work queue (tune key 27) A/B on the bench step
set -o pipefail
out=gpurun_out/r05t
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u scripts/probe_matmul_wq.py > $out/probe.txt 2>&1 || exit 2
cat $out/probe.txt
