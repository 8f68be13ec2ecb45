#!/bin/bash
# Measurement (GPU box): output-burst kernel (tune key 5 = 4, key 15 = tiles
# per burst) against the default kernel, interleaved via probe_rows.py.
set -o pipefail
out=${1:-gpurun_out}
mkdir -p "$out"
PROBE_K=6 PROBE_S=1024 PROBE_R=3 PROBE_ROUNDS=6 PROBE_SHAPES="0:0:0,4:256:1:5=4:15=2,4:256:1:5=4:15=3,0:0:0" \
    timeout -k 10 300 python3 -u scripts/probe_rows.py > "$out/probe_burst_k6.log" 2>&1 || exit 1
PROBE_K=6 PROBE_S=16384 PROBE_R=3 PROBE_CELL=65536 PROBE_SHAPES="0:0:0,4:256:1:5=4:15=2,4:256:1:5=4:15=3" \
    timeout -k 10 300 python3 -u scripts/probe_rows.py > "$out/probe_burst_k6_64k.log" 2>&1 || exit 2
echo probe ok
