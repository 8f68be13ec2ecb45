#!/bin/bash
# Measurement (GPU box): register double-buffered kernel (tune key 5 = 3) and
# its store cache policies (key 13) against the default kernel, interleaved
# rounds via probe_rows.py.  Usage: probe_pipe.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out}
mkdir -p "$out"
P="timeout -k 10 300 python3 -u scripts/probe_rows.py"
PROBE_K=6 PROBE_S=1024 PROBE_R=3 PROBE_SHAPES="0:0:0,1:256:1:5=3,2:256:1:5=3,3:256:1:5=3,1:256:2:5=3,2:256:1:5=3:13=1,2:256:1:5=3:13=2,2:256:1:5=3:13=3,2:256:1:5=3:13=4,1:256:1:5=3:13=1" \
    $P > "$out/probe_pipe_k6.log" 2>&1 || exit 1
PROBE_K=10 PROBE_S=512 PROBE_R=4 PROBE_SHAPES="0:0:0,1:256:1:5=3,2:256:1:5=3,1:256:2:5=3,2:256:1:5=3:13=1,1:256:1:5=3:13=1,2:256:1:5=3:13=2" \
    $P > "$out/probe_pipe_k10.log" 2>&1 || exit 2
PROBE_K=6 PROBE_S=16384 PROBE_R=3 PROBE_CELL=65536 PROBE_SHAPES="0:0:0,4:256:1:5=1,1:256:1:5=3,2:256:1:5=3,3:256:1:5=3,2:256:1:5=3:13=1" \
    $P > "$out/probe_pipe_k6_64k.log" 2>&1 || exit 3
echo probe ok
