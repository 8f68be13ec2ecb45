#!/bin/bash
# Same-box A/B of two in-tree engine builds (GPU box): runs each probe with
# the candidate (default lib/) and the baseline (HEC_LIB_PATH=$BASE)
# alternately, ROUNDS times (AB_FUSED=1 adds the fused encode+CRC probe).
# Usage: ab_libs.sh BASE_SO OUTDIR [ROUNDS]
set -o pipefail
base=$1; out=${2:-gpurun_out/ab}; rounds=${3:-3}
mkdir -p "$out"
run() {  # tag, env..., command
    local tag=$1; shift
    timeout -k 10 200 env "$@" >> "$out/$tag.log" 2>&1 || { echo "FAILED $tag"; exit 1; }
}
for r in $(seq "$rounds"); do
  for lib in new base; do
    L=""; [ $lib = base ] && L="HEC_LIB_PATH=$base"
    run k6_$lib $L PROBE_K=6 PROBE_S=1024 PROBE_R=3 PROBE_ROUNDS=3 PROBE_SHAPES=0:0:0 python3 -u scripts/probe_rows.py
    run k10_$lib $L PROBE_K=10 PROBE_S=512 PROBE_R=4 PROBE_ROUNDS=3 PROBE_SHAPES=0:0:0 python3 -u scripts/probe_rows.py
    run k6s_$lib $L PROBE_K=6 PROBE_S=16384 PROBE_CELL=65536 PROBE_R=3 PROBE_ROUNDS=3 PROBE_SHAPES=0:0:0 \
        python3 -u scripts/probe_rows.py
    [ -n "$AB_FUSED" ] && run fused63_$lib $L PROBE_ENC=1 PROBE_VER=1 PROBE_ROUNDS=3 python3 -u scripts/probe_fused.py
  done
done
for f in "$out"/*.log; do echo "== $(basename $f)"; grep -h "shape\|scheme" "$f"; done
