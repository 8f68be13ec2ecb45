#!/bin/bash
# Same-box A/B (GPU box): the in-tree engine (new) against another build
# (base, HEC_LIB_PATH) on probe_rows.py cases, alternating ROUNDS times.
# Usage: ab_quick.sh BASE_SO OUTDIR ROUNDS "K:S:R[:CELL]" ...
set -o pipefail
base=$1; out=$2; rounds=$3; shift 3
mkdir -p "$out"
for r in $(seq "$rounds"); do
  for c in "$@"; do
    IFS=: read -r K S R CELL <<< "$c"
    CELL=${CELL:-1048576}
    for lib in new base; do
      L=""; [ $lib = base ] && L="HEC_LIB_PATH=$base"
      timeout -k 10 200 env $L PROBE_K=$K PROBE_S=$S PROBE_R=$R PROBE_CELL=$CELL PROBE_ROUNDS=2 PROBE_REPS=8 \
          PROBE_SHAPES=0:0:0 python3 -u scripts/probe_rows.py >> "$out/k${K}_s${S}_r${R}_c${CELL}_$lib.log" 2>&1 \
          || { echo "FAILED $c $lib"; tail -20 "$out/k${K}_s${S}_r${R}_c${CELL}_$lib.log"; exit 1; }
    done
  done
done
for f in "$out"/*.log; do echo "== $(basename "$f")"; grep -h "shape" "$f"; done
