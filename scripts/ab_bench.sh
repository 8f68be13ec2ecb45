#!/bin/bash
# Same-box A/B of the full bench line (GPU box): in-tree engine (new) vs
# another build (base, HEC_LIB_PATH), alternating ROUNDS times, same args.
# Usage: ab_bench.sh BASE_SO OUTFILE ROUNDS [bench args...]
set -o pipefail
base=$1; out=$2; rounds=$3; shift 3
: > "$out"
for r in $(seq "$rounds"); do
  for lib in new base; do
    L=""; [ $lib = base ] && L="HEC_LIB_PATH=$base"
    timeout -k 10 300 env $L python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --host-path 0 "$@" > gpurun_out/_ab.log 2>&1 \
      || { echo "FAILED $lib"; tail -20 gpurun_out/_ab.log; exit 1; }
    tail -1 gpurun_out/_ab.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(sys.argv[1], d["value"], d["roofline"]["frac"], d["encode_GiBps"], d["decode_GiBps"])' $lib | tee -a "$out"
  done
done
