#!/bin/bash
# Measurement sweep (GPU box): bench.py across tuning knobs and configs.
# Each run is bounded by its own timeout; stops at the first failure.
set -o pipefail
out=${1:-gpurun_out/sweep.jsonl}
mkdir -p "$(dirname "$out")"
: > "$out"
run() {
    timeout -k 10 240 python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 "$@" > gpurun_out/_one.log 2>&1 || { echo "FAILED: $*"; cat gpurun_out/_one.log; exit 1; }
    echo "{\"args\": \"$*\", \"result\": $(tail -1 gpurun_out/_one.log)}" >> "$out"
    echo "$* -> $(tail -1 gpurun_out/_one.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["roofline"]["achieved"], d["roofline"]["frac"])')"
}
for t in "2=0,3=0" "2=1,3=0" "2=1,3=2" "2=1,3=3" "2=1,3=4" "1=2,2=1,3=0" "1=2,2=1,3=2" "2=0,3=2"; do
    run --tune "$t"
done
for t in "2=1,3=2" "2=1,3=0" "1=2,2=1,3=2"; do
    run --tune "$t" --k 10 --m 4 --stripes 512
    run --tune "$t" --cell 65536 --stripes 16384
done
