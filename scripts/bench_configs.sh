#!/bin/bash
# Every BASELINE.json config at its exact size on one MI355X (GPU box).
set -o pipefail
out=${1:-gpurun_out/configs.jsonl}
: > "$out"
run() {
    local name="$1"; shift
    timeout -k 10 300 python3 bench.py "$@" > gpurun_out/_cfg.log 2>&1 || { echo "FAILED $name"; tail -20 gpurun_out/_cfg.log; exit 1; }
    echo "{\"config\": \"$name\", \"args\": \"$*\", \"result\": $(tail -1 gpurun_out/_cfg.log)}" >> "$out"
    tail -1 gpurun_out/_cfg.log | python3 -c 'import json,sys; d=json.load(sys.stdin); print("'"$name"'", d["value"], d["unit"], d["roofline"]["achieved"], d["roofline"]["frac"], (d.get("cpu_baseline") or {}).get("value"))'
}
run "RS(3,2) 1MiB x1024 enc+dec" --k 3 --m 2 --stripes 1024 --cpu-seconds 10 --host-path 0
run "RS(6,3) 1MiB x1024 encode" --encode-only --cpu-seconds 0 --host-path 0
run "RS(6,3) 1MiB x1024 enc+dec(0,1,2 missing)" --cpu-seconds 10
run "RS(10,4) 1MiB x2048 enc+dec(0..3 missing)" --k 10 --m 4 --global-stripes 2048 --cpu-seconds 10 --host-path 0
run "RS(6,3) 64KiB x65536 enc+dec" --cell 65536 --stripes 65536 --cpu-seconds 10 --host-path 0
run "RS(6,3) 1MiB x1024 mixed decode (1..3 data lost per stripe)" --decode-mode mixed --cpu-seconds 0 --host-path 0
run "RS(10,4) 1MiB x512 mixed decode (1..4 data lost per stripe)" --k 10 --m 4 --stripes 512 --decode-mode mixed --cpu-seconds 0 --host-path 0
