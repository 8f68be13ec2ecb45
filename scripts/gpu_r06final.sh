#!/bin/bash
# Round-6 final-tree validation (GPU box), the driver's shape: the -m gpu
# suite (product library), smoke, the default bench line, the same bench
# command under rocprofv3 --kernel-trace --stats, and the Rust shim's C
# replay (its bench_mi355x leg prints the device group's rates).  Each GPU
# step under its own time limit; the first failure ends the script.
set -o pipefail
out=${1:-gpurun_out/r06final/v}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$out/tests.txt" 2>&1 \
  || { tail -30 "$out/tests.txt"; exit 1; }
tail -2 "$out/tests.txt"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit 2
tail -1 "$out/smoke.txt"
timeout -k 10 400 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 3; }
cut -c1-300 "$out/bench.json"
timeout -k 10 120 hdfs-native_amd/build/shim_replay > "$out/shim_replay.txt" 2>&1 || { tail -20 "$out/shim_replay.txt"; exit 4; }
grep "bench ec.rs\|shim replay" "$out/shim_replay.txt"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$out/bench_prof" -o run --output-format csv -- python3 bench.py \
  > "$out/bench_prof.json" 2> "$out/bench_prof.err" || { tail -20 "$out/bench_prof.err"; exit 5; }
echo "gpu_r06final ok"
