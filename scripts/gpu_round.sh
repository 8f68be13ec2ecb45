#!/bin/bash
# GPU box, one lease: the -m gpu suite (failures reported, not fatal), smoke,
# the default bench line, and the CRC legs' per-kernel profile.  A crash,
# abort or time limit ends the script (no GPU step after it).
# Usage: gpu_round.sh OUTDIR [profile configs...]
set -o pipefail
out=${1:-gpurun_out/round}
shift
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -v --maxfail=20 --timeout 300 --timeout-method thread \
    > "$out/gpu_tests.txt" 2>&1
rc=$?
tail -4 "$out/gpu_tests.txt"
[ $rc -le 1 ] || { echo "pytest rc=$rc: stop"; exit 1; }
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit 2
timeout -k 10 600 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 3; }
tail -c 600 "$out/bench.json"
if [ $# -gt 0 ]; then
  timeout -k 10 1500 python3 -u scripts/profile_configs.py "$out/prof" "$@" > "$out/prof.log" 2>&1 || { tail -20 "$out/prof.log"; exit 4; }
  cat "$out/prof.log"
fi
echo "gpu_round ok (pytest rc=$rc)"
