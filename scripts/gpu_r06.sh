#!/bin/bash
# round 6 GPU lease: OUT=dir; optional probes, the -m gpu suite, smoke, the
# default bench line.  Every GPU step has its own time limit; a crash,
# abort or time limit ends the script (no GPU step after it).
set -o pipefail
out=${1:-gpurun_out/r06}
mkdir -p "$out"
export TMPDIR=/tmp
if [ "${PROBE_STREAM:-0}" = 1 ]; then
  timeout -k 10 120 python3 -u scripts/probe_stream_id.py rocm > "$out/stream_id_rocm.json" 2>&1 || exit 10
  timeout -k 10 120 python3 -u scripts/probe_stream_id.py torch > "$out/stream_id_torch.json" 2>&1 || exit 11
  cat "$out"/stream_id_*.json
fi
if [ -n "${FIRST_K:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$FIRST_K" \
      > "$out/first.txt" 2>&1 || { tail -40 "$out/first.txt"; exit 12; }
  tail -3 "$out/first.txt"
fi
timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/tests.txt" 2>&1 || { tail -40 "$out/tests.txt"; exit 1; }
tail -3 "$out/tests.txt"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || exit 2
tail -1 "$out/smoke.txt"
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 400 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -20 "$out/bench.err"; exit 3; }
  cut -c1-500 "$out/bench.json"
fi
echo "gpu_r06 ok"
