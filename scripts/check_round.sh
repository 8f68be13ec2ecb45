#!/bin/bash
# GPU box: the whole -m gpu suite, then bench lines for the host-side
# changes (mixed decode, per-call drop-in).  First failure ends the script.
# Usage: check_round.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/check}
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $out/tests.log 2>&1 || exit 1
C="--cpu-seconds 0 --host-path 0"
for r in 1 2; do
  timeout -k 10 200 python3 -u bench.py --k 10 --m 4 --stripes 512 --decode-mode mixed $C > $out/mixed104_r$r.log 2>&1 || exit 2
  timeout -k 10 200 python3 -u bench.py --k 10 --m 4 --stripes 256 --decode-mode mixed $C > $out/mixed104x256_r$r.log 2>&1 || exit 3
done
timeout -k 10 200 python3 -u bench.py --decode-mode mixed $C > $out/mixed63.log 2>&1 || exit 4
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > $out/default.log 2>&1 || exit 5
echo "check_round ok"
