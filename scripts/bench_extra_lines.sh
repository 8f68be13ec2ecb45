#!/bin/bash
# Extra bench lines on the final tree (GPU box): mixed-pattern decode,
# the fused CRC legs, and the rust/benches/ec.rs cases.  Each step under its
# own time limit; the first failure ends the script.
# Usage: bench_extra_lines.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/extra}
mkdir -p $out
C="--cpu-seconds 0 --host-path 0"
timeout -k 10 200 python3 -u bench.py --decode-mode mixed $C > $out/mixed63.log 2>&1 || exit 1
timeout -k 10 200 python3 -u bench.py --k 10 --m 4 --stripes 512 --decode-mode mixed $C > $out/mixed104.log 2>&1 || exit 2
timeout -k 10 200 python3 -u bench.py --k 10 --m 4 --stripes 256 --decode-mode mixed $C > $out/mixed104x256.log 2>&1 || exit 3
timeout -k 10 300 python3 -u bench.py --crc $C > $out/crc63.log 2>&1 || exit 4
timeout -k 10 300 python3 -u bench.py --crc --k 10 --m 4 --stripes 512 $C > $out/crc104.log 2>&1 || exit 5
timeout -k 10 300 python3 -u bench.py --ref-cases > $out/ref.log 2>&1 || exit 6
echo "bench_extra_lines ok"
