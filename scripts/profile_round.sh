#!/bin/bash
# Round profile (GPU box): kernel trace + stats of the default bench, then
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes (never combined with
# sys/runtime traces), then the traffic summary.  Usage: profile_round.sh TAG
set -o pipefail
tag=${1:-r01}
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 3 --cpu-seconds 0 --spinup 0.3 --host-path 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $B > $out/bench_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gf_matmul -d $out/fetch -o run --output-format csv -- $B > $out/bench_fetch.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex gf_matmul -d $out/write -o run --output-format csv -- $B > $out/bench_write.log 2>&1 || exit 3
python3 scripts/pmc_traffic.py $out/fetch $out/write 6 3 1048576 1024 $out/pmc_traffic.json || exit 4
echo profile ok
