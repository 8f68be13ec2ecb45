#!/bin/bash
# round 5 final tree, as the driver runs it: the GPU suite (product library;
# the measurement build does not travel), smoke, the default bench line, and
# the rocprofv3 kernel-trace summary of that same bench command
set -o pipefail
out=gpurun_out/r05final3
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.txt 2>&1
rc=$?
tail -3 $out/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || exit 2
tail -1 $out/smoke.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o bench -- python3 bench.py > $out/bench.json 2> $out/bench.err || exit 3
tail -1 $out/bench.json | cut -c1-400
