#!/bin/bash
# round 5: the whole GPU suite + smoke on the current tree
set -o pipefail
out=gpurun_out/r05o
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.txt 2>&1
rc=$?
tail -5 $out/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || exit 2
cat $out/smoke.txt
