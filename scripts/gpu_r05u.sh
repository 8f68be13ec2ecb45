#!/bin/bash
# round 5: work-queue register kernel as the default -- whole GPU suite,
# smoke, the default bench line, the A/B probe
set -o pipefail
out=gpurun_out/r05ag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.txt 2>&1
rc=$?
tail -5 $out/tests.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.txt 2>&1 || exit 2
tail -2 $out/smoke.txt
timeout -k 10 400 python3 -u bench.py > $out/bench.json 2> $out/bench.err || exit 3
cat $out/bench.json | cut -c1-600
timeout -k 10 700 python3 -u scripts/profile_configs.py $out/prof crc63 > $out/probe.txt 2>&1 || exit 4
cat $out/probe.txt
