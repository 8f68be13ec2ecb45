#!/bin/bash
# round-4 lease e: the GPU suite on the product library, the default bench line
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04e; mkdir -p $o
timeout -k 10 900 python3 -u -m pytest tests -m gpu --ignore=tests/test_gpu_experimental.py -v --maxfail=20 --timeout 300 --timeout-method thread > $o/gpu_tests.txt 2>&1
rc=$?; tail -3 $o/gpu_tests.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 900 python3 -u bench.py > $o/bench.json 2> $o/bench.err || { tail -20 $o/bench.err; exit 2; }
tail -c 200 $o/bench.json

