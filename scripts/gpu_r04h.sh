#!/bin/bash
# round-4 lease h: is the 4-slab plan-specialised decode + verify kernel
# faster when its code object comes from the disk cache than when compiled
# in-process (r04f: 1.66 vs 1.80 ms)?  jit4 (warm cache) / jit4cold (fresh
# cache) / jit8, and the expected sums loaded once per tile (jit8p4, jit4p4),
# three alternations
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04h; mkdir -p $o
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "jit_verify_shapes or rejects_unknown" > $o/tests_new.txt 2>&1
rc=$?; tail -3 $o/tests_new.txt; [ $rc -le 1 ] || exit 1
AB_REPS=3 AB_VARIANTS="jit4 jit4cold jit8 jit8p4 jit4p4" bash scripts/ab_jit.sh $o/ab > $o/ab_summary.txt 2>&1 || { tail -20 $o/ab_summary.txt; exit 1; }
grep -E "6, 3, (8|4), 12, 0, true" $o/ab_summary.txt | cut -c1-120; grep " leg " $o/ab_summary.txt | cut -c1-60
