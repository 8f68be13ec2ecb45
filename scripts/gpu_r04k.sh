#!/bin/bash
# round-4 lease k: parity of the early-output schedule (key 24 = 5), its A/B
# against the default specialised shape (3 alternations), then lease j (this
# tree vs the round-3 build, mixed decode and the bench line)
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04k; mkdir -p $o
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "jit_verify_shapes or rejects_unknown" > $o/tests_new.txt 2>&1
rc=$?; tail -3 $o/tests_new.txt; [ $rc -le 1 ] || exit 1
AB_REPS=3 AB_VARIANTS="jit4 jit4p5 jit8p5" bash scripts/ab_jit.sh $o/ab > $o/ab_summary.txt 2>&1 || { tail -20 $o/ab_summary.txt; exit 1; }
grep -E "6, 3, (8|4), 12, 0, true" $o/ab_summary.txt | cut -c1-120; grep " leg " $o/ab_summary.txt | cut -c1-60
bash scripts/gpu_r04j.sh
