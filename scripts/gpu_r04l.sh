#!/bin/bash
# round-4 lease l: the slicing-by-32 CRC tail (scheme 15, key 11 = 12): parity,
# then same-box A/B against the defaults (encode + CRC at 8 slabs, the
# specialised decode + verify at 4), three alternations
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04l; mkdir -p $o
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "jit_verify_shapes or slice32 or rejects_unknown" > $o/tests_new.txt 2>&1
rc=$?; tail -3 $o/tests_new.txt; [ $rc -le 1 ] || exit 1
AB_REPS=3 AB_VARIANTS="jitdef s15" bash scripts/ab_jit.sh $o/ab > $o/ab_summary.txt 2>&1 || { tail -20 $o/ab_summary.txt; exit 1; }
grep -E "6, 3, (8|4), 1[25], 0, (true|false)" $o/ab_summary.txt | cut -c1-120; grep " leg " $o/ab_summary.txt | cut -c1-200
