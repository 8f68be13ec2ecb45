#!/bin/bash
# round-4 lease m: per-stripe tile-column rotation in the fused kernels (key
# 25): parity, then A/B against the defaults, four alternations (the 4-slab
# specialised decode + verify is bimodal across processes: r04f, r04l)
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04m; mkdir -p $o
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "jit_verify_shapes or fused_variants_encode or slice32 or rejects_unknown" > $o/tests_new.txt 2>&1
rc=$?; tail -3 $o/tests_new.txt; [ $rc -le 1 ] || exit 1
AB_REPS=4 AB_VARIANTS="jitdef rot1 rot16 rot21" bash scripts/ab_jit.sh $o/ab > $o/ab_summary.txt 2>&1 || { tail -20 $o/ab_summary.txt; exit 1; }
grep -E "6, 3, (8|4), 12, 0, (true|false)" $o/ab_summary.txt | cut -c1-110; grep " leg " $o/ab_summary.txt | cut -c1-40
# the same kernels over five fresh buffer sets in one process (placement)
PROBE_SETS=6 timeout -k 10 300 python3 -u scripts/probe_placement.py > $o/placement.txt 2>&1 || { tail $o/placement.txt; exit 2; }
cat $o/placement.txt
