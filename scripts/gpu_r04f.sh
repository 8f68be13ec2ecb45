#!/bin/bash
# round-4 lease f: fused-kernel shape A/B (decode + verify: AOT / JIT at 8 and
# 4 slabs, two pairs ahead, 3 waves per SIMD, early-issued loads at 8 slabs;
# encode + CRC at the same shapes, same runs), then the tile-order skeleton sweep
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04f; mkdir -p $o
# parity of the new shapes first (a failing assertion is fine to continue past, a fault is not)
timeout -k 10 420 python3 -u -m pytest tests/test_gpu_experimental.py -m gpu -v --timeout 300 --timeout-method thread \
  -k "jit_verify_shapes or fused_variants_encode or rejects_unknown" > $o/tests_new.txt 2>&1
rc=$?; tail -3 $o/tests_new.txt; [ $rc -le 1 ] || exit 1
AB_VARIANTS="aot jit8 jit8p3 jit4 jit4p2 jit4w3" bash scripts/ab_jit.sh $o/ab > $o/ab_summary.txt 2>&1 || { tail -20 $o/ab_summary.txt; exit 1; }
grep " leg " $o/ab_summary.txt
PROBE_MODE=order timeout -k 10 240 ./scripts/probe_ratio > $o/skel_order.txt 2>&1 || { tail $o/skel_order.txt; exit 2; }
cat $o/skel_order.txt
