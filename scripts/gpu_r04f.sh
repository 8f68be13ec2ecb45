#!/bin/bash
# round-4 lease f: fused-kernel shape A/B (decode + verify: AOT / JIT at 8 and
# 4 slabs, two pairs ahead, 3 waves per SIMD; encode + CRC at 8 vs 4 slabs and
# two pairs ahead, same runs), then the tile-order skeleton sweep
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04f; mkdir -p $o
AB_VARIANTS="aot jit8 jit4 jit4p2 jit4w3" bash scripts/ab_jit.sh $o/ab > $o/ab_summary.txt 2>&1 || { tail -20 $o/ab_summary.txt; exit 1; }
grep " leg " $o/ab_summary.txt
PROBE_MODE=order timeout -k 10 240 ./scripts/probe_ratio > $o/skel_order.txt 2>&1 || { tail $o/skel_order.txt; exit 2; }
cat $o/skel_order.txt
