#!/bin/bash
# round-4 lease h: is the 4-slab plan-specialised decode + verify kernel
# faster when its code object comes from the disk cache than when compiled
# in-process (r04f: 1.66 vs 1.80 ms)?  jit4 (warm cache) / jit4cold (fresh
# cache) / jit8, four alternations
set -o pipefail
export TMPDIR=/tmp; o=gpurun_out/r04h; mkdir -p $o
AB_REPS=4 AB_VARIANTS="jit4 jit4cold jit8" bash scripts/ab_jit.sh $o/ab > $o/ab_summary.txt 2>&1 || { tail -20 $o/ab_summary.txt; exit 1; }
grep -E "leg|true, 2, true, hec::jit_plan::Net, 1>|true, 2, false, hec::jit_plan::Net, 1>" $o/ab_summary.txt | grep -v "6, 1," | cut -c1-140
