#!/bin/bash
# GPU box: PMC passes over the RS(6,3) register encode at one vs two blocks per
# CU (measurement build, tune key 3), one counter group per pass, kernel trace
# off.  Usage: pmc_waves.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_waves}
mkdir -p "$out"
export TMPDIR=/tmp
B="--encode-only --steps 5 --warmup 2 --verify sample --extra-configs 0 --cpu-seconds 0 --host-path 0 --spinup 0.2"
i=0
for tune in 3=1 3=2; do
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "gf_matmul_v16" -d "$out/p$i" -o run \
      --output-format csv -- python3 bench.py $B --tune $tune > "$out/p$i.log" 2>&1 || { echo "pass $i ($tune: $grp) failed"; tail -5 "$out/p$i.log"; exit $i; }
    echo "pass $i $tune: $grp ok"
  done
done
