#!/bin/bash
# GPU box: PMC passes over the fused decode + verify kernel, ahead-of-time
# (v_perm, HEC_JIT=0) vs plan-specialised (JIT), RS(6,3) x 1024 with data
# shards {0,1,2} lost; one counter group per pass, no trace.
# Usage: pmc_verify.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_verify}
mkdir -p "$out"
export TMPDIR=/tmp
B="--crc --corrupt none --steps 3 --warmup 1 --extra-configs 0 --cpu-seconds 0 --host-path 0 --verify sample --spinup 0.1"
i=0
for v in 0 async; do
  for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
             "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
    i=$((i+1))
    HEC_JIT=$v timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "gf_fused_crc" -d "$out/p$i" -o run \
      --output-format csv -- python3 bench.py $B > "$out/p$i.log" 2>&1 || { echo "pass $i (HEC_JIT=$v: $grp) failed"; tail -5 "$out/p$i.log"; exit $i; }
    echo "pass $i HEC_JIT=$v ok"
  done
done
python3 scripts/summarize_pmc.py "$out" > "$out/summary.txt" && grep -E ", true," "$out/summary.txt" | head -80
