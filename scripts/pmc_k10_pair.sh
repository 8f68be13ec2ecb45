#!/bin/bash
# GPU box: the k = 10 / k = 6 PMC pair.  The register
# encode of RS(6,3) x 1024 and RS(10,4) x 256 (product library), same box,
# one counter group per pass plus a kernel trace (VGPRs, durations).
# Usage: pmc_k10_pair.sh OUTDIR
# PMC_GROUPS="g1;g2;..." replaces the counter groups (one pass each);
# PMC_TRACE=0 skips the kernel trace.
set -o pipefail
out=${1:-gpurun_out/pmc_k10}
mkdir -p "$out"
export TMPDIR=/tmp
B="--encode-only --steps 10 --warmup 3 --verify sample --extra-configs 0 --cpu-seconds 0 --host-path 0 --spinup 0.3"
i=0
for cfg in "--k 6 --m 3 --stripes 1024" "--k 10 --m 4 --stripes 256" "--k 10 --m 4 --stripes 1024"; do
  i=$((i+1))
  [ "${PMC_TRACE:-1}" = 0 ] || timeout -s KILL 150 rocprofv3 --kernel-trace --stats --kernel-include-regex "gf_matmul_v16" -d "$out/t$i" -o run \
    --output-format csv -- python3 bench.py $B $cfg > "$out/t$i.log" 2>&1 || { echo "trace $i failed"; tail -5 "$out/t$i.log"; exit 1; }
  groups="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE;TA_BUSY_avr TA_TA_BUSY_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_LEVEL_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM;FETCH_SIZE;WRITE_SIZE"
  IFS=';' read -ra glist <<< "${PMC_GROUPS:-$groups}"
  for grp in "${glist[@]}"; do
    p=$(echo $grp | cut -c1-24 | tr ' ' '_')
    timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "gf_matmul_v16" -d "$out/p${i}_$p" -o run \
      --output-format csv -- python3 bench.py $B $cfg > "$out/p${i}_$p.log" 2>&1 || { echo "pass $i ($grp) failed"; tail -5 "$out/p${i}_$p.log"; exit 2; }
    echo "cfg $i pass $p ok"
  done
done
