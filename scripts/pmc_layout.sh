#!/bin/bash
# GPU box: PMC passes over the plain encode (gf_matmul_v16) of RS(10,4) x 256
# and RS(6,3) x 1024 in bench.py's split layout and the shard layout
# (scripts/probe_k10_layout.py, one (config, layout) per process, one counter
# group per pass).  Usage: pmc_layout.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_layout}
mkdir -p "$out"
export TMPDIR=/tmp PROBE_ROUNDS=1 PROBE_REPS=6 PROBE_PADS=0
groups="TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_LFIFO_FULL_sum GRBM_GUI_ACTIVE;TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_TAG_STALL_sum TCC_BUSY_sum;TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_STALL_sum;TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_IB_STALL_sum"
IFS=';' read -ra glist <<< "${PMC_GROUPS:-$groups}"
for k in 10 6; do
  for lay in "pad 0" "shard"; do
    tag="k${k}_${lay// /}"
    export PROBE_CFG=$k "PROBE_ONLY=$lay"
    timeout -s KILL 150 rocprofv3 --kernel-trace --stats --kernel-include-regex "gf_matmul_v16" -d "$out/t_$tag" -o run \
      --output-format csv -- python3 scripts/probe_k10_layout.py > "$out/t_$tag.log" 2>&1 \
      || { echo "trace $tag failed"; tail -5 "$out/t_$tag.log"; exit 1; }
    j=0
    for grp in "${glist[@]}"; do
      j=$((j+1))
      timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "gf_matmul_v16" -d "$out/p_${tag}_$j" -o run \
        --output-format csv -- python3 scripts/probe_k10_layout.py > "$out/p_${tag}_$j.log" 2>&1 \
        || { echo "pass $tag $j failed"; tail -5 "$out/p_${tag}_$j.log"; exit 2; }
      echo "$tag pass $j ok"
    done
  done
done
