#!/bin/bash
# LDS / VALU PMC passes (GPU box) over the fused encode+CRC probe and the CRC
# probe, one counter group per pass, never combined with traces.
# Usage: [PMC_PROGS="scripts/probe_fused.py"] [PROBE_ENC=1,5] pmc_lds.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_lds}
mkdir -p $out
export TMPDIR=/tmp PROBE_REPS=3 PROBE_ROUNDS=1
i=0
for prog in ${PMC_PROGS:-scripts/probe_fused.py scripts/probe_crc.py}; do
  for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
             "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
    i=$((i+1))
    PROBE_ENC=${PROBE_ENC:-1} PROBE_VER=${PROBE_VER:-1} PROBE_VARIANTS="${PMC_CRC_VARIANTS:-1:2,5:2}" timeout -k 10 200 rocprofv3 --pmc $grp \
      --kernel-include-regex "gf_fused_crc|checksum_chunks512" -d $out/p$i -o run --output-format csv \
      -- python3 $prog > $out/p$i.log 2>&1 || exit $i
  done
done
python3 scripts/summarize_pmc.py $out > $out/summary.txt && cat $out/summary.txt
