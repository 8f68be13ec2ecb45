#!/bin/bash
# PMC passes over scripts/probe_crc.py (GPU box), one counter group per pass,
# never combined with traces.  Usage: pmc_crc.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_crc}
mkdir -p $out
export TMPDIR=/tmp PROBE_REPS=3
timeout -k 10 200 python3 scripts/probe_crc.py > $out/probe.log 2>&1 || exit 1
i=0
for grp in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex crc32c -d $out/p$i -o run --output-format csv \
    -- python3 scripts/probe_crc.py > $out/p$i.log 2>&1 || exit $((i+1))
done
python3 scripts/summarize_pmc.py $out > $out/summary.txt && cat $out/summary.txt
