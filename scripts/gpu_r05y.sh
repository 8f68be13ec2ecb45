#!/bin/bash
# round 5 final tree: per-config roofline evidence (scripts/profile_configs.py)
# usage: bash scripts/gpu_r05y.sh OUTDIR config...
set -o pipefail
export TMPDIR=/tmp
out=$1
shift
mkdir -p $out
timeout -k 10 1100 python3 -u scripts/profile_configs.py $out "$@" > $out/profile.log 2>&1
rc=$?
tail -12 $out/profile.log
exit $rc
