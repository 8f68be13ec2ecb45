#!/bin/bash
# GPU box, one lease: optional -m gpu test subset, then same-box A/B of bench.py
# over measurement knobs.  Each variant is NAME=TUNE ("" = product library);
# a crash or time limit ends the script.
# Usage: ab_tune.sh OUTDIR "TEST_K_EXPR|-" "BENCH ARGS" NAME=TUNE...
set -o pipefail
o=$1; tk=$2; B=$3; shift 3
mkdir -p "$o"; export TMPDIR=/tmp
if [ "$tk" != "-" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "$tk" \
      > "$o/tests.txt" 2>&1 || { tail -30 "$o/tests.txt"; exit 1; }
  tail -2 "$o/tests.txt"
fi
for nv in "$@"; do
  n=${nv%%=*}; t=${nv#*=}
  T=""; E=""
  case "$t" in @*) E="HEC_LIB_PATH=${t#@}";; ?*) T="--tune $t";; esac
  timeout -k 10 300 env $E python3 -u bench.py $B $T > "$o/$n.json" 2> "$o/$n.err" || { tail -20 "$o/$n.err"; exit 2; }
  python3 - "$o/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keep = {k: d[k] for k in ("value", "ms_per_step", "encode_GiBps", "decode_GiBps") if k in d}
c = d.get("crc32c") or {}
keep.update({k: c[k] for k in c if k.endswith("_ms") or k.endswith("frac")})
print(sys.argv[2], keep)
PY
done
