#!/bin/bash
# GPU box, one lease: same-box A/B of the fused decode + verify kernel --
# ahead-of-time v_perm kernel (HEC_JIT=0) vs the plan-specialised (JIT)
# kernel at 8 and 4 slabs (measurement build, tune key 10; AB_VARIANTS adds
# jit4p2 = two input pairs loaded ahead, jit4w3 = 3 waves per SIMD, jit8p3 = loads
# issued before the parity math, jit4cold = jit4 compiled in-process from an
# empty code-object cache, jit8p4 / jit4p4 = expected sums loaded per tile,
# jit4p5 / jit8p5 = rebuilt rows stored and the next tile's first inputs loaded
# before the last CRC round, jitdef = the measurement build at its defaults,
# s15 = the CRC tail through slicing-by-32 tables (key 11 = 12), rotN = the
# per-stripe column rotation key 25 = N; the
# encode + CRC leg follows keys 10 / 24 too) -- each variant
# under rocprofv3 --kernel-trace --stats (no counters), alternated twice.
# Usage: ab_jit.sh OUTDIR [extra bench args]
set -o pipefail
o=${1:-gpurun_out/ab_jit}; shift
mkdir -p "$o"; export TMPDIR=/tmp
B="--crc --corrupt none --steps 10 --warmup 3 --extra-configs 0 --cpu-seconds 0 --host-path 0 --verify sample $*"
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in ${AB_VARIANTS:-aot jit8 jit4}; do
    case $v in
      aot) E="HEC_JIT=0"; T="";;
      jit8) E="HEC_JIT=async"; T="--tune 10=8";;
      jit4) E="HEC_JIT=async"; T="--tune 10=4";;
      jit4p2) E="HEC_JIT=async"; T="--tune 10=4,24=2";;
      jit4w3) E="HEC_JIT=async"; T="--tune 10=4,16=3";;
      jit8p3) E="HEC_JIT=async"; T="--tune 10=8,24=3";;
      jit8p4) E="HEC_JIT=async"; T="--tune 10=8,24=4";;
      jit4p4) E="HEC_JIT=async"; T="--tune 10=4,24=4";;
      jit4p5) E="HEC_JIT=async"; T="--tune 10=4,24=5";;
      jitdef) E="HEC_JIT=async"; T="--tune 11=0";;
      s15) E="HEC_JIT=async"; T="--tune 11=12";;
      rot*) E="HEC_JIT=async"; T="--tune 25=${v#rot}";;
      jit8p5) E="HEC_JIT=async"; T="--tune 10=8,24=5";;
      jit4cold) E="HEC_JIT=async HEC_JIT_CACHE=$o/cache.$rep.$RANDOM"; T="--tune 10=4";;
    esac
    d="$o/$v.$rep"
    export $E
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv -- \
      python3 -u bench.py $B $T > "$d.log" 2>&1 || { tail -20 "$d.log"; exit 2; }
    unset HEC_JIT HEC_JIT_CACHE
    python3 - "$d" "$v" "$d.log" <<'PY'
import csv, glob, json, sys
d, v, log = sys.argv[1:]
rows = []
for p in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
line = [l for l in open(log) if l.startswith("{") and '"metric"' in l][-1]
c = json.loads(line).get("crc32c", {})
for r in rows:
    if "gf_fused_crc" in r["Name"]:
        print(v, round(float(r["AverageNs"]) / 1e6, 4), "ms x", r["Calls"], r["Name"][:110])
print(v, "leg", c.get("decode_verify_ms"), "frac", c.get("decode_verify_frac"), c.get("decode_verify_kernel"), c.get("jit"),
      "| encode+crc leg", c.get("encode_crc_ms"), "frac", c.get("encode_crc_frac"))
PY
  done
done
