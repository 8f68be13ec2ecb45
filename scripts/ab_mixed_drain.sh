set -o pipefail
mkdir -p gpurun_out/abm
C="--cpu-seconds 0 --host-path 0 --decode-mode mixed --k 10 --m 4"
for r in 1 2; do
for S in 512 256; do
for t in "" "6=1"; do
  timeout -k 10 120 python3 -u bench.py $C --stripes $S ${t:+--tune $t} > gpurun_out/abm/s${S}_t${t:-def}_r$r.log 2>&1 || exit 1
done; done; done
echo ok
