#!/bin/bash
# pitch-padding sweep (GPU box)
set -o pipefail
for cfg in "1048576 1024 6 3" "1048576 512 10 4" "65536 16384 6 3"; do
  for pad in 0 256 4096 8192 65536 69632; do
    timeout -k 10 120 ./scripts/probe_bw $cfg $pad q || exit 1
  done
done
