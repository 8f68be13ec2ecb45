#!/bin/bash
# round-4 final tree, product library only (the measurement build does not
# travel): the -m gpu suite, smoke, the default bench line, and one-lease
# profiles of the bench config, the CRC legs and the mixed decode
# (scripts/gpu_round.sh)
set -o pipefail
bash scripts/gpu_round.sh gpurun_out/r04z rs63 crc63 mx104
