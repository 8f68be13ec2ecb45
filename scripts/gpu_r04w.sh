#!/bin/bash
# round-4 last tree (fused grid 32 per CU, 8-stripe groups), product library only: the -m gpu suite, smoke, the default
# bench line, and the bench config / CRC legs / mixed decode profiles
set -o pipefail
bash scripts/gpu_round.sh gpurun_out/r04w rs63 crc63 mx104
