#!/bin/bash
# round-4 final tree after the last measurement knob: GPU suite, smoke, bench,
# and the CRC legs' profile
set -o pipefail
bash scripts/gpu_round.sh gpurun_out/r04v crc63
