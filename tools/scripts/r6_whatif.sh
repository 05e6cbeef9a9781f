#!/bin/bash
# Round 6 what-ifs on the batched -s0 pipeline (measurement only; outputs invalid for EXP != 0):
# the checking build (knobs on) with HOH_EXP = 0 (as shipped), 1 (every chain table gather an L2
# hit: 64 shared tables), 2 (no LZ screen in k_front256), 3 (both).  ms/image, encode / both.
set -e
cd "$(dirname "$0")/../.."
for e in ${EXPS:-0 1 2 3}; do
  echo "EXP=$e"
  HOH_LIB=hoh-ans_amd/lib/libhohgpu_check.so HOH_EXP=$e HOH_QUIET=1 timeout -k 10 120 \
    python3 tools/scripts/batch_pipe.py 4 8 40 enc,both
done
