#!/bin/bash
# A/B of two library builds on the batched -s0 pipeline (tools/scripts/batch_pipe.py 4 8 K both),
# alternating A, B, A, B ... REPS times.  Usage: tools/scripts/r6_ab.sh LIB_A LIB_B [REPS] [K]
set -e
cd "$(dirname "$0")/../.."
A=$1; B=$2; R=${3:-3}; K=${4:-40}
for r in $(seq 1 $R); do
  for L in $A $B; do
    echo -n "$L: "
    HOH_LIB=$L HOH_QUIET=1 timeout -k 10 120 python3 tools/scripts/batch_pipe.py 4 8 $K both 2>/dev/null | grep -v lossless | tr '\n' ' '
    echo
  done
done
