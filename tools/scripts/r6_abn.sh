#!/bin/bash
# A/B/C... of library builds on the batched -s0 pipeline (batch_pipe.py 4 8 K both), alternating
# REPS times.  Usage: tools/scripts/r6_abn.sh REPS K LIB...
set -e
cd "$(dirname "$0")/../.."
R=$1; K=$2; shift 2
for r in $(seq 1 $R); do
  for L in "$@"; do
    echo -n "$L: "
    HOH_LIB=$L HOH_QUIET=1 timeout -k 10 120 python3 tools/scripts/batch_pipe.py 4 8 $K both 2>/dev/null | grep -v lossless | tr '\n' ' '
    echo
  done
done
