#!/bin/bash
# A/B/C... of library builds on batch_pipe.py D B K MODE, alternating REPS times.
# Usage: tools/scripts/r6_abmode.sh REPS "D B K MODE" LIB...
set -e
cd "$(dirname "$0")/../.."
R=$1; ARGS=$2; shift 2
for r in $(seq 1 $R); do
  for L in "$@"; do
    echo -n "$L: "
    HOH_LIB=$L HOH_QUIET=1 timeout -k 10 120 python3 tools/scripts/batch_pipe.py $ARGS 2>/dev/null | grep -v lossless | tr '\n' ' '
    echo
  done
done
