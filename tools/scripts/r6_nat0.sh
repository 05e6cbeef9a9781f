#!/bin/bash
# Round 6: natural 8192^2 -s0 one image at a time (natural_prof.py: encode + decode, 3 reps) with
# several library builds, alternating; prints each build's times.  Usage: r6_nat0.sh LIB...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for L in "$@"; do
    echo -n "$L: "
    HOH_LIB=$L HOH_QUIET=1 timeout -k 10 120 python3 tools/scripts/natural_prof.py 8192 0 5 2>&1 | grep '^natural' || exit 1
  done
done
