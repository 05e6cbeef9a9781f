#!/bin/bash
# Round 6: the no-index decoder (k_drans_multi pinned, synthetic and natural 8192^2, one image at a
# time) with several library builds, alternating.  Usage: r6_noix.sh LIB...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for r in 1 2; do
  for L in "$@"; do
    for k in synth natural; do
      echo -n "$L: "
      HOH_LIB=$L HOH_QUIET=1 timeout -k 10 120 python3 tools/scripts/noix_bench.py $k 8192 5 multi 2>&1 | grep '^no-index' || exit 1
    done
  done
done
