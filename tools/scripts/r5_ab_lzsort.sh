#!/bin/bash
# Measurement (GPU box): natural 8192^2 -sN encodes (best of 5 per process), configurations
# alternated 3 times: "LIB:LZSORT_GRID" pairs.  Usage: r5_ab_lzsort.sh "SPEEDS" CFG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
speeds=$1; shift
for sp in $speeds; do
  for rep in 1 2 3; do
    for cfg in "$@"; do
      lib=${cfg%%:*}; g=${cfg##*:}
      r=$(HOH_LIB=$lib HOH_LZSORT_GRID=$g timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 $sp 5 2>&1 | grep '^natural') || exit 1
      echo "-s$sp rep $rep $cfg: $(echo "$r" | sed 's/.*B (sha/(sha/;s/, decode.*//')"
    done
  done
done
