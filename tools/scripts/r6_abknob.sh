#!/bin/bash
# Measurement (GPU box): natural 8192^2 -sN encodes (best of 5 per process) through var/knobs.so,
# knob settings alternated 3 times.  Usage: r6_abknob.sh "SPEEDS" "ENV1" "ENV2" ...
#   e.g. r6_abknob.sh "1 2 3 4" "HOH_LZFP_FIRST=0" "HOH_LZFP_FIRST=4"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
speeds=$1; shift
for sp in $speeds; do
  for rep in 1 2 3; do
    for cfg in "$@"; do
      r=$(env HOH_LIB=var/knobs.so $cfg timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 $sp 5 2>&1 | grep '^natural') || exit 1
      echo "-s$sp rep $rep $cfg: $(echo "$r" | sed 's/.*B (sha/(sha/;s/, decode.*//')"
    done
  done
done
