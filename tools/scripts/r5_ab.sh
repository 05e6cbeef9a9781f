#!/bin/bash
# Measurement (GPU box): natural 8192^2 -sN encodes (best of 5 per process), configurations
# alternated 3 times.  A configuration is LIB[:VAR=VAL[,VAR=VAL...]] (HOH_ knobs of a knobs build).
# Usage: r5_ab.sh "SPEEDS" CFG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
speeds=$1; shift
for sp in $speeds; do
  for rep in 1 2 3; do
    for cfg in "$@"; do
      lib=${cfg%%:*}; envs=""
      [ "$lib" != "$cfg" ] && envs=${cfg#*:}
      r=$(env HOH_LIB=$lib ${envs//,/ } timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 $sp 5 2>&1 | grep '^natural') || exit 1
      echo "-s$sp rep $rep $cfg: $(echo "$r" | sed 's/.*B (sha/(sha/;s/, lossless.*//')"
    done
  done
done
