#!/bin/bash
# Measurement (GPU box): the natural -s0 pipeline (nat0_pipe.py 4 8 6), natural -s0 single
# encode / decode and the -s4 encode (natural_prof.py) per configuration LIB[:VAR=VAL,...],
# alternated 3 times.  Usage: r5_ab_nat0.sh CFG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for cfg in "$@"; do
    lib=${cfg%%:*}; envs=""
    [ "$lib" != "$cfg" ] && envs=${cfg#*:}
    a=$(env HOH_LIB=$lib ${envs//,/ } timeout -k 10 120 python3 tools/scripts/nat0_pipe.py 4 8 6 2>&1 | grep '^natural' | sed 's/natural -s0 pipeline //') || exit 1
    b=$(env HOH_LIB=$lib ${envs//,/ } timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 0 5 2>&1 | grep '^natural' | sed 's/.*B (sha/(sha/') || exit 1
    c=$(env HOH_LIB=$lib ${envs//,/ } timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 4 3 2>&1 | grep '^natural' | sed 's/.*B (sha/(sha/;s/, decode.*//') || exit 1
    echo "rep $rep $cfg: $a | $b | s4 $c"
  done
done
