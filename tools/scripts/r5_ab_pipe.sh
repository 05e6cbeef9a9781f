#!/bin/bash
# Measurement (GPU box): the batched synthetic pipeline (batch_pipe.py: encode only, decode only,
# both; 4 contexts x 8 images, 40 steps) for several libraries, alternated 3 times, plus natural
# -s0 single-image encode / decode (natural_prof.py).  A configuration is LIB[:VAR=VAL[,VAR=VAL...]]
# (HOH_ knobs of a knobs build).  Usage: r5_ab_pipe.sh CFG...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2 3; do
  for cfg in "$@"; do
    lib=${cfg%%:*}; envs=""
    [ "$lib" != "$cfg" ] && envs=${cfg#*:}
    r=$(env HOH_LIB=$lib ${envs//,/ } timeout -k 10 120 python3 tools/scripts/batch_pipe.py 4 8 40 2>&1 | grep -E "ms/image|lossless" | tr '\n' ' ') || exit 1
    n=$(env HOH_LIB=$lib ${envs//,/ } timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 0 5 2>&1 | grep '^natural' | sed 's/.*B (sha/(sha/') || exit 1
    echo "rep $rep $cfg: $r | $n"
  done
done
