#!/bin/bash
# Measurement (GPU box): natural 8192^2 encodes under rocprofv3 with the knobs library and a list
# of knob settings; per setting the file (size, sha) and the kernel timeline of the last encode.
# Usage: bash tools/scripts/r5_knobprof.sh TAG SPEED "KNOB=V[,KNOB=V] ..."   ("-" = defaults)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; sp=$2; cfgs=$3
for cfg in $cfgs; do
  envs=""
  [ "$cfg" != "-" ] && envs=$(echo "$cfg" | tr ',' '\n' | sed 's/^/HOH_/' | tr '\n' ' ')
  d=gpurun_out/${tag}_$(echo "$cfg" | tr ',=' '__')
  env $envs HOH_LIB=var/knobs.so timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o p -- \
    python3 tools/scripts/natural_prof.py 8192 $sp 2 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  echo "== $cfg"; grep '^natural' $d.log
  python3 tools/scripts/timeline.py $d/*.db k_front256 0.3
done
