#!/bin/bash
# Measurement (GPU box): the kernel timeline of the last natural 8192^2 -sN encode (natural_prof.py)
# under rocprofv3 --kernel-trace.  Usage: r5_tl.sh TAG "SPEEDS"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
for sp in $2; do
  d=gpurun_out/${tag}_s$sp
  timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o p -- python3 tools/scripts/natural_prof.py 8192 $sp 3 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep '^natural' $d.log
  python3 tools/scripts/timeline.py $(ls $d/*.db | head -1) k_colours 0.05
done
