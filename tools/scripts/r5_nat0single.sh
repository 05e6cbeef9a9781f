#!/bin/bash
# Measurement (GPU box): natural 8192^2 -s0, one image at a time (natural_prof.py), under
# rocprofv3 --kernel-trace: the kernel timeline of the last encode and the decodes after it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$tag -o p -- python3 tools/scripts/natural_prof.py 8192 0 3 \
  > gpurun_out/$tag.log 2>&1 || { tail -5 gpurun_out/$tag.log; exit 1; }
grep '^natural' gpurun_out/$tag.log
python3 tools/scripts/timeline.py $(ls gpurun_out/$tag/*.db | head -1) k_colours 0.02
