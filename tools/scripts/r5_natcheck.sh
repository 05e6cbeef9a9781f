#!/bin/bash
# Round 5: natural-image parity + repeatability + per-speed kernel stats (one image at a time).
# Usage (GPU box): bash tools/scripts/r5_natcheck.sh TAG [SPEEDS]   -> gpurun_out/TAG_*
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; speeds=${2:-"1 2 3 4"}
timeout -k 10 400 python -u -m pytest tests/test_gpu_natural.py tests/test_gpu_search.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
REPS=${REPS:-8} timeout -k 10 300 python -u tools/scripts/rep_speed.py $speeds > gpurun_out/${tag}_rep.txt 2>&1 || exit 1
cat gpurun_out/${tag}_rep.txt
for sp in $speeds; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_prof$sp -o p -- \
    python3 tools/scripts/natural_prof.py 8192 $sp 3 > gpurun_out/${tag}_nat$sp.txt 2>&1 || exit 1
  grep natural gpurun_out/${tag}_nat$sp.txt
done
exit 0
