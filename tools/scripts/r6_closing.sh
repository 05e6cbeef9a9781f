#!/bin/bash
# Round-6 closing evidence (GPU box): the whole -m gpu suite, then r6_final.sh (the driver-shaped
# bench line, the bench command's kernel stats, the one-image-in-flight kernel stats).
# Usage: r6_closing.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r6y}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
bash tools/scripts/r6_final.sh $tag || exit 1
