#!/bin/bash
# Round 5 quick check (GPU box): the one-image trace (tools/scripts/single_trace.py) and a subset of
# parity tests.  Usage: bash tools/scripts/r5_quick.sh TAG [pytest args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; shift
(cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_tr -o t -- \
   python3 $GRAFT_REPO_ROOT/tools/scripts/single_trace.py 8192 4) > gpurun_out/${tag}_tr.log 2>&1 || { tail gpurun_out/${tag}_tr.log; exit 1; }
grep -E "^encode" gpurun_out/${tag}_tr.log
python3 tools/scripts/single_trace.py --show gpurun_out/${tag}_tr/t_kernel_trace.csv | grep -v -E "at::native|rocclr" | tail -28
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > gpurun_out/${tag}_tests.log 2>&1
  rc=$?; tail -4 gpurun_out/${tag}_tests.log; exit $rc
fi
