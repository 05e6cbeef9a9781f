#!/bin/bash
# Pipelined encode/decode throughput under measurement knobs (see pipe.py); results appended to
# gpurun_out/pipe.txt.  usage: pipe_run.sh "MODE D K [ENC_DBG]" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in "$@"; do
  set -- $m
  HOH_ENC_DBG=${4:-0} timeout -k 5 120 python tools/scripts/pipe.py $1 $2 $3 >> gpurun_out/pipe.txt 2>&1 || exit 1
done
