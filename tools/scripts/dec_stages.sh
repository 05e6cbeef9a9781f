#!/bin/bash
# pipelined decode cost per stage (HOH_DEC_DBG stage stops; output invalid when stopped)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for d in 0 256; do
  HOH_DEC_DBG=$d timeout -k 5 120 python tools/scripts/pipe.py dec 12 96 >> gpurun_out/dec_stages.txt 2>&1 || exit 1
done
