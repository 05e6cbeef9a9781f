#!/bin/bash
# pipelined cost per stage (12 in flight, enqueue-only): encode / decode only, with stage stops
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/stages.txt
run() { HOH_ENC_DBG=$1 HOH_DEC_DBG=$2 timeout -k 5 120 python tools/scripts/pipe.py $3 12 96 >> gpurun_out/stages.txt 2>&1; }
run 0 0 both && run 0 0 enc && run 0 0 dec && run 65536 0 enc && run 262144 0 enc && run 4 0 enc && run 0 256 dec
