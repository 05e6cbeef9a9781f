#!/bin/bash
# bench.py under several settings: each argument is "ENC_DBG extra-bench-args"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in "$@"; do
  set -- $m
  dbg=$1; shift
  echo "== HOH_ENC_DBG=$dbg $*" >> gpurun_out/sweep.txt
  HOH_ENC_DBG=$dbg timeout -k 5 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/sweep_one.json 2>> gpurun_out/sweep.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sweep_one.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['detail']['latency_ms_enc'],d['detail']['latency_ms_dec'],d['detail']['kernel_avg_ms'])" >> gpurun_out/sweep.txt
done
