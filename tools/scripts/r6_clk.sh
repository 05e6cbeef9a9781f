#!/bin/bash
# Measurement: sclk / power / GPU use sampled by rocm-smi while the batched pipeline runs.
cd $GRAFT_REPO_ROOT
timeout -k 10 150 python3 tools/scripts/batch_pipe.py 4 8 ${1:-3000} both > gpurun_out/clk_pipe.txt 2>&1 &
P=$!
: > gpurun_out/clk_load.txt
while kill -0 $P 2>/dev/null; do
  echo "t=$SECONDS $(rocm-smi --showclocks --showpower --showuse 2>&1 | grep -E 'sclk|Power \(W\)|GPU use' | sed 's/GPU\[0\]\s*: //' | tr '\n' ' ')" >> gpurun_out/clk_load.txt
  sleep 1
done
wait $P
cat gpurun_out/clk_load.txt; cat gpurun_out/clk_pipe.txt
