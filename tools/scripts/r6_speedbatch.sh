#!/bin/bash
# Measurement: -s>=1 stacked batches of small natural images (check build: stack knob) against one
# image per stack.  Output: gpurun_out/speedbatch.txt
cd $GRAFT_REPO_ROOT
CL=hoh-ans_amd/lib/libhohgpu_check.so
for cfg in "1024 1024 32 1" "1024 1024 32 4" "2048 2048 8 2" "512 512 64 3"; do
  for stk in 1 1024; do
    HOH_LIB=$CL HOH_SPEED_STACK_TILES=$stk timeout -k 10 120 python3 tools/scripts/speed_batch_small.py $cfg 3 2>&1 | grep ms/image || exit 1
  done
done
