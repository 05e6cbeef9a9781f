#!/bin/bash
# HBM traffic per kernel (rocprofv3 PMC, one counter group per pass as the MI355X guide requires),
# on the bench workload with one image in flight.  Output: gpurun_out/pmc_{fetch,write}/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o p -- python3 bench.py --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o p -- python3 bench.py --inflight 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --inflight 1 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof1_bench.json 2> gpurun_out/prof1.err
