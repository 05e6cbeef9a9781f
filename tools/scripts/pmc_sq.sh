#!/bin/bash
# Issue cost per kernel (rocprofv3 PMC, SQ counters in one pass) on the bench workload with one
# image in flight: SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / clock = the kernel's share of the
# chip's VALU issue, which bounds throughput when many images are in flight.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_sq -o p -- python3 bench.py --inflight 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq.log 2>&1
