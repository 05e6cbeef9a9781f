#!/bin/bash
# Instruction mix per kernel (rocprofv3 SQ counters, one pass) over two encode+decode passes of
# the bench image (bench.py --pmc-probe).  Output: gpurun_out/pmc_insts/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmc_insts -o p -- python3 bench.py --pmc-probe > gpurun_out/pmc_insts.log 2>&1
