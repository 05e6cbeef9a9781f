#!/bin/bash
# Where the natural -s0 image's kernels spend their wave cycles (two rocprofv3 SQ passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_nat1 -o p -- python3 tools/scripts/natural_prof.py 8192 0 1 > gpurun_out/pmc_nat1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM --output-format csv -d gpurun_out/pmc_nat2 -o p -- python3 tools/scripts/natural_prof.py 8192 0 1 > gpurun_out/pmc_nat2.log 2>&1
