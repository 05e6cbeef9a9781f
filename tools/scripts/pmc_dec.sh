#!/bin/bash
# PMC passes over the decode kernels (measurement only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmcA -o p -- python3 tools/scripts/dec_timing.py 8192 > gpurun_out/pmcA.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmcB -o p -- python3 tools/scripts/dec_timing.py 8192 > gpurun_out/pmcB.log 2>&1
