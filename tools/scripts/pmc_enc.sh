#!/bin/bash
# PMC passes over the encoder kernels (measurement only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmcEA -o p -- python3 tools/scripts/enc_timing.py 8192 > gpurun_out/pmcEA.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmcEB -o p -- python3 tools/scripts/enc_timing.py 8192 > gpurun_out/pmcEB.log 2>&1
