#!/bin/bash
# Front kernel stall profile: instruction mix, then LDS / barrier waits (two --pmc passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAVES --output-format csv -d gpurun_out/pf1 -o p -- python3 tools/scripts/knobs.py front 0 > gpurun_out/pf1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pf2 -o p -- python3 tools/scripts/knobs.py front 0 > gpurun_out/pf2.log 2>&1 || { tail -5 gpurun_out/pf2.log; exit 1; }
