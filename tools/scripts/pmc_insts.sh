#!/bin/bash
# Instruction mix per kernel (one rocprofv3 --pmc pass, 8 SQ counters) of a command.
# usage: pmc_insts.sh OUTDIR -- python3 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
out=$1; shift; shift
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d gpurun_out/$out -o p -- "$@" > gpurun_out/$out.log 2>&1
