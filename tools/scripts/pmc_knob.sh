#!/bin/bash
# instruction mix of one kernel under an HOH_ENC_DBG knob (knobs.py KERNEL DBG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmcK -o p -- python3 tools/scripts/knobs.py $1 $2 > gpurun_out/pmcK.log 2>&1
