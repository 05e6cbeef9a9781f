#!/bin/bash
# L1 (TCP) behaviour of the encoder under two HOH_ENC_DBG settings (knobs.py rans_enc_fast DBG)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for d in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d gpurun_out/pmcT_$d -o p -- python3 tools/scripts/knobs.py rans_enc_fast $d > gpurun_out/pmcT_$d.log 2>&1 || exit 1
done
