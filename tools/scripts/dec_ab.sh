#!/bin/bash
# A/B of a decoder knob (HOH_DEC_DBG value $1) in the pipelined decode-only and encode+decode rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
for d in 0 $1; do
  HOH_DEC_DBG=$d timeout -k 5 120 python tools/scripts/pipe.py dec 12 96 2>/dev/null | grep mode || exit 1
  HOH_DEC_DBG=$d timeout -k 5 120 python tools/scripts/pipe.py both 12 96 2>/dev/null | grep mode || exit 1
done
done
