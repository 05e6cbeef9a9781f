#!/bin/bash
# End-of-round evidence: parity tests, smoke, bench, rocprofv3 stats, PMC traffic passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tools/scripts/round_gpu.sh > gpurun_out/round.log 2>&1 || { tail -30 gpurun_out/round.log; exit 1; }
tail -4 gpurun_out/gpu_tests.log
tools/scripts/pmc.sh || { echo "pmc failed"; exit 1; }
python tools/scripts/make_pmc_json.py gpurun_out/pmc_fetch/p_counter_collection.csv gpurun_out/pmc_write/p_counter_collection.csv gpurun_out/pmc.json
find gpurun_out/prof gpurun_out/prof1 -name "*stats*"
cat gpurun_out/bench.json
