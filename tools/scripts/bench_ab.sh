#!/bin/bash
# bench.py value with and without a decoder knob (HOH_DEC_DBG=$1), alternating, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
for d in 0 $1; do
  HOH_DEC_DBG=$d timeout -k 5 300 python bench.py --no-cpu-baseline > gpurun_out/bab.json 2>gpurun_out/bab.err || { tail -5 gpurun_out/bab.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/bab.json'));print('dec_dbg=$d', d['value'], d['ms_per_step'])"
done
done
