#!/bin/bash
# Measurement (GPU box): the no-index pipeline (bench.py --no-index: 4 contexts x batches of 8,
# every stream decoded as one serial chain) through var/knobs.so at several k_drans_lanes LDS
# budgets / workgroups per CU.  Usage: r6_noixknobs.sh "BUDGET_KB:WG" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for cfg in "$@"; do
    b=${cfg%%:*}; w=${cfg##*:}
    r=$(HOH_LIB=var/knobs.so HOH_DL_BUDGET_KB=$b HOH_DL_WG=$w timeout -k 10 200 python3 bench.py --no-index --steps 10 --warmup 3 \
        --no-legs --no-pmc --no-cpu-baseline --no-config2 2>/dev/null | grep '^{' | tail -1) || exit 1
    echo "rep $rep budget ${b} KB x $w WG/CU: $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["unit"], d["ms_per_step"])')"
  done
done
