#!/bin/bash
# A/B of variant libraries (HOH_LIB) on the bench: 200 steps and the driver's 20 steps
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/abb; mkdir -p $O
B="--no-legs --no-pmc --no-cpu-baseline --no-config2"
for v in "$@"; do
  n=$(basename $v .so)
  if [ "$v" = base ]; then unset HOH_LIB; else export HOH_LIB=$GRAFT_REPO_ROOT/$v; fi
  timeout -k 10 200 python -u bench.py --steps 200 $B > $O/${n}_200.json 2>$O/err || { tail $O/err; exit 1; }
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 $B > $O/${n}_20.json 2>$O/err || { tail $O/err; exit 1; }
  python -c "import json; a=json.load(open('$O/${n}_200.json')); b=json.load(open('$O/${n}_20.json')); print('$n', '200:', a['value'], '20:', b['value'])"
done
