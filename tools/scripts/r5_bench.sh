#!/bin/bash
# Round 5 bench runs (GPU box).  Usage: bash tools/scripts/r5_bench.sh TAG [MODE]
#   MODE full: the driver's command (python bench.py --steps 20 --warmup 5), everything on
#   MODE q4:   --hw-queues 4 (HIP's default) without legs/baselines
#   MODE legs: legs only (no cpu baseline / config2 / pmc)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1; mode=${2:-full}
case $mode in
  full) args="--steps 20 --warmup 5" ;;
  q4)   args="--steps 20 --warmup 5 --hw-queues 4 --no-legs --no-cpu-baseline --no-config2 --no-pmc" ;;
  legs) args="--steps 20 --warmup 5 --no-cpu-baseline --no-config2 --no-pmc" ;;
  *)    args="$mode" ;;
esac
timeout -k 10 900 python -u bench.py $args > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc=$?
tail -c 3000 gpurun_out/${tag}_bench.json; tail -3 gpurun_out/${tag}_bench.err
exit $rc
