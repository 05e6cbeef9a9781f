#!/bin/bash
# Round-5 closing evidence (GPU box): the driver-shaped bench line, then the same bench command
# under rocprofv3 --kernel-trace --stats (kernel summary for profiles/).  Usage: r5_final2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r5g}
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
grep '^{' gpurun_out/${tag}_bench.json | tail -1 | cut -c1-240
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o p -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc \
  > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
find gpurun_out/${tag}_prof -name '*stats*' | head
