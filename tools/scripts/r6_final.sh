#!/bin/bash
# Round-6 closing evidence (GPU box): the driver-shaped bench line, the same bench command under
# rocprofv3 --kernel-trace --stats (kernel summary for profiles/), and the one-image-in-flight
# command whose k_rans_fast01 average is the line's roofline.avg_launch_ms.  Usage: r6_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=${1:-r6z}
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
grep '^{' gpurun_out/${tag}_bench.json | tail -1 | cut -c1-240
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o p -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-pmc \
  > gpurun_out/${tag}_prof.log 2>&1 || { tail -20 gpurun_out/${tag}_prof.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_one -o p -- python3 bench.py --batch 1 --inflight 1 --steps 10 --warmup 2 --no-legs --no-pmc --no-cpu-baseline --no-config2 \
  > gpurun_out/${tag}_one.log 2>&1 || { tail -20 gpurun_out/${tag}_one.log; exit 1; }
find gpurun_out/${tag}_prof gpurun_out/${tag}_one -name '*stats*' | head
