#!/bin/bash
# Round 6, the batch chain-tile threshold: the whole -m gpu suite, the natural -s0 pipeline and one
# natural image, then the driver-shaped bench line (its natural_s0 leg is the batched decode).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6x_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6x_tests.log; exit 1; }
tail -1 gpurun_out/r6x_tests.log
timeout -k 10 150 python3 tools/scripts/nat0_pipe.py 4 8 10 || exit 1
timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 0 5 || exit 1
timeout -k 10 600 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r6x_bench.json 2> gpurun_out/r6x_bench.err || { tail -20 gpurun_out/r6x_bench.err; exit 1; }
grep '^{' gpurun_out/r6x_bench.json | tail -1 | cut -c1-200
