#!/bin/bash
# Round 6, last GPU check at the final code: smoke(), the whole -m gpu suite, and the N > 1 code
# path's one-rank rehearsal (bench.py --sharded: batched shards + the RCCL gather on a one-rank group).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6l_smoke.log 2>&1 || { tail -20 gpurun_out/r6l_smoke.log; exit 1; }
tail -1 gpurun_out/r6l_smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6l_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6l_tests.log; exit 1; }
tail -1 gpurun_out/r6l_tests.log
timeout -k 10 300 python -u bench.py --sharded --steps 20 --no-cpu-baseline --no-pmc --no-legs --no-config2 > gpurun_out/r6l_sharded.json 2> gpurun_out/r6l_sharded.err \
  || { tail -20 gpurun_out/r6l_sharded.err; exit 1; }
grep '^{' gpurun_out/r6l_sharded.json | tail -1 | cut -c1-220
