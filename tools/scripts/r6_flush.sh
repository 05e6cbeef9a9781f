#!/bin/bash
# Measurement (GPU box): counting trial lanes count their emitted words by one popcount per flush
# -- parity (ladder bounds and lists through the checking build, natural goldens, search, batches),
# then natural 8192^2 -s1/-s4 encodes against var/preflush.so, alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_search.py tests/test_gpu_check_build.py tests/test_gpu_batch_speed.py > gpurun_out/r6fl_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6fl_tests.log; exit 1; }
tail -1 gpurun_out/r6fl_tests.log
bash tools/scripts/r5_ab_lzsort.sh "1 4" var/preflush.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
