#!/bin/bash
# Measurement (GPU box): k_lzscan at -s1/-s2 loading each vertical hit's first image word during the
# horizontal walk -- parity (natural goldens, search, posting lists, batches), then natural 8192^2
# -s1/-s2 encodes against var/prevert.so (HEAD without it), alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_search.py tests/test_gpu_check_build.py tests/test_gpu_batch_speed.py > gpurun_out/r6vp_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6vp_tests.log; exit 1; }
tail -1 gpurun_out/r6vp_tests.log
bash tools/scripts/r5_ab_lzsort.sh "1 2" var/prevert.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
