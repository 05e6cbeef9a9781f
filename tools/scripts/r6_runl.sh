#!/bin/bash
# Measurement (GPU box): k_lzscan's image-path run lengths with the older side's first 16 words in
# one round trip -- parity (natural goldens, search, posting lists), then natural 8192^2 -s1..-s4
# encodes against var/prerunl.so (the same code with two round trips) and the k_lzscan timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_search.py tests/test_gpu_check_build.py tests/test_gpu_batch_speed.py > gpurun_out/r6r_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6r_tests.log; exit 1; }
tail -1 gpurun_out/r6r_tests.log
bash tools/scripts/r5_ab_lzsort.sh "1 2 3 4" var/prerunl.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
bash tools/scripts/r5_tl.sh r6rtl "3 4" || exit 1
