#!/bin/bash
# Measurement (GPU box): k_lzvert beside k_lzsort at -s1/-s2 (its own bitmap) -- parity (natural
# goldens, search, posting lists, -s>=1 batches), then natural 8192^2 -s1/-s2 encodes through
# var/knobs.so, LZVERT_SEP=0 (after k_lzsort) against 2, and the -s1 timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_search.py tests/test_gpu_check_build.py tests/test_gpu_batch_speed.py tests/test_gpu_dropin_ref.py > gpurun_out/r6v_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6v_tests.log; exit 1; }
tail -1 gpurun_out/r6v_tests.log
bash tools/scripts/r6_abknob.sh "1 2" "HOH_LZVERT_SEP=0" "HOH_LZVERT_SEP=2" || exit 1
bash tools/scripts/r5_tl.sh r6vtl "1" || exit 1
