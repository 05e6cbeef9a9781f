#!/bin/bash
# Measurement (GPU box): the -s>=1 chains with 32-bit table offsets when the job's tables stay
# under 4 GB -- parity (search, natural, posting lists / ladder bounds, batches incl. the 4.7 GB
# stack, entropy API, drop-in choh), then natural 8192^2 -s1..-s4 encodes against var/knobs.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_search.py tests/test_gpu_check_build.py tests/test_gpu_batch_speed.py tests/test_gpu_encode.py tests/test_gpu_dropin_ref.py tests/test_gpu_plane_s.py > gpurun_out/r6nw_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6nw_tests.log; exit 1; }
tail -1 gpurun_out/r6nw_tests.log
bash tools/scripts/r5_ab_lzsort.sh "1 4" var/knobs.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
