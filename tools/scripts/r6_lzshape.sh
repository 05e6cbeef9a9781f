#!/bin/bash
# Measurement (GPU box): the per-speed k_lzsort shape -- parity (natural goldens, search, posting
# lists at -s2 (1024 shape) and -s4 (512 shape), batches, drop-in choh), then natural 8192^2
# -s3/-s4 encodes against var/knobs.so (1024 shape at every speed) and the -s4 HBM bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_search.py tests/test_gpu_check_build.py tests/test_gpu_batch_speed.py tests/test_gpu_dropin_ref.py tests/test_gpu_encode.py > gpurun_out/r6z_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6z_tests.log; exit 1; }
tail -1 gpurun_out/r6z_tests.log
bash tools/scripts/r5_ab_lzsort.sh "3 4" var/knobs.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
HOH_LIB=hoh-ans_amd/lib/libhohgpu.so bash tools/scripts/r5_spmc.sh r6z_new 4 || exit 1
