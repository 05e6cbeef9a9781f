#!/bin/bash
# Measurement (GPU box): the chunk-staged k_lzsort -- posting-list exactness, natural and search
# parity, then natural 8192^2 -s1/-s4 encodes A/B against var/base.so and the -s4 HBM bytes per
# launch (FETCH / WRITE passes).  Usage: r6_lzsort.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_check_build.py tests/test_gpu_natural.py tests/test_gpu_search.py > gpurun_out/${tag}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
bash tools/scripts/r5_ab_lzsort.sh "1 4" var/base.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
HOH_LIB=hoh-ans_amd/lib/libhohgpu.so bash tools/scripts/r5_spmc.sh ${tag}_new 4 || exit 1
HOH_LIB=var/base.so bash tools/scripts/r5_spmc.sh ${tag}_base 4 || exit 1
