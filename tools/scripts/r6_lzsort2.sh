#!/bin/bash
# Measurement (GPU box): the whole -m gpu suite, then natural 8192^2 -s0/-s1/-s4 encodes A/B against
# var/base.so and the -s4 HBM bytes per launch.  Usage: r6_lzsort2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
tag=$1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 \
  || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
bash tools/scripts/r5_ab_lzsort.sh "0 1 4" var/base.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
HOH_LIB=hoh-ans_amd/lib/libhohgpu.so bash tools/scripts/r5_spmc.sh ${tag}_new 4 || exit 1
