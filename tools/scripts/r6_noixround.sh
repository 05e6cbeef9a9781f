#!/bin/bash
# Measurement (GPU box): the one-round rule for k_drans_multi -- decode parity, then the no-index
# pipeline (bench.py --no-index) with var/knobs.so (before) and the product library, alternated,
# and one 8192^2 image decoded without the index (adaptive: still k_drans_multi).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_decode.py tests/test_gpu_batch.py tests/test_gpu_sizes.py > gpurun_out/r6nr_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6nr_tests.log; exit 1; }
tail -1 gpurun_out/r6nr_tests.log
for rep in 1 2; do
  for L in var/knobs.so hoh-ans_amd/lib/libhohgpu.so; do
    r=$(HOH_LIB=$L timeout -k 10 200 python3 bench.py --no-index --steps 10 --warmup 3 --no-legs --no-pmc --no-cpu-baseline --no-config2 2>/dev/null | grep '^{' | tail -1) || exit 1
    echo "rep $rep $L: $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["unit"], d["ms_per_step"], d["detail"].get("lossless"))')"
  done
done
for L in var/knobs.so hoh-ans_amd/lib/libhohgpu.so; do
  echo -n "$L: "; HOH_LIB=$L HOH_QUIET=1 timeout -k 10 120 python3 tools/scripts/noix_bench.py synth 8192 5 adaptive 2>&1 | grep '^no-index' || exit 1
done
