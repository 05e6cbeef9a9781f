#!/bin/bash
# Measurement (GPU box): k_nuke / k_dunpred_lz grids capped at a few workgroups per CU (they
# stride over the tiles) -- parity, then the headline pipeline, the natural -s0 pipeline and one
# natural -s0 image with var/knobs.so (grids of one workgroup per tile) and the product library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_decode.py tests/test_gpu_batch.py tests/test_gpu_encode.py tests/test_gpu_sizes.py > gpurun_out/r6cap_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6cap_tests.log; exit 1; }
tail -1 gpurun_out/r6cap_tests.log
for rep in 1 2 3; do
  for L in var/knobs.so hoh-ans_amd/lib/libhohgpu.so; do
    r=$(HOH_LIB=$L timeout -k 10 200 python3 bench.py --steps 40 --warmup 5 --no-legs --no-pmc --no-cpu-baseline --no-config2 2>/dev/null | grep '^{' | tail -1) || exit 1
    echo "rep $rep headline $L: $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["unit"], d["ms_per_step"], d["detail"]["slot_files_bit_exact"])')"
  done
done
for rep in 1 2; do
  for L in var/knobs.so hoh-ans_amd/lib/libhohgpu.so; do
    echo -n "rep $rep nat0 $L: "; HOH_LIB=$L timeout -k 10 200 python3 tools/scripts/nat0_pipe.py 4 8 10 || exit 1
  done
done
for L in var/knobs.so hoh-ans_amd/lib/libhohgpu.so; do
  echo -n "$L: "; HOH_LIB=$L timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 0 5 || exit 1
done
