set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in var/nukeold.so var/lzold.so hoh-ans_amd/lib/libhohgpu.so; do
  echo "== $lib"
  HOH_LIB=$lib timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_batch_speed.py tests/test_gpu_natural.py -k "natural_768 or vs_reference" 2>&1 | tail -4
done
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_check_build.py -k posting 2>&1 | tail -4
