# round 3: no-index decoder timing + the parity tests touched this round (one process each step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/scripts/noix_bench.py synth 8192 5 2>&1 | tee gpurun_out/noix.txt
timeout -k 10 120 python -u tools/scripts/noix_bench.py natural 8192 3 2>&1 | tee -a gpurun_out/noix.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_sizes.py tests/test_gpu_decode.py tests/test_gpu_cli.py tests/test_gpu_mgpu.py tests/test_gpu_natural.py -x -v --timeout 170 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t1.log | tail -20
exit $rc
