# round 3: natural decode (chain tiles) lossless + kernel trace; then the natural / decode tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/scripts/natural_prof.py 8192 0 3 2>&1 | tee gpurun_out/chain2.txt || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_chain -o p -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 0 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_chain.txt 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_natural.py tests/test_gpu_decode.py tests/test_gpu_sizes.py -x -v --timeout 170 --timeout-method thread > gpurun_out/t4.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t4.log | tail -20
exit $rc
