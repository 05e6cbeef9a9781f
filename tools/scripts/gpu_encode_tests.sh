set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_encode.py -x -q -m gpu > gpurun_out/t1.log 2>&1
rc=$?
tail -30 gpurun_out/t1.log
exit $rc
