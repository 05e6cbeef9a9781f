set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; rm -f gpurun_out/sweep.txt
timeout -k 10 500 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_search.py tests/test_gpu_shard.py tests/test_gpu_async.py tests/test_gpu_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 5 200 python tools/scripts/knobs.py front 0 2>/dev/null | grep dbg || exit 1
tools/scripts/bench_sweep.sh 0 0 0 && cut -c1-60 gpurun_out/sweep.txt
