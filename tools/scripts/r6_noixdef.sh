set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_natural.py tests/test_gpu_decode.py tests/test_gpu_batch.py tests/test_gpu_sizes.py tests/test_gpu_async.py tests/test_gpu_shard_batch.py > gpurun_out/r6nb_tests.log 2>&1 \
  || { tail -30 gpurun_out/r6nb_tests.log; exit 1; }
tail -1 gpurun_out/r6nb_tests.log
for rep in 1 2; do
  r=$(timeout -k 10 200 python3 bench.py --no-index --steps 10 --warmup 3 --no-legs --no-pmc --no-cpu-baseline --no-config2 2>/dev/null | grep '^{' | tail -1) || exit 1
  echo "rep $rep product no-index pipeline: $(echo "$r" | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["unit"], d["ms_per_step"], d["detail"].get("lossless"))')"
done
for sz in 8192 16384; do
  HOH_QUIET=1 timeout -k 10 200 python3 tools/scripts/noix_bench.py natural $sz 3 adaptive 2>&1 | grep '^no-index' || exit 1
done
