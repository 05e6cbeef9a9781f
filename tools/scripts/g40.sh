#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_decode.py tests/test_gpu_shard.py tests/test_gpu_search.py tests/test_gpu_async.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 5 300 python bench.py --no-cpu-baseline --steps 64 > gpurun_out/bench.json 2>gpurun_out/bench.err && python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d['detail']['kernel_avg_ms_one_in_flight'])"
