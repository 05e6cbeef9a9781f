#!/bin/bash
# Decoder parity, then pipelined decode-only and encode+decode rates.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_async.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/dec_tests.log 2>&1 || { tail -30 gpurun_out/dec_tests.log; exit 1; }
tail -2 gpurun_out/dec_tests.log
timeout -k 5 120 python tools/scripts/pipe.py dec 12 96 2>/dev/null | grep mode || exit 1
timeout -k 5 120 python tools/scripts/pipe.py both 12 96 2>/dev/null | grep mode || exit 1
timeout -k 5 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err && python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'])"
