#!/bin/bash
# Encoder/decoder parity subset, then the chain time alone, the pipelined encode rate and a bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_encode.py tests/test_gpu_decode.py tests/test_gpu_search.py tests/test_gpu_async.py tests/test_gpu_shard.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 5 200 python tools/scripts/knobs.py rans_enc_fast 0 > gpurun_out/knobs.txt 2>&1 && cat gpurun_out/knobs.txt
timeout -k 5 200 python tools/scripts/pipe.py enc 12 96 > gpurun_out/pipe1.txt 2>&1 && cat gpurun_out/pipe1.txt
timeout -k 5 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err && python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
