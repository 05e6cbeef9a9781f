#!/bin/bash
# Decoder parity, then decode-only / encode+decode pipelines and the bench with and without a
# decoder knob (HOH_DEC_DBG=$1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_async.py tests/test_gpu_shard.py tests/test_gpu_cli.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
tools/scripts/dec_ab.sh $1 && tools/scripts/bench_ab.sh $1
