#!/bin/bash
# Encoder parity, then the front kernel alone and the pipelined encode rate.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/enc_tests.log 2>&1 || { tail -30 gpurun_out/enc_tests.log; exit 1; }
tail -2 gpurun_out/enc_tests.log
timeout -k 5 200 python tools/scripts/knobs.py front 0 4 2>/dev/null | grep dbg || exit 1
timeout -k 5 120 python tools/scripts/pipe.py enc 12 96 2>/dev/null | grep mode || exit 1
timeout -k 5 120 python tools/scripts/pipe.py both 12 96 2>/dev/null | grep mode
