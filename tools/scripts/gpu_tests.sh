#!/bin/bash
# All -m gpu parity tests in one process (outputs gpurun_out/gpu_tests.log); extra args go to pytest.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread --durations=20 "$@" > gpurun_out/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|serial|natural 8192|s[0-9] 8192" gpurun_out/gpu_tests.log | tail -60
tail -30 gpurun_out/gpu_tests.log
exit $rc
