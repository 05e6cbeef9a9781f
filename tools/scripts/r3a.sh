# round 3: no-index decoder timing, natural -s1 encode timing, then every -m gpu test (one process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/scripts/noix_bench.py synth 8192 5 2>&1 | tee gpurun_out/noix.txt
timeout -k 10 120 python -u tools/scripts/noix_bench.py natural 8192 3 2>&1 | tee -a gpurun_out/noix.txt
timeout -k 10 150 python -u tools/scripts/natural_prof.py 8192 1 2 2>&1 | tee -a gpurun_out/noix.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t1.log | tail -20
exit $rc
