# round 3: every -m gpu test, then the default bench line (driver's command shape)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/t2.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t2.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r3.json 2> gpurun_out/bench_r3.err; rc=$?
tail -c 6000 gpurun_out/bench_r3.json; tail -5 gpurun_out/bench_r3.err
exit $rc
