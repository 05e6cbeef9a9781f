# round 3: config-5 goldens at -s0..-s4 (timings printed), then kernel-trace profiles of the
# natural -s1 encode and the no-index decode
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_natural.py -v -s --timeout 170 --timeout-method thread > gpurun_out/nat.log 2>&1; rc=$?
grep -E "natural 8192|PASS|FAIL|passed|failed|SKIP" gpurun_out/nat.log | tail -20
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_s1 -o p -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 1 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_s1.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_noix -o p -- python3 $GRAFT_REPO_ROOT/tools/scripts/noix_bench.py synth 8192 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_noix.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_nat0 -o p -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 0 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_nat0.txt 2>&1 || exit 1
ls -R $GRAFT_REPO_ROOT/gpurun_out | head -30
