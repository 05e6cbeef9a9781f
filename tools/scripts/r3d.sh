# round 3: natural decode with the chain tiles (lossless, timing per LZ_XROW), then every -m gpu test
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for x in 16 4 1 64; do
  HOH_LZ_XROW=$x timeout -k 10 120 python -u tools/scripts/natural_prof.py 8192 0 3 2>&1 | sed "s/^/xrow=$x /" | tee -a gpurun_out/chain.txt || exit 1
done
timeout -k 10 120 python -u tools/scripts/noix_bench.py natural 8192 3 2>&1 | tee -a gpurun_out/chain.txt || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/t3.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t3.log | tail -20
exit $rc
