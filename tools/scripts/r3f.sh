# round 3: natural decode timing per LZ_XROW with the chain tiles on a second stream, then tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for x in 16 8 4 1; do
  HOH_LZ_XROW=$x timeout -k 10 120 python -u tools/scripts/natural_prof.py 8192 0 3 2>&1 | grep natural | sed "s/^/xrow=$x /" | tee -a gpurun_out/chain3.txt || exit 1
done
timeout -k 10 120 python -u tools/scripts/noix_bench.py synth 8192 3 2>&1 | grep no-index | tee -a gpurun_out/chain3.txt || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread > gpurun_out/t5.log 2>&1; rc=$?
grep -E "FAIL|ERROR|passed|failed" gpurun_out/t5.log | tail -20
[ $rc -eq 0 ] || exit $rc
# the driver's bench shape (20 steps, 5 warmup) for chain LDS requests and in-flight counts
for cfg in "56 20" "40 20" "28 20" "56 12" "40 12"; do
  set -- $cfg
  HOH_CHAIN_LDS_KB=$1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inflight $2 --no-cpu-baseline --no-config2 --no-pmc --no-legs > gpurun_out/bv.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/bv.json'));print('lds=$1 inflight=$2', d['value'], d['ms_per_step'], d['detail']['bit_exact_vs_reference'])" | tee -a gpurun_out/chain3.txt
done
