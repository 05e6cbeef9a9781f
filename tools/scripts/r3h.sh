# round 3: natural decode timing, LZ/decode tests, then driver-shaped bench variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/scripts/natural_prof.py 8192 0 3 2>&1 | grep natural | tee gpurun_out/h.txt || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_natural.py tests/test_gpu_decode.py tests/test_gpu_sizes.py tests/test_gpu_shard.py -x -v --timeout 170 --timeout-method thread > gpurun_out/t6.log 2>&1 || { grep -E "FAIL|ERROR" gpurun_out/t6.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/t6.log | tail -2
for cfg in "56 20" "40 20" "56 16"; do
  set -- $cfg
  HOH_CHAIN_LDS_KB=$1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inflight $2 --no-cpu-baseline --no-config2 --no-pmc --no-legs > gpurun_out/bv.json 2> gpurun_out/bv.err || { tail -20 gpurun_out/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bv.json'));print('lds=$1 inflight=$2', d['value'], d['ms_per_step'], d['detail']['bit_exact_vs_reference'])" | tee -a gpurun_out/h.txt
done
timeout -k 10 300 python -u bench.py --steps 200 --warmup 5 --no-cpu-baseline --no-config2 --no-pmc --no-legs > gpurun_out/bv.json 2> gpurun_out/bv.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bv.json'));print('200 steps', d['value'], d['ms_per_step'])" | tee -a gpurun_out/h.txt
