# round 3: driver-shaped bench (20 steps, 5 warmup) for chain LDS requests and in-flight counts
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "56 20" "40 20" "28 20" "56 12" "40 12"; do
  set -- $cfg
  HOH_CHAIN_LDS_KB=$1 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --inflight $2 --no-cpu-baseline --no-config2 --no-pmc --no-legs > gpurun_out/bv.json 2> gpurun_out/bv.err || { tail -20 gpurun_out/bv.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bv.json'));print('lds=$1 inflight=$2', d['value'], d['ms_per_step'], d['detail']['bit_exact_vs_reference'])" | tee -a gpurun_out/bv.txt
done
