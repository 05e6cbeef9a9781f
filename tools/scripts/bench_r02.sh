#!/bin/bash
# Round-2 bench evidence (outputs in gpurun_out/): the default bench line (live PMC traffic, CPU
# baselines), the N > 1 code path on a 1-rank RCCL group, config 4 (--strong) at N = 1, and
# rocprofv3 kernel stats of the one-in-flight run whose HIP-event averages the line reports.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 200 python -u bench.py --sharded --steps 40 --no-cpu-baseline --no-pmc > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err || { tail -20 gpurun_out/bench_sharded.err; exit 1; }
cat gpurun_out/bench_sharded.json
timeout -k 10 200 python -u bench.py --strong --steps 20 --inflight 8 --no-cpu-baseline --no-pmc > gpurun_out/bench_strong.json 2> gpurun_out/bench_strong.err || { tail -20 gpurun_out/bench_strong.err; exit 1; }
cat gpurun_out/bench_strong.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o run -- python3 bench.py --inflight 1 --steps 20 --warmup 2 --no-cpu-baseline --no-pmc --no-config2 > gpurun_out/prof1_bench.json 2> gpurun_out/prof1.err || { tail -20 gpurun_out/prof1.err; exit 1; }
cat gpurun_out/prof1_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof20 -o run -- python3 bench.py --steps 200 --no-cpu-baseline --no-pmc --no-config2 > gpurun_out/prof20_bench.json 2> gpurun_out/prof20.err || { tail -20 gpurun_out/prof20.err; exit 1; }
find gpurun_out/prof1 gpurun_out/prof20 -name "*stats*"
