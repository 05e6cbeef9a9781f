#!/bin/bash
# Round-4 bench evidence (outputs in gpurun_out/r04/): the driver-shaped bench line (20 steps, 5
# warmup: live PMC traffic, CPU baselines, no-index and natural legs), the 200-step line, the
# N > 1 code path on a 1-rank RCCL group (with the 16384^2 strong leg), config 4 (--strong), rocprofv3 kernel stats with one
# image in flight and with 20, and the natural-image kernel stats at -s0 / -s1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_shape.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench_driver_shape.json
timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline --no-pmc --no-config2 --no-legs > $O/bench_200.json 2> $O/bench200.err || { tail -20 $O/bench200.err; exit 1; }
timeout -k 10 200 python -u bench.py --sharded --steps 40 --no-cpu-baseline --no-pmc --no-legs --no-config2 > $O/bench_sharded.json 2> $O/bench_sharded.err || { tail -20 $O/bench_sharded.err; exit 1; }
timeout -k 10 200 python -u bench.py --strong --steps 20 --inflight 8 --no-cpu-baseline --no-pmc --no-legs --no-config2 > $O/bench_strong.json 2> $O/bench_strong.err || { tail -20 $O/bench_strong.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 bench.py --inflight 1 --steps 20 --warmup 2 --no-cpu-baseline --no-pmc --no-config2 --no-legs > $O/prof1_bench.json 2> $O/prof1.err || { tail -20 $O/prof1.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof20 -o run -- python3 bench.py --steps 200 --no-cpu-baseline --no-pmc --no-config2 --no-legs > $O/prof20_bench.json 2> $O/prof20.err || { tail -20 $O/prof20.err; exit 1; }
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/nat0 -o run -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 0 3 > $GRAFT_REPO_ROOT/$O/nat0.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/nat1 -o run -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 1 2 > $GRAFT_REPO_ROOT/$O/nat1.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/noix -o run -- python3 $GRAFT_REPO_ROOT/tools/scripts/noix_bench.py synth 8192 3 > $GRAFT_REPO_ROOT/$O/noix.txt 2>&1 || exit 1
find $GRAFT_REPO_ROOT/$O -name "*stats*"
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/scripts/natural_prof.py 8192 3 1 > $O/nat3.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/scripts/natural_prof.py 8192 4 1 > $O/nat4.txt 2>&1 || exit 1
cat $O/nat3.txt $O/nat4.txt
cd /tmp
for sp in 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/nat$sp -o run -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 $sp 2 > $GRAFT_REPO_ROOT/$O/nat${sp}p.txt 2>&1 || exit 1
done
# HBM counters of the -s>=1 LZ / search kernels (one pass per TCC group; FETCH_SIZE is half the
# bytes of wide reads on gfx950, MI355X_MICROARCH.md)
for sp in 1 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_s${sp}_$c -o p -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 $sp 1 > $GRAFT_REPO_ROOT/$O/pmc_s${sp}_$c.log 2>&1 || exit 1
  done
done
cd $GRAFT_REPO_ROOT
python3 tools/scripts/pmc_summary2.py $O/pmc_s1_* > $O/pmc_s1_summary.txt
python3 tools/scripts/pmc_summary2.py $O/pmc_s4_* > $O/pmc_s4_summary.txt
bash tools/scripts/round_check.sh r04 inflight noix
