#!/bin/bash
# Round-4 closing check (outputs in gpurun_out/r04f/): every GPU test, repeatability of the -s2..-s4
# encodes (tools/scripts/rep_speed.py), natural 8192^2 encode times at -s1..-s4 and the
# driver-shaped bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r04f; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
REPS=25 timeout -k 10 600 python3 tools/scripts/rep_speed.py 2 3 4 > $O/rep.txt 2>&1 || { tail $O/rep.txt; exit 1; }
cat $O/rep.txt
for sp in 1 2 3 4; do
  timeout -k 10 300 python3 tools/scripts/natural_prof.py 8192 $sp 3 >> $O/natural.txt 2>&1 || { tail $O/natural.txt; exit 1; }
done
grep ^natural $O/natural.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench_driver_shape.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench_driver_shape.json
