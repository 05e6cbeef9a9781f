#!/bin/bash
# Natural-statistic 8192^2 (configs[4]) timings and per-kernel stats: -s0 encode + decode, -s1 and
# -s2 encode (outputs in gpurun_out/nat*).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nat0 -o run -- python3 tools/scripts/natural_prof.py 8192 0 3 > gpurun_out/nat0.txt 2>&1 || { tail -20 gpurun_out/nat0.txt; exit 1; }
grep natural gpurun_out/nat0.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nat1 -o run -- python3 tools/scripts/natural_prof.py 8192 1 3 > gpurun_out/nat1.txt 2>&1 || { tail -20 gpurun_out/nat1.txt; exit 1; }
grep natural gpurun_out/nat1.txt
timeout -k 10 300 python3 tools/scripts/natural_prof.py 8192 2 2 > gpurun_out/nat2.txt 2>&1 || { tail -20 gpurun_out/nat2.txt; exit 1; }
grep natural gpurun_out/nat2.txt
find gpurun_out/nat0 gpurun_out/nat1 -name "*kernel_stats*"
