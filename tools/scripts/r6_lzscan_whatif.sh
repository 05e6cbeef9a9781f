#!/bin/bash
# Round 6 what-if: k_lzscan without its vertical search (EXP=16, checking build, output invalid)
# against the shipped search (EXP=0): the -s4 kernel timeline of one natural 8192^2 encode and the
# pipelined -s4 rate (speed_pipe.py, D = 4).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for e in 0 16; do
  echo "EXP=$e"
  d=gpurun_out/r6lzw_$e
  HOH_LIB=hoh-ans_amd/lib/libhohgpu_check.so HOH_EXP=$e HOH_QUIET=1 timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o p -- python3 tools/scripts/natural_prof.py 8192 4 3 > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
  grep '^natural' $d.log
  python3 tools/scripts/timeline.py $(ls $d/*.db | head -1) k_colours 1.0
  HOH_LIB=hoh-ans_amd/lib/libhohgpu_check.so HOH_EXP=$e HOH_QUIET=1 timeout -k 10 120 python3 tools/scripts/speed_pipe.py 4 4 6 2>&1 | grep -v amdgpu.ids
done
