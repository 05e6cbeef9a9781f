# round 3: kernel traces of natural 8192^2 encodes at -s1 and -s4
set -o pipefail
cd /tmp; export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s1b -o p -- python3 $R/tools/scripts/natural_prof.py 8192 1 2 > $R/gpurun_out/prof_s1b.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s4 -o p -- python3 $R/tools/scripts/natural_prof.py 8192 4 1 > $R/gpurun_out/prof_s4.txt 2>&1 || exit 1
grep natural $R/gpurun_out/prof_s1b.txt $R/gpurun_out/prof_s4.txt
