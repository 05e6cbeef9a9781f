cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for lib in knobs knobs4; do
 for sp in 1 4; do
  d=gpurun_out/seg_${lib}_$sp
  HOH_LZ_FORK=0 HOH_LIB=var/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o p -- python3 tools/scripts/natural_prof.py 8192 $sp 2 > $d.log 2>&1 || exit 1
  echo "== $lib -s$sp fork0"; grep "^natural" $d.log; python3 tools/scripts/timeline.py $d/*.db k_front256 0.3 | grep lzscan
  d=gpurun_out/seg_${lib}_${sp}f
  HOH_LIB=var/$lib.so timeout -k 10 120 rocprofv3 --kernel-trace -d $d -o p -- python3 tools/scripts/natural_prof.py 8192 $sp 2 > $d.log 2>&1 || exit 1
  echo "== $lib -s$sp forked"; grep "^natural" $d.log; python3 tools/scripts/timeline.py $d/*.db k_front256 0.3 | grep lzscan
 done
done
