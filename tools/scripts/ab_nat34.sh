#!/bin/bash
# A/B of variant libraries (HOH_LIB) on the natural 8192^2 image at -s3 and -s4: kernel stats
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab34; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  n=$(basename $v .so)
  cd /tmp
  if [ "$v" = base ]; then unset HOH_LIB; else export HOH_LIB=$GRAFT_REPO_ROOT/$v; fi
  for sp in ${SPEEDS:-3 4}; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/$n$sp -o run -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 $sp 1 > $GRAFT_REPO_ROOT/$O/$n$sp.txt 2>&1 || exit 1
    grep "^natural" $GRAFT_REPO_ROOT/$O/$n$sp.txt
    head -7 $GRAFT_REPO_ROOT/$O/$n$sp/run_kernel_stats.csv | cut -d, -f1-4
  done
  cd $GRAFT_REPO_ROOT
done
