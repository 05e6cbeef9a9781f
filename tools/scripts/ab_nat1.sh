#!/bin/bash
# A/B of variant libraries (HOH_LIB) on the natural 8192^2 image at -s1: kernel stats
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ab1; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  n=$(basename $v .so)
  cd /tmp
  if [ "$v" = base ]; then unset HOH_LIB; else export HOH_LIB=$GRAFT_REPO_ROOT/$v; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/$n -o run -- python3 $GRAFT_REPO_ROOT/tools/scripts/natural_prof.py 8192 1 2 > $GRAFT_REPO_ROOT/$O/$n.txt 2>&1 || exit 1
  grep "^natural" $GRAFT_REPO_ROOT/$O/$n.txt
  head -6 $GRAFT_REPO_ROOT/$O/$n/run_kernel_stats.csv | cut -d, -f1-4
  cd $GRAFT_REPO_ROOT
done
