set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/g14; mkdir -p $O; export TMPDIR=/tmp
HOH_LIB=$GRAFT_REPO_ROOT/var/vmap.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "natural or sizes or search or plane_s" > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
bash tools/scripts/ab_nat1.sh var/vmap.so base || exit 1
SPEEDS="2 3 4" bash tools/scripts/ab_nat34.sh var/vmap.so base || exit 1
