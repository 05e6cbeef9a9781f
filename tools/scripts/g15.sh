set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/g15; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
bash tools/scripts/ab_nat1.sh var/head.so base || exit 1
SPEEDS="2 3 4" bash tools/scripts/ab_nat34.sh var/head.so base || exit 1
