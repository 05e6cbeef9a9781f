set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/g2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "search or natural or plane_s or lz or sizes" > $O/gputests.log 2>&1 || { tail -30 $O/gputests.log; exit 1; }
tail -2 $O/gputests.log
bash tools/scripts/ab_nat1.sh var/old.so base var/loose.so var/nov.so || exit 1
bash tools/scripts/ab_nat.sh base || exit 1
