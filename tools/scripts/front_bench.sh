set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tools/scripts/front_check.sh || exit 1
tools/scripts/bench_ab.sh 0
