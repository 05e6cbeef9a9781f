set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/scripts/r5_ab_lzsort.sh "1 2 4" var/knobs.so:0 var/lz512.so:512 var/lz512.so:256 || exit 1
