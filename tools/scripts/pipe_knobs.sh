set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for d in 0 4 7; do HOH_ENC_DBG=$d timeout -k 5 120 python tools/scripts/pipe.py enc 12 96 2>/dev/null | grep mode || exit 1; done
for d in 0 4; do HOH_ENC_DBG=$d timeout -k 5 120 python tools/scripts/pipe.py both 12 96 2>/dev/null | grep mode || exit 1; done
