set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/scripts/r6_abknob.sh "1 2 3 4" "HOH_LZFP_FIRST=0" "HOH_LZFP_FIRST=4" > gpurun_out/r6k_lzfp.txt 2>&1 || { tail gpurun_out/r6k_lzfp.txt; exit 1; }
cat gpurun_out/r6k_lzfp.txt
bash tools/scripts/r5_tl.sh r6tl "1 4" > gpurun_out/r6tl.txt 2>&1 || { tail gpurun_out/r6tl.txt; exit 1; }
cat gpurun_out/r6tl.txt
