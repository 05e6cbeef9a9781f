#!/bin/bash
# Measurement (GPU box): k_nuke (256-pixel walk, var/nukeold.so) against k_nuke_v (16-B walk, the
# product library), natural 8192^2 -s0/-s1/-s4 encodes alternated; then k_lzscan's per-tile
# counters through the checking build (HOH_DEBUG_READ).  Usage: r6_nukeab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/scripts/r5_ab_lzsort.sh "0 1 4" var/nukeold.so:0 hoh-ans_amd/lib/libhohgpu.so:0 || exit 1
HOH_LIB=hoh-ans_amd/lib/libhohgpu_check.so timeout -k 10 200 python3 tools/scripts/lzscan_stats.py 1 4 || exit 1
