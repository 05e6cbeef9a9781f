#!/bin/bash
# Measurement (GPU box): the decoder's chain-tile threshold (knob LZ_XROW: copies reading the row
# above that make an LZ tile a raster-chain tile) on the natural 8192^2 -s0 image: one image
# encode + decode, and the natural -s0 pipeline, through var/knobs.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for x in ${XROWS:-16 4 64 1000000}; do
    echo -n "rep $rep LZ_XROW=$x single: "; HOH_LIB=var/knobs.so HOH_LZ_XROW=$x timeout -k 10 100 python3 tools/scripts/natural_prof.py 8192 0 5 | sed 's/.*encode/encode/' || exit 1
    echo -n "rep $rep LZ_XROW=$x pipeline: "; HOH_LIB=var/knobs.so HOH_LZ_XROW=$x timeout -k 10 150 python3 tools/scripts/nat0_pipe.py 4 8 6 || exit 1
  done
done
