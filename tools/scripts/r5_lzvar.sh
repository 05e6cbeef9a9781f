#!/bin/bash
# Measurement (GPU box): the natural -s0 pipeline (nat0_pipe.py) and one image (natural_prof.py)
# with k_lz build variants var/lz_*.so against the product library.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for lib in hoh-ans_amd/lib/libhohgpu.so var/lz_*.so; do
  echo "== $lib"
  HOH_LIB=$lib timeout -k 10 200 python3 tools/scripts/nat0_pipe.py 4 8 4 2>/dev/null | grep natural || exit 1
  HOH_LIB=$lib timeout -k 10 200 python3 tools/scripts/natural_prof.py 8192 0 3 2>/dev/null | grep natural || exit 1
done
