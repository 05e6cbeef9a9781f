#!/bin/bash
# Round 5: encode-only batched pipeline with stage stops (var/knobs.so, HOH_ENC_STOP), GPU box.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for st in 0 1 2 3 4 5 6 7; do
  echo -n "stop $st: "; HOH_LIB=var/knobs.so HOH_ENC_STOP=$st timeout -k 10 120 python3 -u tools/scripts/batch_pipe.py 4 8 24 enc | head -1
done
