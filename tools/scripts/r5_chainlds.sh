#!/bin/bash
# Round 5: chain LDS request (knob CHAIN_LDS_KB) in the batched pipeline (var/knobs.so), GPU box.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for kb in ${KBS:-9 16 28 40 56 80}; do
  echo -n "chain lds $kb KB: "; HOH_LIB=var/knobs.so HOH_CHAIN_LDS_KB=$kb timeout -k 10 120 python3 -u tools/scripts/batch_pipe.py ${DB:-4 8} 24 enc,both | tr '\n' ' '; echo
done
