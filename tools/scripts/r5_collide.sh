#!/bin/bash
# Correctness stress (GPU box, knobs build): the LZ posting hash narrowed to 8 / 12 bits, so that
# hash collisions (non-flat windows listed inside flat runs' spans, foreign groups mixed in) are
# the rule; the natural 8192^2 -s2..-s4 files must still be the reference's (golden SHAs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
declare -A want=([2]=f6b12a45ed90 [3]=ccbbd6279066 [4]=505520615dd7)
rc=0
for m in 255 4095; do
  for sp in 2 3 4; do
    line=$(HOH_LZS_HMASK=$m HOH_LIB=var/knobs.so timeout -k 10 200 python3 tools/scripts/natural_prof.py 8192 $sp 1 2>/dev/null | grep '^natural') || exit 1
    got=$(echo "$line" | sed -n 's/.*sha \([0-9a-f]*\).*/\1/p')
    ok=$([ "$got" = "${want[$sp]}" ] && echo OK || echo MISMATCH)
    [ $ok = OK ] || rc=1
    echo "mask $m -s$sp: $line  $ok"
  done
done
exit $rc
