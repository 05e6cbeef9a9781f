#!/bin/bash
# The round-4 -s2..-s4 nondeterminism, reproduced on purpose.
# Builds (here, on the CPU) two debug libraries whose k_lzsort makes its last wave sleep ~13 us
# before clearing the per-wave digit counts of a chunk:
#   var/race_old.so  the round-4 k_lzsort (git 88ccbb2): every thread clears cnt[*][tid] after a
#                    barrier, so a faster wave's next-chunk count store can be wiped
#   var/race_new.so  the fixed round-5 k_lzsort (git 3af4c21): each wave clears only its own row
# (the current k_lzsort ranks each wave's quarter alone: no count row is shared between waves)
# and, with `run` (on the GPU box), checks the posting lists of -s2 encodes against an exact
# recomputation (tools/scripts/lzsort_check.py).  Expected: wrong lists with race_old, none with
# race_new.
set -e
cd "$(dirname "$0")/../.."
if [ "$1" = run ]; then
  export TMPDIR=/tmp; mkdir -p gpurun_out
  HOH_LIB=var/race_old.so timeout -k 10 240 python -u tools/scripts/lzsort_check.py 2 3
  HOH_LIB=var/race_new.so timeout -k 10 240 python -u tools/scripts/lzsort_check.py 2 3
  exit 0
fi
mkdir -p var build/var
make -s -j8 >/dev/null            # build/*.o current: the variants link them (same struct layouts)
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -I hoh-ans_amd/csrc"
git show 88ccbb2:hoh-ans_amd/csrc/k_search.hip > build/var/k_search_r4.hip
# the same adversarial sleep, placed before the round-4 code's clear loop
python3 - <<'EOF'
p = "build/var/k_search_r4.hip"
s = open(p).read()
old = "      __syncthreads();\n      if (tid < 256)\n#pragma unroll\n        for (int w = 0; w < LZSORT_T / 64; w++) cnt[w][tid] = 0;"
assert s.count(old) == 1, "round-4 clear loop not found"
new = ("      __syncthreads();\n      if (wv == LZSORT_T / 64 - 1)\n        for (int z = 0; z < 4; z++) __builtin_amdgcn_s_sleep(127);\n"
       "      if (tid < 256)\n#pragma unroll\n        for (int w = 0; w < LZSORT_T / 64; w++) cnt[w][tid] = 0;")
open(p, "w").write(s.replace(old, new))
EOF
/opt/rocm/bin/hipcc $F -DHOH_DEBUG_READ -c -o build/var/dbg.hoh_api.o hoh-ans_amd/csrc/hoh_api.cpp
/opt/rocm/bin/hipcc $F -c -o build/var/race_old.k_search.o build/var/k_search_r4.hip
git show 3af4c21:hoh-ans_amd/csrc/k_search.hip > build/var/k_search_r5fix.hip
/opt/rocm/bin/hipcc $F -DLZSORT_DELAY_TEST -c -o build/var/race_new.k_search.o build/var/k_search_r5fix.hip
objs=$(ls build/*.o | grep -v -e /hoh_api.cpp.o -e /k_search.hip.o)
for v in old new; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/race_$v.so $objs build/var/dbg.hoh_api.o \
    build/var/race_$v.k_search.o -ldl -lpthread
done
ls -la var/race_old.so var/race_new.so
