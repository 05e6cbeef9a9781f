#!/bin/bash
# Measurement builds: libhohgpu.so with some sources compiled with extra -D flags, the rest from
# build/*.o (run make first).  Usage: tools/scripts/variant.sh OUT.so "-DX=1 -DY=2" src.hip...
set -e
cd "$(dirname "$0")/../.."
OUT=$1; DEFS=$2; shift 2
tmp=$(mktemp -d)
objs=""
for o in build/*.o; do
  b=$(basename $o .o)
  skip=0
  for s in "$@"; do [ "$(basename $s)" = "$b" ] && skip=1; done
  [ $skip = 0 ] && objs="$objs $o"
done
for s in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result $DEFS -c -o $tmp/$(basename $s).o $s
  objs="$objs $tmp/$(basename $s).o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT $objs -ldl -lpthread
rm -rf $tmp
