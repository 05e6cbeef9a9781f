#!/bin/bash
# Variant library for A/B runs: var/NAME.so = libhohgpu.so's objects with SRC (a .hip file, default
# the in-tree one of the same name) recompiled with extra FLAGS.  Usage: mkvar.sh NAME SRC.hip "FLAGS"
set -e
cd "$(dirname "$0")/../.."
# the other objects come from build/ (the product build): bring them up to date first, so every
# object of the variant was compiled against the same headers (struct layouts must agree)
make -s -j8 >/dev/null
name=$1; src=$2; flags=$3
mkdir -p var build/var
b=$(basename $src .hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -I hoh-ans_amd/csrc $flags -c -o build/var/$name.$b.o $src
objs=$(ls build/*.o | grep -v "/$b.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/$name.so $objs build/var/$name.$b.o -ldl -lpthread
echo var/$name.so
