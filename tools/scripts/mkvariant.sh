#!/bin/bash
# Measurement library var/NAME.so: EVERY source recompiled with FLAGS into build/NAME/ (never a
# mix with objects of another build: the kernels share structs, e.g. EncodeJob, whose layout must
# agree across all objects).  Usage: tools/scripts/mkvariant.sh NAME "FLAGS"
#   e.g. mkvariant.sh dbg "-DHOH_DEBUG_READ"   (hoh_debug_read + per-tile kernel counters)
#        mkvariant.sh knobs "-DHOH_KNOBS"      (environment knobs; = tools/scripts/mkknobs.sh)
set -e
cd "$(dirname "$0")/../.."
name=$1; flags=$2
[ -n "$name" ] || { echo "usage: $0 NAME FLAGS"; exit 1; }
rm -rf build/$name; mkdir -p var build/$name
objs=""
for src in hoh-ans_amd/csrc/*.hip hoh-ans_amd/csrc/*.cpp; do
  o=build/$name/$(basename $src).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -I hoh-ans_amd/csrc $flags \
    -c -o $o $src &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/$name.so $objs -ldl -lpthread
echo var/$name.so
