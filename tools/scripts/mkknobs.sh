#!/bin/bash
# Measurement library var/knobs.so: every source compiled with -DHOH_KNOBS, so the HOH_<name>
# environment variables of the HOH_KNOB sites (hoh_internal.h) take effect.  The product library
# (hoh-ans_amd/lib/libhohgpu.so) has none: its knobs are their compile-time defaults.
# Usage: tools/scripts/mkknobs.sh [EXTRA FLAGS]; then HOH_LIB=var/knobs.so HOH_LZ_FORK=0 ...
set -e
cd "$(dirname "$0")/../.."
mkdir -p var build/knobs
objs=""
for src in hoh-ans_amd/csrc/*.hip hoh-ans_amd/csrc/*.cpp; do
  o=build/knobs/$(basename $src).o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-result -I hoh-ans_amd/csrc -DHOH_KNOBS $1 \
    -c -o $o $src &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o var/knobs.so $objs -ldl -lpthread
echo var/knobs.so
