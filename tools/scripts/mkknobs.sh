#!/bin/bash
# Measurement library var/knobs.so: every source compiled with -DHOH_KNOBS, so the HOH_<name>
# environment variables of the HOH_KNOB sites (hoh_internal.h) take effect.  The product library
# (hoh-ans_amd/lib/libhohgpu.so) has none: its knobs are their compile-time defaults.
# Usage: tools/scripts/mkknobs.sh [EXTRA FLAGS]; then HOH_LIB=var/knobs.so HOH_LZ_FORK=0 ...
exec "$(dirname "$0")/mkvariant.sh" knobs "-DHOH_KNOBS $1"
