#!/bin/bash
# usage: tools/build_variant.sh NAME "-DFLAG=... ..." — builds tools/var/libslat_NAME.so: the whole
# library with the extra compiler flags, in its own object directory (kernel experiments; load it
# with SLAT_LIB_PATH=tools/var/libslat_NAME.so)
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$root/tools/var"
make -s -j8 -C "$root/sparse-linear-algebra-tests_amd" BUILD=/tmp/slat_var_$1 "EXTRA=-DSLAT_AB_KNOBS $2" OUT="$root/tools/var/libslat_$1.so"
