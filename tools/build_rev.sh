#!/bin/bash
# usage: tools/build_rev.sh REV NAME — builds the library as committed at git revision REV into
# tools/var/libslat_NAME.so (A/B of a change against the tree before it; load with SLAT_LIB_PATH)
set -e
root="$(cd "$(dirname "$0")/.." && pwd)"
src=/tmp/slat_rev_$2
rm -rf "$src" && mkdir -p "$src"
git -C "$root" archive "$1" sparse-linear-algebra-tests_amd include | tar -x -C "$src"
mkdir -p "$root/tools/var"
make -s -j8 -C "$src/sparse-linear-algebra-tests_amd" BUILD=/tmp/slat_rev_obj_$2 OUT="$root/tools/var/libslat_$2.so"
