#!/bin/bash
# C4 phase times (symbolic / numeric ms) across library variants and the short-row category switch
set -o pipefail
OUT=gpurun_out/r02_c4ab
mkdir -p $OUT
for v in "$@"; do
  name=${v%%:*}; mode=${v##*:}
  if [ $name = tree ]; then unset SLAT_LIB_PATH; else export SLAT_LIB_PATH=tools/bin/libslat_$name.so; fi
  if [ $mode = sort ]; then export SLAT_SORT_SHORT=1; else unset SLAT_SORT_SHORT; fi
  timeout -k 10 120 python tools/prof_c4.py > $OUT/$name-$mode.txt 2>&1 || { cat $OUT/$name-$mode.txt; exit 1; }
  echo "$v $(tail -n 1 $OUT/$name-$mode.txt)"
done
