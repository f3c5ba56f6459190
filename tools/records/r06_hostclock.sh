#!/bin/bash
# host split of the headline call (knobs build, SLAT_HOST_CLOCK): returning after the scan vs not
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06hc}; mkdir -p $OUT
for v in early noearly early noearly; do
  if [ $v = early ]; then E=""; else E="SLAT_NO_EARLY=1"; fi
  env SLAT_LIB_PATH=tools/var/libslat_knobs.so SLAT_HOST_CLOCK=1 $E timeout -k 10 120 python3 tools/prof_head.py 600 > $OUT/$v.txt 2>&1 || { tail $OUT/$v.txt; exit 1; }
  echo "== $v"; tail -3 $OUT/$v.txt
done
