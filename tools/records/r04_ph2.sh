#!/bin/bash
# phase split of the lane kernel on C1 (a -DSLAT_PHASES=1 build)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ph2}; mkdir -p $OUT
SLAT_LIB_PATH=$GRAFT_REPO_ROOT/tools/var/libslat_ph.so timeout -k 10 120 python tools/phases_chain.py 4 > $OUT/phases.txt 2>&1 || { tail -20 $OUT/phases.txt; exit 1; }
cat $OUT/phases.txt
