#!/bin/bash
# C1 (the lane kernel): phase split (variant build) and the per-call time of the tree
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r05lane2}; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_phases.so timeout -k 10 120 python3 tools/prof_c1.py > $OUT/phases.out 2> $OUT/phases.log || { tail $OUT/phases.log; exit 1; }
tail -2 $OUT/phases.log; cat $OUT/phases.out
timeout -k 10 120 python3 tools/prof_c1.py > $OUT/c1.out 2>&1 || { tail $OUT/c1.out; exit 1; }
cat $OUT/c1.out
