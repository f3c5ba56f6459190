#!/bin/bash
# k_symbolic_short blocks per CU (knobs build, SLAT_SHORT_BPC; 16 in the tree): C4 whole / eighth and
# the R-MAT 2^16 A^2 leg (tools/ab_env.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r06c4sweep2}; mkdir -p $OUT
timeout -k 10 800 python3 tools/ab_env.py --lib tools/var/libslat_knobs.so --reps 2 - SLAT_SHORT_BPC=8 SLAT_SHORT_BPC=10 SLAT_SHORT_BPC=12 > $OUT/sweep.txt 2>&1 || { tail $OUT/sweep.txt; exit 1; }
cat $OUT/sweep.txt
