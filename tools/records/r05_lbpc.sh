#!/bin/bash
# A/B: blocks per CU of the wide launches' listed-row launches (SLAT_LIST_BPC), C4 whole / eighth and R-MAT 2^16
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05_lbpc; mkdir -p $OUT
timeout -k 10 600 python3 -u tools/ab_env.py --lib tools/var/libslat_lbpc.so --reps 2 - SLAT_LIST_BPC=1 SLAT_LIST_BPC=2 > $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
cut -c1-300 $OUT/ab.txt
