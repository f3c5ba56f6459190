#!/bin/bash
# wide launches' short-row tile rows: by row count (the tree's rule) against 64 always, on the heavy
# legs (R-MAT 2^16 / 2^18 rows) and C4's eighth
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab17}; mkdir -p $OUT
timeout -k 10 700 python tools/ab_heavy.py --reps 2 --big --legs rg,c5any,chain,c5big_any knob knob:SLAT_TILE_ROWS=64 knob:SLAT_TILE_ROWS=32 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A5 summary $OUT/ab.txt
