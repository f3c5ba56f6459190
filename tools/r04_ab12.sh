#!/bin/bash
# C4's short-row tiles: 64 rows (default) against 48 / 32 / 16 (SLAT_TILE_ROWS, now also for wide launches)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab12}; mkdir -p $OUT
timeout -k 10 500 python tools/ab.py --reps 2 --steps 100 --c4 k16 k16:SLAT_TILE_ROWS=48 k16:SLAT_TILE_ROWS=32 k16:SLAT_TILE_ROWS=16 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A5 summary $OUT/ab.txt | cut -c1-300
