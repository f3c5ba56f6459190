#!/bin/bash
# RG (R-MAT 2^16 A^2): the library at the r04ab5 record (b4302bb3, 4.39 ms there), right after the
# pattern-B fat walk (bf4ca692), the tree, and the tree without the pattern-B shortcut (nouni)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r04ab19}; mkdir -p $OUT
timeout -k 10 700 python tools/ab_heavy.py --reps 2 --legs rg,c5any b4302bb3 bf4ca692 tree nouni > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A6 summary $OUT/ab.txt
