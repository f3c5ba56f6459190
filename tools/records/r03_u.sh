#!/bin/bash
# Round-3 call u: RowWalker without group counts or tail compaction (variant g8: every entry's first
# two ELL groups loaded at once, B rows of more than 8 entries walk their further groups alone):
# the GPU suite on it, then A/B on the headline / C4 / Sat64
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03u; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_g8.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_g8.log 2>&1 || { tail -40 $OUT/tests_g8.log; exit 1; }
tail -n 1 $OUT/tests_g8.log
timeout -k 10 900 python tools/ab.py --reps 4 --c4 --sat64 tree g8 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
echo done
