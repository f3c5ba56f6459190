#!/bin/bash
# Round-3 call ah: numeric's stored-bitmap rows compact their tail items through LDS (the bitmap
# region before the stored bitmap lands) instead of ds_permute rounds (variant tl): GPU suite, A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03ah; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_tl.so timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests_tl.log 2>&1 || { tail -40 $OUT/tests_tl.log; exit 1; }
tail -n 1 $OUT/tests_tl.log
timeout -k 10 900 python tools/ab.py --reps 5 --c4 --sat64 tree tl > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A3 summary $OUT/ab.txt
echo done
