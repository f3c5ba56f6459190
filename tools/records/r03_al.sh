#!/bin/bash
# Round-3 call al: k_fr_symbolic's bitmap sized by the column count (several blocks per CU on
# matrices narrower than 2^20 columns) against the 2^20-column bitmap (SLAT_FAT_SYM_FULL=1): the GPU
# suite, then the heavy products
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03al; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -n 1 $OUT/pytest.log
timeout -k 10 900 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_FAT_SYM_FULL=1 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
echo done
