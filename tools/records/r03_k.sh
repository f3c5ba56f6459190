#!/bin/bash
# Round-3 call k: (1) the max row count and long rows' max(A row) recorded by symbolic (the scan skips
# its atomicMax, numeric its A-value loads; SLAT_NO_SYM_AMAX=1: numeric loads them; sym8: symbolic
# capped at 8 waves/SIMD) and the symbolic grid; (2) B in CSR form bucketed by the window passes'
# column chunk (SLAT_NO_WIN_SPLIT=1: whole B rows with a column filter) on the power-law products.
# GPU tests first; the host split of a call last.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03k; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --c4 --sat64 tree tree:SLAT_NO_SYM_AMAX=1 sym8 tree:SLAT_SYM_BPC=8 tree:SLAT_SYM_BPC=24 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A6 summary $OUT/ab.txt
timeout -k 10 1000 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_NO_WIN_SPLIT=1 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
tail -4 $OUT/host.txt
echo done
