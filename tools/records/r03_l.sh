#!/bin/bash
# Round-3 call l: per-block max row counts in symbolic (reduced by the scan's last tile), symbolic's
# max(A row) of long rows for numeric (SLAT_NO_SYM_AMAX=1: numeric loads them), the symbolic grid;
# GPU tests first, host split last
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03l; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --c4 --sat64 tree tree:SLAT_NO_SYM_AMAX=1 tree:SLAT_SYM_BPC=8 tree:SLAT_SYM_BPC=12 > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A6 summary $OUT/ab.txt
SLAT_HOST_CLOCK=1 timeout -k 10 300 python tools/host_overhead.py > $OUT/host.txt 2>&1 || { tail -30 $OUT/host.txt; exit 1; }
tail -4 $OUT/host.txt
echo done
