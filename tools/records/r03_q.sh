#!/bin/bash
# Round-3 call q: C4 short-row paths — triangular probing in the LDS hash tables (variant qp), the
# payload-free packed emit sort (variant pack), both (qppack): their wide-launch tests, then A/B on
# C4; the small cells with the C-ABI clock
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03q; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_qppack.so timeout -k 10 300 python -u -m pytest tests/test_wide_hash_gpu.py tests/test_short_sort_gpu.py tests/test_spgemm_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_qppack.log 2>&1 || { tail -40 $OUT/tests_qppack.log; exit 1; }
tail -n 2 $OUT/tests_qppack.log
timeout -k 10 900 python tools/ab.py --reps 3 --c4 tree qp pack qppack > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
grep -A5 summary $OUT/ab.txt
timeout -k 10 400 python tools/small_cells.py > $OUT/small_cells.csv 2>&1 || { tail -30 $OUT/small_cells.csv; exit 1; }
cat $OUT/small_cells.csv
echo done
