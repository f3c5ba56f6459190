#!/bin/bash
# Round-3 call aj: fat-row numeric with 64 KB accumulator chunks, two blocks per CU (variant fr64)
# against 128 KB / one block: fat-row tests, then the heavy products
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03aj; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_fr64.so timeout -k 10 400 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_real_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_fr64.log 2>&1 || { tail -40 $OUT/tests_fr64.log; exit 1; }
tail -n 1 $OUT/tests_fr64.log
timeout -k 10 900 python tools/ab_heavy.py --reps 2 --big tree fr64 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
echo done
