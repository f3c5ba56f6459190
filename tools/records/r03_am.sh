#!/bin/bash
# Round-3 call am: fat-row numeric with 32 KB accumulator chunks and four blocks per CU (fr32) against
# 64 KB / two blocks (tree) for the atomic semirings: fat-row tests, heavy products
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03am; mkdir -p $OUT
SLAT_LIB_PATH=tools/var/libslat_fr32.so timeout -k 10 400 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_real_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests_fr32.log 2>&1 || { tail -40 $OUT/tests_fr32.log; exit 1; }
tail -n 1 $OUT/tests_fr32.log
timeout -k 10 900 python tools/ab_heavy.py --reps 2 --big tree fr32 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A3 summary $OUT/ab_heavy.txt
echo done
