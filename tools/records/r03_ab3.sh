#!/bin/bash
# Round-3 A/B 3: Sat64 rows in u32 slots under the bound (tree; nonarrow = before), k_numeric capped
# at 3 waves/SIMD (w3), early stored-bitmap loads (early); the fat-row split table (tree) against
# range-filtered walks (SLAT_NO_FAT_SPLIT=1) on the power-law products; parity tests first
set -o pipefail
OUT=gpurun_out/r03d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_spgemm_gpu.py tests/test_magnus_usize_gpu.py tests/test_graph_gpu.py tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_real_graph_gpu.py tests/test_dist_gpu.py tests/test_btree_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 2 $OUT/tests.log
timeout -k 10 900 python tools/ab.py --reps 2 --sat64 tree nonarrow w3 early > $OUT/ab.txt 2>&1 || { tail -30 $OUT/ab.txt; exit 1; }
cat $OUT/ab.txt
timeout -k 10 1200 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_NO_FAT_SPLIT=1 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
cat $OUT/ab_heavy.txt
