#!/bin/bash
# Round-3 call x: the fat-row threshold (SLAT_FAT_MIN: 4096 / 8192 products against 16384): rows
# between move from the window pass (hub rows accumulating into C with global atomics) to the
# workgroup-per-row dense accumulator; fat-row tests at 4096 first
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r03x; mkdir -p $OUT
SLAT_FAT_MIN=4096 timeout -k 10 400 python -u -m pytest tests/test_fat_rows_gpu.py tests/test_f64_any_order_gpu.py tests/test_real_graph_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -n 1 $OUT/tests.log
timeout -k 10 900 python tools/ab_heavy.py --reps 2 --big tree tree:SLAT_FAT_MIN=8192 tree:SLAT_FAT_MIN=4096 > $OUT/ab_heavy.txt 2>&1 || { tail -30 $OUT/ab_heavy.txt; exit 1; }
grep -A4 summary $OUT/ab_heavy.txt
echo done
