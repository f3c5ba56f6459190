#!/bin/bash
# Short-row category changes: wide-launch parity tests, C4 phase split (diagnostic build), C4 kernel trace
set -o pipefail
OUT=gpurun_out/r02_short
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_short_sort_gpu.py \
  tests/test_wide_hash_gpu.py tests/test_f64_any_order_gpu.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -n 2 $OUT/pytest.log
SLAT_LIB_PATH=tools/bin/libslat_phases.so timeout -k 10 100 python tools/prof_c4.py > $OUT/c4_phases.txt 2>&1 || { cat $OUT/c4_phases.txt; exit 1; }
tail -n 2 $OUT/c4_phases.txt
timeout -k 10 100 python tools/prof_c4.py > $OUT/c4.txt 2>&1 || { cat $OUT/c4.txt; exit 1; }
tail -n 2 $OUT/c4.txt
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o c4 -- python3 tools/prof_c4.py > $OUT/prof.log 2>&1 || { tail $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 $f | cut -c1-150 | head -8
