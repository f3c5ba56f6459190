#!/bin/bash
# Short-row categories: parity tests of the wide launches, then C4 sorted (SLAT_SORT_SHORT) vs hash.
set -o pipefail
OUT=gpurun_out/r02_sort
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_short_sort_gpu.py \
  tests/test_wide_hash_gpu.py tests/test_f64_any_order_gpu.py > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
fi
for v in sort hash; do
  if [ $v = sort ]; then export SLAT_SORT_SHORT=1; else unset SLAT_SORT_SHORT; fi
  timeout -k 10 120 python tools/prof_c4.py > $OUT/c4_$v.txt 2>&1 || { cat $OUT/c4_$v.txt; exit 1; }
  tail -n 2 $OUT/c4_$v.txt
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o c4 -- python3 tools/prof_c4.py > $OUT/prof_$v.log 2>&1 || { tail $OUT/prof_$v.log; exit 1; }
  f=$(find $OUT/prof_$v -name "*kernel_stats.csv" | head -1)
  cut -d, -f1-4 $f | head -12
done
