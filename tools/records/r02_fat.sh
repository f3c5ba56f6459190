#!/bin/bash
# fat-row category: its parity tests, the whole GPU suite, then the heavy products' timings
set -o pipefail
OUT=gpurun_out/${1:-fat}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fat_rows_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/fat.log 2>&1 || { tail -40 $OUT/fat.log; exit 1; }
tail -2 $OUT/fat.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/all.log 2>&1 || { tail -40 $OUT/all.log; exit 1; }
tail -2 $OUT/all.log
timeout -k 10 300 python -u tools/prof_heavy.py > $OUT/heavy.txt 2>&1 || { tail -20 $OUT/heavy.txt; exit 1; }
cat $OUT/heavy.txt
